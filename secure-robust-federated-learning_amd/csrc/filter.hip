// k6 — spectral filters: filterL2 and ex_noregret (and, after k5 bucketing,
// mom_filterL2 / mom_ex_noregret).
//
// Replaces src/robust_estimator.py:42-133 (ex_noregret_, ex_noregret) and
// :144-208 (filterL2_, filterL2).  Each layer is cut into itv-wide chunks
// (restarting at every layer, last chunk partial); each chunk is filtered
// independently.  One 256-thread workgroup per chunk (persistent over chunks).
//
// The reference builds the k x k (k <= itv = 1000) fp64 weighted covariance
// from N outer products and calls eigh for its top eigenpair, 2*int(eps*N)
// times per chunk.  Here everything after one pass over the chunk runs in
// client space (n x n, n <= 128):
//
//   Phase A  centred chunk Gram G = Z Z^T, Z = X_chunk - column mean, on the
//            fp64 MFMA (v_mfma_f64_16x16x4_f64), 36 upper 16x16 tiles over 4
//            waves; G then lives in registers (two lanes per row, 64 fp64 each).
//   Phase C  per iteration, with weights w = c / sum(c):
//              C = G - g 1^T - 1 g^T + s 1 1^T  (g = G w, s = w^T G w) is the
//              Gram of x_i - mu (mu the weighted mean), so the covariance's
//              nonzero spectrum is that of M = W^1/2 C W^1/2;
//              top eigenpair (lambda, u) of M by Lanczos with full
//              reorthogonalisation (fp64) + multisection bisection on the
//              tridiagonal + inverse iteration;
//              tau_j = ((x_j - mu).v)^2 = (C W^1/2 u)_j^2 / lambda;
//              early exit if lambda^2 <= expansion * sigma^2;
//              filterL2: c *= 1 - tau/tau_max, drop argmax, c /= |c|_1;
//              ex_noregret: c *= 1 - step*tau, KL projection onto the capped
//              simplex (every candidate evaluated in parallel, numpy's
//              pairwise fp64 sums emulated for the feasibility tests and KL).
//            ex_noregret first drops the ceil(eps*n) clients with the largest
//            Krum scores (fp32 distances from G, numpy pairwise score sums)
//            and sets step = 0.5 / max pairwise distance^2 in fp32.
//   Phase D  mu_j = sum_i c_i x_ij / sum_i c_i in fp64 over the kept clients
//            in client order (the reference's np.average), second pass over
//            the chunk (L2-resident).
#include "sra_common.hpp"

namespace sra {

constexpr int FNP = 128;           // padded client count
constexpr int FST = 64;            // coordinates per Gram stage
constexpr int FROW = FST + 4;      // stage row stride (floats)
constexpr int LMAX = 62;           // Lanczos steps per restart (V fills the 64 KB union)
constexpr int VST = FNP + 4;       // Lanczos basis row stride (doubles): spreads rows over LDS banks
constexpr int LRESTART = 6;        // explicit restarts from the Ritz vector

struct FilterShared {
  // union region: stage buffer (Phase A) / G transfer half (Phase B) /
  // Lanczos basis V[k][i] (Phase C) / Krum distance rows (ex_noregret)
  static constexpr int kUnionBytes = 65536;
  static constexpr int kVec = FNP;  // doubles per vector
};

struct FilterArgs {
  const float* X;
  int n;
  int64_t d;
  int64_t ldx;
  int itv;
  int nchunks;
  double eps;
  double sigma;
  double expansion;
  double* out;
  int* status;
  double* dbg;   // optional diagnostics of chunk 0 (see sra_filter_debug_f32)
};

// diagnostics layout (doubles): [0, FNP*FNP) chunk-0 Gram; then per outer
// iteration it a record of FNP+4: c[0..FNP) before the update, lam, Lanczos
// steps, Ritz residual, restarts used, then 12 solver scalars (scal[4..15]).
constexpr int kDbgRec = 128 + 16;

// ----- wave / block helpers (256 threads) --------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), l);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
// v with lane l replaced by x (l uniform)
__device__ __forceinline__ double writelane_f64(double x, int l, double v) {
  return static_cast<int>(threadIdx.x & 63) == l ? x : v;
}
// sum over the wave, identical in every lane (DPP within rows, readlane across)
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);   // row_half_mirror
  v += dpp_f64<0x140>(v);   // row_mirror
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  v = fmax(v, dpp_f64<0x140>(v));
  return fmax(fmax(readlane_f64(v, 0), readlane_f64(v, 16)), fmax(readlane_f64(v, 32), readlane_f64(v, 48)));
}
__device__ __forceinline__ double wave_min(double v) { return -wave_max(-v); }
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  const double r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// numpy pairwise fp32 sum of f(0..n) (n <= 255 via one or two splits)
template <typename F>
__device__ float np_pw32(int n, F&& f) {
  auto block = [&](int lo, int m) -> float {
    if (m < 8) {
      float r = 0.f;
      for (int i = 0; i < m; ++i) r += f(lo + i);
      return r;
    }
    float r0 = f(lo), r1 = f(lo + 1), r2 = f(lo + 2), r3 = f(lo + 3), r4 = f(lo + 4), r5 = f(lo + 5),
          r6 = f(lo + 6), r7 = f(lo + 7);
    int i = 8;
    for (; i < m - (m % 8); i += 8) {
      r0 += f(lo + i); r1 += f(lo + i + 1); r2 += f(lo + i + 2); r3 += f(lo + i + 3);
      r4 += f(lo + i + 4); r5 += f(lo + i + 5); r6 += f(lo + i + 6); r7 += f(lo + i + 7);
    }
    float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < m; ++i) res += f(lo + i);
    return res;
  };
  if (n <= 128) return block(0, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return block(0, n2) + block(n2, n - n2);
}

// 36 upper-triangle 16x16 tiles (I <= J) of the 128 x 128 chunk Gram
__constant__ int kFTileI[36] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2,
                                2, 2, 2, 3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 6, 6, 7};
__constant__ int kFTileJ[36] = {0, 1, 2, 3, 4, 5, 6, 7, 1, 2, 3, 4, 5, 6, 7, 2, 3, 4,
                                5, 6, 7, 3, 4, 5, 6, 7, 4, 5, 6, 7, 5, 6, 7, 6, 7, 7};
constexpr int ftile_i(int t) {
  int c = 0;
  for (int i = 0; i < 8; ++i)
    for (int j = i; j < 8; ++j) {
      if (c == t) return i;
      ++c;
    }
  return 0;
}
constexpr int ftile_j(int t) {
  int c = 0;
  for (int i = 0; i < 8; ++i)
    for (int j = i; j < 8; ++j) {
      if (c == t) return j;
      ++c;
    }
  return 0;
}

// Phase A for wave W: its 9 tiles (W + 4t) accumulate G over the chunk in
// 64-coordinate stages staged through LDS and centred by the stage's column
// means (fp64); tile -> row block mapping is compile-time.
template <int W>
__device__ __forceinline__ void filter_gram_phase(const FilterArgs& A, int64_t k0, int k, char* uni,
                                                  f64x4 (&acc)[9]) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int n = A.n;
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  float* stage = reinterpret_cast<float*>(uni);
  double* smean = reinterpret_cast<double*>(uni + FNP * FROW * 4);
  for (int s0 = 0; s0 < k; s0 += FST) {
    for (int e = tid; e < FNP * FST; e += 256) {
      const int r = e / FST, cc = e - (e / FST) * FST;
      float v = 0.f;
      if (r < n && s0 + cc < k) v = A.X[static_cast<int64_t>(r) * A.ldx + k0 + s0 + cc];
      stage[r * FROW + cc] = v;
    }
    __syncthreads();
    if (tid < FST) {
      double sm = 0.0;
      for (int r = 0; r < n; ++r) sm += static_cast<double>(stage[r * FROW + tid]);
      smean[tid] = sm / n;
    }
    __syncthreads();
#pragma unroll 2
    for (int ks = 0; ks < FST / 4; ++ks) {
      const int cc = 4 * ks + (lane >> 4);
      const double mu = smean[cc];
      double fr[8];
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int r = 16 * b + (lane & 15);
        fr[b] = r < n ? static_cast<double>(stage[r * FROW + cc]) - mu : 0.0;
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[ftile_i(W + 4 * t)], fr[ftile_j(W + 4 * t)], acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
}

// ----- block reductions (256 threads = 4 waves) -------------------------------
__device__ __forceinline__ void block_sum2(double& a, double& b, double* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[wave] = a;
    red[4 + wave] = b;
  }
  __syncthreads();
  a = (red[0] + red[1]) + (red[2] + red[3]);
  b = (red[4] + red[5]) + (red[6] + red[7]);
  __syncthreads();
}

// index of the largest v (first index on ties); inactive lanes pass -inf.
// Returns the index; *vbest receives its value.
__device__ __forceinline__ int block_argmax_first(double v, int i, double* red, int* ired, double* vbest) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ov = __shfl_xor(v, off);
    const int oi = __shfl_xor(i, off);
    if (ov > v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[wave] = v;
    ired[wave] = i;
  }
  __syncthreads();
  double bv = red[0];
  int bi = ired[0];
  for (int q = 1; q < 4; ++q)
    if (red[q] > bv || (red[q] == bv && ired[q] < bi)) {
      bv = red[q];
      bi = ired[q];
    }
  __syncthreads();
  *vbest = bv;
  return bi;
}

__device__ __forceinline__ int block_min_int(int v, int* ired) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int o = __shfl_xor(v, off);
    v = o < v ? o : v;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) ired[4 + wave] = v;
  __syncthreads();
  int r = ired[4];
  for (int q = 5; q < 8; ++q) r = ired[q] < r ? ired[q] : r;
  __syncthreads();
  return r;
}

// a / b from the hardware reciprocal with one Newton step and one residual
// correction (within an ulp or two; the twisted factorisation's pivots only)
__device__ __forceinline__ double fdiv(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = fma(fma(-b, r, 1.0), r, r);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}

template <int MODE>  // 0: filterL2, 1: ex_noregret
__global__ void __launch_bounds__(256, 2) spectral_filter_kernel(FilterArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* uni = smem;                                     // 64 KB union
  double* vec = reinterpret_cast<double*>(smem + FilterShared::kUnionBytes);
  double* c = vec;                 // weights (active clients)
  double* w = vec + 1 * FNP;       // normalised weights
  double* sw = vec + 2 * FNP;      // sqrt(w)
  double* gw = vec + 3 * FNP;      // G w
  double* xv = vec + 4 * FNP;      // operator input (sw o vector)
  double* yv = vec + 5 * FNP;      // G xv
  double* rv = vec + 6 * FNP;      // Lanczos residual / scratch
  double* uv = vec + 7 * FNP;      // Ritz vector (warm start)
  double* tau = vec + 8 * FNP;     // outlier scores / Krum scores
  double* sv = yv;                 // ex_noregret projection: weights in descending order
  double* hl = xv;                 // ex_noregret projection: sv * log(sv / cap)
  double* alpha = vec + 9 * FNP;   // [LMAX]
  double* beta = alpha + LMAX;     // [LMAX]
  double* beta2 = beta + LMAX;     // [LMAX] beta^2 (Sturm)
  double* svec = beta2 + LMAX;     // [LMAX] eigenvector of T
  double* hq = svec + LMAX;        // [LMAX] re-orthogonalisation coefficients
  double* tcp = hq + LMAX;         // [LMAX] tridiagonal solve scratch
  double* red = tcp + LMAX;        // [16]
  double* scal = red + 16;         // [16] broadcast scalars
  int* active = reinterpret_cast<int*>(scal + 16);  // [FNP]
  int* kidx = active + FNP;                         // [FNP] compact -> client
  int* irank = kidx + FNP;                          // [FNP] descending rank of compact entry
  int* iscal = irank + FNP;                         // [16]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int n = A.n;
  const int grow = tid >> 1;   // G row owned by this thread
  const int ghalf = tid & 1;   // which 64 columns
  const bool own = tid < FNP;  // thread owns client tid

  for (int chunk = blockIdx.x; chunk < A.nchunks; chunk += gridDim.x) {
    const int64_t k0 = static_cast<int64_t>(chunk) * A.itv;
    const int k = static_cast<int>((k0 + A.itv < A.d ? k0 + A.itv : A.d) - k0);

    // ================= Phase A: centred chunk Gram (fp64 MFMA) ==============
    f64x4 acc[9];
    if (wave == 0) filter_gram_phase<0>(A, k0, k, uni, acc);
    else if (wave == 1) filter_gram_phase<1>(A, k0, k, uni, acc);
    else if (wave == 2) filter_gram_phase<2>(A, k0, k, uni, acc);
    else filter_gram_phase<3>(A, k0, k, uni, acc);

    // ================= Phase B: G tiles -> registers (row layout) ===========
    double g[64];
    double* gbuf = reinterpret_cast<double*>(uni);  // [64 rows][128]
#pragma unroll 1
    for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int tile = wave + 4 * t;
        const int I = kFTileI[tile], J = kFTileJ[tile];
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          const int row = 16 * I + (lane >> 4) + 4 * rg;
          const int col = 16 * J + (lane & 15);
          const double v = acc[t][rg];
          if ((row >> 6) == hh) gbuf[(row & 63) * FNP + col] = v;
          if ((col >> 6) == hh) gbuf[(col & 63) * FNP + row] = v;
        }
      }
      __syncthreads();
      if ((grow >> 6) == hh) {
#pragma unroll
        for (int j = 0; j < 64; ++j) g[j] = gbuf[(grow & 63) * FNP + 64 * ghalf + j];
      }
      __syncthreads();
    }
    const bool dbg = A.dbg != nullptr && chunk == 0;
    if (dbg) {
#pragma unroll
      for (int j = 0; j < 64; ++j) A.dbg[grow * FNP + 64 * ghalf + j] = g[j];
    }

    // y = G x for x in LDS; every thread of the row pair gets the row value
    auto gmv_row = [&](const double* x) -> double {
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
      const double* xh = x + 64 * ghalf;
#pragma unroll
      for (int j = 0; j < 64; j += 4) {
        p0 += g[j] * xh[j];
        p1 += g[j + 1] * xh[j + 1];
        p2 += g[j + 2] * xh[j + 2];
        p3 += g[j + 3] * xh[j + 3];
      }
      const double p = (p0 + p1) + (p2 + p3);
      return p + dpp_f64<0xB1>(p);   // the row's other half lives in lane ^ 1
    };
    // (C xv)[tid] for the owning threads, C = G - g1' - 1g' + s11' with
    // g = gw, s = scal[0]; xv must be visible.  Two barriers.
    auto cmul = [&]() -> double {
      const double p = gmv_row(xv);
      double a1 = own ? xv[tid] : 0.0;
      double a2 = own ? gw[tid] * xv[tid] : 0.0;
      a1 = wave_sum(a1);
      a2 = wave_sum(a2);
      if (lane == 0) {
        red[wave] = a1;
        red[4 + wave] = a2;
      }
      if (ghalf == 0) yv[grow] = p;
      __syncthreads();
      const double s1 = (red[0] + red[1]) + (red[2] + red[3]);
      const double gy = (red[4] + red[5]) + (red[6] + red[7]);
      const double r = own ? yv[tid] - gw[tid] * s1 - gy + scal[0] * s1 : 0.0;
      __syncthreads();
      return r;
    };

    // ============ ex_noregret: Krum pre-filter on the chunk =================
    int n_keep = n;
    double step = 0.0;
    if constexpr (MODE == 1) {
      const int fp = static_cast<int>(ceil(A.eps * n));
      float* drow = reinterpret_cast<float*>(uni);   // [FNP][FNP] fp32 distances
      {
        double dg = 0.0;
#pragma unroll
        for (int j = 0; j < 64; ++j)
          if (64 * ghalf + j == grow) dg = g[j];
        if ((grow >> 6) == ghalf) xv[grow] = dg;
      }
      __syncthreads();
      for (int j = 0; j < 64; ++j) {
        const int col = 64 * ghalf + j;
        if (grow < n && col < n) {
          const double sq = xv[grow] + xv[col] - 2.0 * g[j];
          drow[grow * FNP + col] = grow == col ? 0.f : static_cast<float>(sqrt(sq > 0.0 ? sq : 0.0));
        }
      }
      __syncthreads();
      // each wave sorts whole rows (the n-1 off-diagonal distances, +inf
      // padded to 128) with a register bitonic network, 2 elements per lane
      for (int row = wave; row < n; row += 4) {
        auto ld = [&](int e) -> float {
          if (e >= n - 1) return __builtin_inff();
          return drow[row * FNP + (e < row ? e : e + 1)];
        };
        float v0 = ld(2 * lane), v1 = ld(2 * lane + 1);
#pragma unroll
        for (int size = 2; size <= 128; size <<= 1) {
#pragma unroll
          for (int stride = size >> 1; stride >= 1; stride >>= 1) {
            const bool asc = ((2 * lane) & size) == 0;
            if (stride == 1) {
              const float lo = fminf(v0, v1), hi = fmaxf(v0, v1);
              v0 = asc ? lo : hi;
              v1 = asc ? hi : lo;
            } else {
              const int ls = stride >> 1;
              const float p0 = __shfl_xor(v0, ls), p1 = __shfl_xor(v1, ls);
              const bool takemin = asc != ((lane & ls) != 0);
              v0 = takemin ? fminf(v0, p0) : fmaxf(v0, p0);
              v1 = takemin ? fminf(v1, p1) : fmaxf(v1, p1);
            }
          }
        }
        drow[row * FNP + 2 * lane] = v0;
        drow[row * FNP + 2 * lane + 1] = v1;
      }
      __syncthreads();
      // score = numpy pairwise fp32 sum of the m smallest (slice semantics)
      const int m = n - fp - 2 >= 0 ? (n - fp - 2 < n - 1 ? n - fp - 2 : n - 1)
                                    : ((n - 1) + (n - fp - 2) > 0 ? (n - 1) + (n - fp - 2) : 0);
      if (tid < n) {
        const float* row = drow + tid * FNP;
        tau[tid] = static_cast<double>(np_pw32(m, [&](int q) { return row[q]; }));
      }
      __syncthreads();
      // drop the fp largest scores (ties: later index dropped first)
      if (own) {
        int keep = 0;
        if (tid < n) {
          const double si = tau[tid];
          int above = 0;
          for (int j = 0; j < n; ++j) above += (tau[j] > si || (tau[j] == si && j > tid)) ? 1 : 0;
          keep = above >= fp ? 1 : 0;
        }
        active[tid] = keep;
      }
      __syncthreads();
      // compaction of the kept clients (client order)
      if (own && active[tid]) {
        int pos = 0;
        for (int j = 0; j < tid; ++j) pos += active[j];
        kidx[pos] = tid;
      }
      n_keep = n - (fp < n ? fp : n);
      // max pairwise fp32 distance among kept clients
      float md = 0.f;
      for (int j = 0; j < 64; ++j) {
        const int col = 64 * ghalf + j;
        if (grow < n && col < n && grow < col && active[grow] && active[col]) {
          const double sq = xv[grow] + xv[col] - 2.0 * g[j];
          const float dd = static_cast<float>(sqrt(sq > 0.0 ? sq : 0.0));
          md = dd > md ? dd : md;
        }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const float o = __shfl_xor(md, off);
        md = o > md ? o : md;
      }
      if (lane == 0) red[wave] = md;
      __syncthreads();
      float mdall = static_cast<float>(red[0]);
      for (int q = 1; q < 4; ++q) mdall = static_cast<float>(red[q]) > mdall ? static_cast<float>(red[q]) : mdall;
      __syncthreads();
      step = static_cast<double>(0.5f / (mdall * mdall));
      if (own) c[tid] = (tid < n && active[tid]) ? 1.0 : 0.0;
      __syncthreads();
    } else {
      if (own) {
        active[tid] = tid < n ? 1 : 0;
        c[tid] = tid < n ? 1.0 : 0.0;
      }
      __syncthreads();
    }

    // ================= Phase C: iterations ==================================
    const int iters = MODE == 0 ? 2 * static_cast<int>(A.eps * n)
                                : static_cast<int>(2 * A.eps * n_keep);
    bool have_u = false;
    int m_hint = 0;   // Lanczos steps the previous iteration needed
    double* V = reinterpret_cast<double*>(uni);   // [LMAX][VST] Lanczos basis
    for (int it = 0; it < iters; ++it) {
      // weights, G w, w'Gw, number of active clients
      double csum = own && active[tid] ? c[tid] : 0.0;
      csum = block_sum(csum, red);
      double wi = 0.0;
      if (own) {
        wi = active[tid] ? c[tid] / csum : 0.0;
        w[tid] = wi;
        sw[tid] = sqrt(wi > 0.0 ? wi : 0.0);
      }
      __syncthreads();
      {
        const double p = gmv_row(w);
        if (ghalf == 0) gw[grow] = p;
      }
      double sacc = 0.0, cnt = own && wi > 0.0 ? 1.0 : 0.0;
      __syncthreads();
      sacc = own ? wi * gw[tid] : 0.0;
      block_sum2(sacc, cnt, red);
      if (tid == 0) scal[0] = sacc;
      const int nact = static_cast<int>(cnt);
      __syncthreads();

      // ---- top eigenpair of M = W^1/2 C W^1/2: Lanczos, full reorth ----
      const int msteps = nact < 1 ? 1 : (nact < LMAX ? nact : LMAX);
      double lam = 0.0, resid_last = 0.0;
      int rs_used = 0, m_last = 0;
      long long tm[6] = {0, 0, 0, 0, 0, 0};   // cycle probes (diagnostics only)
      long long t0c = clock64();
#pragma unroll 1
      for (int rs = 0; rs < LRESTART; ++rs) {
        // start: warm Ritz vector (perturbed on a new outer iteration) or
        // sqrt-weights times a fixed non-uniform pattern (sqrt-weights alone
        // span the null vector: M W^1/2 1 = W^1/2 C w = 0)
        double r0 = 0.0;
        if (own && sw[tid] > 0.0) {
          const double h = 0.5 + (tid * 0.6180339887498949 - floor(tid * 0.6180339887498949));
          r0 = rs > 0 ? uv[tid] : (have_u ? uv[tid] + 1e-3 * sw[tid] * h : sw[tid] * h);
        }
        const double nrm = sqrt(block_sum(r0 * r0, red));
        if (own) {
          const double q = r0 / nrm;
          V[tid] = q;
          xv[tid] = sw[tid] * q;
        }
        __syncthreads();
        int m = 0;
        bool done = false;
        double tscale = 0.0;
        double theta_lb = -1e300;   // top Ritz value of the previous check
        int next_check = m_hint > 8 ? m_hint : 8;
        // Lanczos with deferred normalisation (3-4 barriers per step):
        //   xv = W^1/2 rr, rr = beta_{j-1} q_j when `pend` (q_j not yet stored),
        //   else rr = q_j.  One operator pass yields M rr, alpha_j and |rr|^2
        //   together; full re-orthogonalisation by classical Gram-Schmidt with
        //   a second pass only when the first removed more than half of |r|^2
        //   (DGKS criterion, |r1|^2 = |r0|^2 - |h|^2).
        bool pend = false;
        double rr = own ? V[tid] : 0.0;
        double r = 0.0;
        double bprev = 0.0;
        for (int j = 0; j < msteps; ++j) {
          if (dbg) t0c = clock64();
          // ---- (1) y = G xv with the sums for the centring, alpha and |rr|^2
          {
            const double p = gmv_row(xv);
            double a1 = own ? xv[tid] : 0.0;
            double a2 = own ? gw[tid] * xv[tid] : 0.0;
            double a3 = ghalf == 0 ? xv[grow] * p : 0.0;
            double a4 = own ? rr * rr : 0.0;
            a1 = wave_sum(a1);
            a2 = wave_sum(a2);
            a3 = wave_sum(a3);
            a4 = wave_sum(a4);
            if (lane == 0) {
              red[wave] = a1;
              red[4 + wave] = a2;
              red[8 + wave] = a3;
              red[12 + wave] = a4;
            }
            if (ghalf == 0) yv[grow] = p;
          }
          __syncthreads();
          if (dbg) { const long long t = clock64(); tm[0] += t - t0c; t0c = t; }
          // ---- (2) r = M q_j - alpha_j q_j - beta_{j-1} q_{j-1}
          double aj;
          {
            const double s1 = (red[0] + red[1]) + (red[2] + red[3]);
            const double gy = (red[4] + red[5]) + (red[6] + red[7]);
            const double xgx = (red[8] + red[9]) + (red[10] + red[11]);
            const double nrm2 = (red[12] + red[13]) + (red[14] + red[15]);
            const double bet = pend ? sqrt(nrm2) : 1.0;
            if (pend) {
              bprev = bet;
              if (tid == 0) {
                beta[j - 1] = bet;
                beta2[j - 1] = bet * bet;
              }
            }
            aj = (xgx - 2.0 * s1 * gy + scal[0] * s1 * s1) / (bet * bet);
            tscale = fmax(tscale, fabs(aj) + bprev);
            if (own) {
              const double q = rr / bet;
              if (pend) V[j * VST + tid] = q;
              r = sw[tid] * (yv[tid] - gw[tid] * s1 - gy + scal[0] * s1) / bet - aj * q;
              if (j > 0) r -= bprev * V[(j - 1) * VST + tid];
              rv[tid] = r;
            }
          }
          __syncthreads();
          if (dbg) { const long long t = clock64(); tm[1] += t - t0c; t0c = t; }
          // ---- (3) re-orthogonalisation against q_0..q_j
          double est2 = 0.0;   // |r|^2 after the last pass (Pythagoras)
#pragma unroll 1
          for (int pass = 0; pass < 2; ++pass) {
            {
              // 4 lanes per basis vector, 16-byte chunks interleaved; slot
              // j+1 is |r|^2 itself
              const int qq = tid >> 2, part = tid & 3;
              double h0 = 0.0, h1 = 0.0;
              if (qq <= j + 1) {
                const double2* vq = reinterpret_cast<const double2*>(qq <= j ? V + qq * VST : rv) + part;
                const double2* rp = reinterpret_cast<const double2*>(rv) + part;
#pragma unroll
                for (int e = 0; e < 64; e += 8) {
                  const double2 a = vq[e], b = rp[e];
                  const double2 c2 = vq[e + 4], d2 = rp[e + 4];
                  h0 += a.x * b.x + a.y * b.y;
                  h1 += c2.x * d2.x + c2.y * d2.y;
                }
              }
              double h = h0 + h1;
              h += dpp_f64<0xB1>(h);
              h += dpp_f64<0x4E>(h);
              if (part == 0 && qq <= j + 1) hq[qq] = h;
            }
            __syncthreads();
            double hn2 = 0.0;
            {
              double u0 = 0.0, u1 = 0.0, u2 = 0.0, u3 = 0.0;
              int qq = 0;
              for (; qq + 3 <= j; qq += 4) {
                const double c0 = hq[qq], c1 = hq[qq + 1], c2 = hq[qq + 2], c3 = hq[qq + 3];
                hn2 += (c0 * c0 + c1 * c1) + (c2 * c2 + c3 * c3);
                if (own) {
                  u0 += c0 * V[qq * VST + tid];
                  u1 += c1 * V[(qq + 1) * VST + tid];
                  u2 += c2 * V[(qq + 2) * VST + tid];
                  u3 += c3 * V[(qq + 3) * VST + tid];
                }
              }
              for (; qq <= j; ++qq) {
                const double c0 = hq[qq];
                hn2 += c0 * c0;
                if (own) u0 += c0 * V[qq * VST + tid];
              }
              if (own) r -= (u0 + u1) + (u2 + u3);
            }
            const double r02 = hq[j + 1];
            est2 = r02 - hn2;
            if (tid == 0) alpha[j] = pass == 0 ? aj + hq[j] : alpha[j] + hq[j];
            // DGKS: a second pass only if the first removed over half of |r|^2
            if (pass == 1 || !(est2 < 0.5 * r02)) break;
            if (own) rv[tid] = r;
            __syncthreads();
          }
          if (dbg) { const long long t = clock64(); tm[2] += t - t0c; t0c = t; }
          m = j + 1;
          const bool maybe_breakdown = !(est2 > 1e-26 * tscale * tscale);
          const bool check = m == msteps || maybe_breakdown || m >= next_check;
          if (!check) {
            // deferred normalisation: the next step's operator pass measures |r|
            if (own) {
              rr = r;
              xv[tid] = sw[tid] * r;
            }
            pend = true;
            __syncthreads();
            continue;
          }
          const double bj = sqrt(block_sum(own ? r * r : 0.0, red));
          if (dbg) { const long long t = clock64(); tm[3] += t - t0c; t0c = t; }
          if (tid == 0) {
            beta[j] = bj;
            beta2[j] = bj * bj;
          }
          const bool breakdown = !(bj > 1e-14 * tscale);
          const bool last = m == msteps || breakdown;
          {
            __syncthreads();
            // top eigenpair of T_m (wave 0, T in registers: lane q holds
            // alpha_q, beta_q): multisection on Sturm counts, bracket from the
            // previous check's Ritz value (interlacing: it only grows with m),
            // then the eigenvector from a twisted factorisation
            if (wave == 0) {
              const double al = lane < m ? alpha[lane] : 0.0;
              const double bl = lane + 1 < m ? beta[lane] : 0.0;
              const double bp = (lane >= 1 && lane < m) ? beta[lane - 1] : 0.0;
              const double rad = fabs(bp) + fabs(bl);
              double lo = wave_min(lane < m ? al - rad : 1e300);
              double hi = wave_max(lane < m ? al + rad : -1e300);
              const double tiny = 1e-300 + 1e-30 * tscale;
              // 64-point multisection on Sturm counts.  The count uses the
              // division-free three-term recurrence of the leading principal
              // minors p_q (d_q = p_q / p_{q-1} of the LDL^T pivots, same
              // tiny-pivot rule), rescaled by exact powers of two every 4
              // steps, so the dependent chain is one FMA per step.  With a
              // previous Ritz value (a lower bound, interlacing) the first
              // round's points are geometric above it, since the top value
              // has moved little.
              const bool geo = theta_lb > lo && theta_lb < hi;
              if (geo) lo = theta_lb;
              for (int round = 0; round < 16; ++round) {
                const double fr = (geo && round == 0) ? __builtin_amdgcn_ldexp(1.0, lane - 63)
                                                      : (lane + 1) / 65.0;
                const double x = lo + (hi - lo) * fr;
                // alpha / beta^2 come from LDS at wave-uniform addresses (off
                // the dependent chain); a zero minor keeps its sign bit (no
                // division, so no tiny-pivot substitution is needed)
                double p2 = 1.0;
                double p1 = alpha[0] - x;
                int cntb = __builtin_signbit(p1) ? 1 : 0;
#pragma unroll 4
                for (int q = 1; q < m; ++q) {
                  const double pk = fma(alpha[q] - x, p1, -(beta2[q - 1] * p2));
                  cntb += (__builtin_signbit(pk) ? 1 : 0) != (__builtin_signbit(p1) ? 1 : 0);
                  p2 = p1;
                  p1 = pk;
                  if ((q & 3) == 3) {
                    const int e = __builtin_amdgcn_frexp_exp(p1);
                    p1 = __builtin_amdgcn_ldexp(p1, -e);
                    p2 = __builtin_amdgcn_ldexp(p2, -e);
                  }
                }
                const unsigned long long ok = __builtin_amdgcn_ballot_w64(cntb >= m);
                const int first = ok ? __builtin_ctzll(ok) : 64;
                const double flo = first == 0 ? 0.0
                                              : ((geo && round == 0) ? __builtin_amdgcn_ldexp(1.0, first - 64)
                                                                     : first / 65.0);
                const double fhi = (geo && round == 0) ? __builtin_amdgcn_ldexp(1.0, first - 63)
                                                       : (first + 1) / 65.0;
                const double nlo = lo + (hi - lo) * flo;
                const double nhi = first < 64 ? lo + (hi - lo) * fhi : hi;
                lo = nlo;
                hi = nhi;
                if (hi - lo <= 2e-16 * fmax(fabs(lo), fabs(hi))) break;
              }
              if (dbg) tm[5] += clock64() - t0c;
              const double lm = 0.5 * (lo + hi);
              // twisted factorisation of T - lm I: forward pivots dp, backward dm
              double dpv = 0.0, dmv = 0.0;
              {
                double dp = readlane_f64(al, 0) - lm;
                if (fabs(dp) < tiny) dp = -tiny;
                dpv = writelane_f64(dp, 0, dpv);
                for (int q = 1; q < m; ++q) {
                  dp = (alpha[q] - lm) - fdiv(beta2[q - 1], dp);
                  if (fabs(dp) < tiny) dp = -tiny;
                  dpv = writelane_f64(dp, q, dpv);
                }
                double dm = readlane_f64(al, m - 1) - lm;
                if (fabs(dm) < tiny) dm = -tiny;
                dmv = writelane_f64(dm, m - 1, dmv);
                for (int q = m - 2; q >= 0; --q) {
                  dm = (alpha[q] - lm) - fdiv(beta2[q], dm);
                  if (fabs(dm) < tiny) dm = -tiny;
                  dmv = writelane_f64(dm, q, dmv);
                }
              }
              // twist index: smallest |gamma_q| = |dp_q + dm_q - (alpha_q - lm)|
              double gam = lane < m ? fabs(dpv + dmv - (al - lm)) : 1e308;
              int tw = lane;
#pragma unroll
              for (int off = 32; off >= 1; off >>= 1) {
                const double og = __shfl_xor(gam, off);
                const int ot = __shfl_xor(tw, off);
                if (og < gam || (og == gam && ot < tw)) {
                  gam = og;
                  tw = ot;
                }
              }
              tw = __builtin_amdgcn_readfirstlane(tw);
              // z_tw = 1; z_q = -(b_q / dp_q) z_{q+1} below, z_{q+1} = -(b_q / dm_{q+1}) z_q above
              const double dmn = __shfl_down(dmv, 1);
              const double fdown = lane < m ? -bl / dpv : 0.0;
              const double fup = lane + 1 < m ? -bl / dmn : 0.0;
              double zv = lane == tw ? 1.0 : 0.0;
              double z = 1.0;
              for (int q = tw - 1; q >= 0; --q) {
                z *= readlane_f64(fdown, q);
                zv = writelane_f64(z, q, zv);
              }
              z = 1.0;
              for (int q = tw; q + 1 < m; ++q) {
                z *= readlane_f64(fup, q);
                zv = writelane_f64(z, q + 1, zv);
              }
              if (lane >= m) zv = 0.0;
              const double amax = wave_max(fabs(zv));
              const double zs = zv / amax;
              const double nn = amax * sqrt(wave_sum(zs * zs));
              zv = zv / nn;
              if (lane < m) svec[lane] = zv;
              if (lane == 0) {
                scal[1] = lm;
                scal[2] = fabs(bj * readlane_f64(zv, m - 1));
              }
            }
            __syncthreads();
            lam = scal[1];
            resid_last = scal[2];
            theta_lb = lam;
            next_check = m + 8;
            if (dbg) { const long long t = clock64(); tm[4] += t - t0c; t0c = t; }
            done = last || resid_last <= 1e-13 * fabs(lam);
            if (done) break;
          }
          if (own) {
            const double qn = r / bj;
            V[(j + 1) * VST + tid] = qn;
            xv[tid] = sw[tid] * qn;
            rr = qn;
          }
          pend = false;
          bprev = bj;
          __syncthreads();
        }
        // Ritz vector
        if (own) {
          double u = 0.0;
          for (int q = 0; q < m; ++q) u += V[q * VST + tid] * svec[q];
          uv[tid] = u;
        }
        m_last = m;
        rs_used = rs + 1;
        m_hint = m;
        __syncthreads();
        if (m >= nact || resid_last <= 1e-13 * fabs(lam)) break;
      }
      have_u = true;
      if (dbg && it < 256) {
        double* rec = A.dbg + FNP * FNP + static_cast<int64_t>(it) * kDbgRec;
        if (own) rec[tid] = c[tid];
        if (tid == 0) {
          rec[FNP] = lam;
          rec[FNP + 1] = m_last;
          rec[FNP + 2] = resid_last;
          rec[FNP + 3] = rs_used;
          rec[FNP + 4] = nact;
          rec[FNP + 5] = scal[0];
          for (int q = 0; q < 6; ++q) rec[FNP + 6 + q] = static_cast<double>(tm[q]);
        }
      }
      // ---- early exit (robust_estimator.py:164 / :70) ----
      if (lam * lam <= A.expansion * A.sigma * A.sigma) break;
      // ---- tau_j = ((x_j - mu).v)^2 = (C W^1/2 u)_j^2 / lam ----
      if (own) xv[tid] = sw[tid] * uv[tid];
      __syncthreads();
      const double cu = cmul();
      const double ti = own ? cu * cu / lam : 0.0;
      if constexpr (MODE == 0) {
        // c *= 1 - tau/tau_max; drop argmax (first index); c /= |c|_1
        double tmax = 0.0;
        const int p = block_argmax_first(own && active[tid] ? ti : -__builtin_inf(), tid, red,
                                         reinterpret_cast<int*>(iscal), &tmax);
        double cn = 0.0;
        if (own && active[tid] && tid != p) cn = c[tid] * (1.0 - ti / tmax);
        const double l1 = block_sum(fabs(cn), red);
        if (own) {
          c[tid] = cn / l1;
          if (tid == p) active[tid] = 0;
        }
        __syncthreads();
      } else {
        // c *= 1 - step*tau, then the KL projection onto
        // {sum c = 1, c <= cap} (robust_estimator.py:77-99)
        const int nk = n_keep;
        const double cap = 1.0 / (1.0 - A.eps) / nk;
        if (own && active[tid]) c[tid] = c[tid] * (1.0 - step * ti);
        __syncthreads();
        double* cc = rv;   // compacted weights
        if (tid < nk) cc[tid] = c[kidx[tid]];
        __syncthreads();
        // descending rank; ties: later compact index first (flip of a
        // stable ascending order)
        if (tid < nk) {
          const double v = cc[tid];
          int rk = 0;
          for (int q = 0; q < nk; ++q) rk += (cc[q] > v || (cc[q] == v && q > tid)) ? 1 : 0;
          irank[tid] = rk;
          sv[rk] = v;
          hl[rk] = v * log(v / cap);
        }
        __syncthreads();
        // candidate i caps the i+1 largest at cap and rescales the rest
        double negkl = -__builtin_inf(), scale = 0.0;
        int stop = 1 << 30;
        if (tid < nk) {
          const int i = tid;
          const double clip = 1.0 - np_pw64(0, i + 1, [&](int) { return cap; });
          if (clip <= 0.0) {
            stop = i;
          } else if (i + 1 < nk) {
            const double norm = np_pw64(i + 1, nk - i - 1, [&](int q) { return sv[q]; });
            scale = clip / norm;
            if (!(sv[i + 1] * scale > cap)) {
              double head = 0.0;
              for (int q = 0; q <= i; ++q) head += hl[q];
              negkl = -(head - norm * log(scale));
            }
          }
        }
        const int istop = block_min_int(stop, reinterpret_cast<int*>(iscal));
        if (tid >= istop) negkl = -__builtin_inf();
        double best = 0.0;
        const int bi = block_argmax_first(negkl, tid, red, reinterpret_cast<int*>(iscal), &best);
        if (!(best > -__builtin_inf())) {
          if (tid == 0) *A.status = 2;   // projected_c None -> TypeError in the reference
          break;
        }
        if (tid == bi) scal[3] = scale;
        __syncthreads();
        if (tid < nk) c[kidx[tid]] = irank[tid] <= bi ? cap : cc[tid] * scal[3];
        __syncthreads();
      }
    }

    // ================= Phase D: weighted mean over the chunk ================
    {
      if (tid == 0) {
        // np.average's scale: pairwise sum of the kept weights in order
        int q = 0;
        for (int i = 0; i < n; ++i)
          if (active[i]) rv[q++] = c[i];
        scal[4] = np_pw64(0, q, [&](int z) { return rv[z]; });
      }
      __syncthreads();
      const double cs = scal[4];
      for (int cc2 = tid; cc2 < k; cc2 += 256) {
        double s = 0.0;
        for (int i = 0; i < n; ++i)
          if (active[i]) s += static_cast<double>(A.X[static_cast<int64_t>(i) * A.ldx + k0 + cc2]) * c[i];
        A.out[k0 + cc2] = s / cs;
      }
      __syncthreads();
    }
  }
}

size_t filter_lds_bytes() {
  return FilterShared::kUnionBytes + sizeof(double) * (9 * FNP + 6 * LMAX + 32) + sizeof(int) * (3 * FNP + 16);
}

int launch_filter(int mode, const float* X, int n, int64_t d, int64_t ldx, int itv, double eps, double sigma,
                  double expansion, double* out, int* status, double* dbg, hipStream_t s) {
  SRA_REQUIRE(n >= 1 && n <= FNP, SRA_ERR_UNSUPPORTED, "spectral filters support 1 <= N <= %d (got %d)", FNP, n);
  SRA_REQUIRE(itv >= 1, SRA_ERR_ARG, "itv must be >= 1");
  const int64_t nchunks = cdiv(d, itv);
  SRA_REQUIRE(nchunks < (int64_t(1) << 31), SRA_ERR_ARG, "too many chunks");
  FilterArgs a{X, n, d, ldx, itv, static_cast<int>(nchunks), eps, sigma, expansion, out, status, dbg};
  const size_t lds = filter_lds_bytes();
  const int grid = static_cast<int>(nchunks < 512 ? nchunks : 512);
  if (mode == 0) {
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&spectral_filter_kernel<0>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    hipLaunchKernelGGL(spectral_filter_kernel<0>, dim3(grid), dim3(256), lds, s, a);
  } else {
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&spectral_filter_kernel<1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    hipLaunchKernelGGL(spectral_filter_kernel<1>, dim3(grid), dim3(256), lds, s, a);
  }
  return launch_status("spectral_filter_kernel");
}

}  // namespace sra

extern "C" int sra_filter_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                              double eps, double sigma, double expansion, double* out, int32_t* status,
                              void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr && status != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx");
  SRA_REQUIRE(mode == 0 || mode == 1, SRA_ERR_ARG, "mode must be 0 (filterL2) or 1 (ex_noregret)");
  // ex_noregret drops ceil(eps*n) clients and takes the max over the pairwise
  // distances of the rest: the reference raises (amax of an empty list) below 2
  SRA_REQUIRE(mode == 0 || n - static_cast<int64_t>(std::ceil(eps * n)) >= 2, SRA_ERR_ARG,
              "ex_noregret needs at least 2 clients after dropping ceil(eps*n)");
  return sra::launch_filter(mode, X, static_cast<int>(n), d, ldx, itv, eps, sigma, expansion, out, status,
                            nullptr, static_cast<hipStream_t>(stream));
}

extern "C" int sra_filter_debug_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                                    double eps, double sigma, double expansion, double* out, int32_t* status,
                                    double* dbg, void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr && status != nullptr && dbg != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx");
  SRA_REQUIRE(mode == 0 || mode == 1, SRA_ERR_ARG, "mode must be 0 (filterL2) or 1 (ex_noregret)");
  SRA_REQUIRE(mode == 0 || n - static_cast<int64_t>(std::ceil(eps * n)) >= 2, SRA_ERR_ARG,
              "ex_noregret needs at least 2 clients after dropping ceil(eps*n)");
  return sra::launch_filter(mode, X, static_cast<int>(n), d, ldx, itv, eps, sigma, expansion, out, status, dbg,
                            static_cast<hipStream_t>(stream));
}
