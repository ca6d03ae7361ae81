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
constexpr int LMAX = 64;           // Lanczos steps per restart (V fills the 64 KB union)
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

// ----- block helpers (256 threads) ------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
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

// ----- Sturm count: eigenvalues of the tridiagonal (a, b) below x ------------
__device__ __forceinline__ int sturm_count(const double* a, const double* b, int m, double x) {
  int cnt = 0;
  double dd = a[0] - x;
  if (dd < 0) ++cnt;
  for (int k = 1; k < m; ++k) {
    const double den = (dd == 0.0) ? 1e-300 : dd;
    dd = (a[k] - x) - b[k - 1] * b[k - 1] / den;
    if (dd < 0) ++cnt;
  }
  return cnt;
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

template <int MODE>  // 0: filterL2, 1: ex_noregret
__global__ void __launch_bounds__(256) spectral_filter_kernel(FilterArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* uni = smem;                                     // 64 KB union
  double* vec = reinterpret_cast<double*>(smem + FilterShared::kUnionBytes);
  double* c = vec;                 // weights (kept/active clients)
  double* w = vec + 1 * FNP;       // normalised weights
  double* sw = vec + 2 * FNP;      // sqrt(w)
  double* gw = vec + 3 * FNP;      // G w
  double* xv = vec + 4 * FNP;      // Lanczos work vector / generic input
  double* yv = vec + 5 * FNP;      // output of the operator
  double* rv = vec + 6 * FNP;      // Lanczos residual
  double* uv = vec + 7 * FNP;      // Ritz vector (warm start)
  double* tau = vec + 8 * FNP;
  double* alpha = vec + 9 * FNP;             // [LMAX]
  double* beta = alpha + LMAX;               // [LMAX]
  double* svec = beta + LMAX;                // [LMAX] eigenvector of T
  double* red = svec + LMAX;                 // [8]
  double* scal = red + 8;                    // [16] broadcast scalars
  double* tcp = scal + 16;                   // [LMAX] tridiagonal solve scratch
  double* tdp = tcp + LMAX;                  // [LMAX]
  int* active = reinterpret_cast<int*>(tdp + LMAX);   // [FNP]
  int* iscal = active + FNP;                          // [16]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int n = A.n;
  const int grow = tid >> 1;   // G row owned by this thread
  const int ghalf = tid & 1;   // which 64 columns

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

    // operator helpers -------------------------------------------------------
    // yv = G * xv  (all rows)
    auto gmv = [&](const double* x, double* y) {
      double p = 0.0;
#pragma unroll
      for (int j = 0; j < 64; ++j) p += g[j] * x[64 * ghalf + j];
      p += __shfl_xor(p, 1);
      if (ghalf == 0) y[grow] = p;
      __syncthreads();
    };
    // y = C (sw o x) [post-scaled by sw if scale_out]; s_gw = w^T G w in scal[0]
    auto cop = [&](const double* x, double* y, bool scale_out) {
      if (tid < FNP) xv[tid] = sw[tid] * x[tid];
      __syncthreads();
      const double s1 = block_sum(tid < FNP ? xv[tid] : 0.0, red);
      const double gy = block_sum(tid < FNP ? gw[tid] * xv[tid] : 0.0, red);
      gmv(xv, yv);
      if (tid < FNP) {
        const double cy = yv[tid] - gw[tid] * s1 - gy + scal[0] * s1;
        y[tid] = scale_out ? sw[tid] * cy : cy;
      }
      __syncthreads();
    };

    // ============ ex_noregret: Krum pre-filter on the chunk =================
    int n_keep = n;
    double step = 0.0;
    if constexpr (MODE == 1) {
      const int fp = static_cast<int>(ceil(A.eps * n));
      float* drow = reinterpret_cast<float*>(uni);   // [FNP][FNP] fp32 distances, row i sorted later
      // diag of G into xv (compile-time register indices only)
      {
        double dg = 0.0;
#pragma unroll
        for (int j = 0; j < 64; ++j)
          if (64 * ghalf + j == grow) dg = g[j];
        if ((grow >> 6) == ghalf) xv[grow] = dg;
      }
      __syncthreads();
      // fill distances from the register rows: thread (row, half) writes its 64 entries
      for (int j = 0; j < 64; ++j) {
        const int col = 64 * ghalf + j;
        if (grow < n && col < n) {
          const double sq = xv[grow] + xv[col] - 2.0 * g[j];
          drow[grow * FNP + col] = grow == col ? 0.f : static_cast<float>(sqrt(sq > 0.0 ? sq : 0.0));
        }
      }
      __syncthreads();
      // per row: sort the n-1 off-diagonal distances (insertion sort, one lane
      // per row) and score with numpy's pairwise fp32 sum of the m smallest
      const int m = n - fp - 2 >= 0 ? (n - fp - 2 < n - 1 ? n - fp - 2 : n - 1)
                                    : ((n - 1) + (n - fp - 2) > 0 ? (n - 1) + (n - fp - 2) : 0);
      if (tid < n) {
        float* row = drow + tid * FNP;
        // move the diagonal out: compact to n-1 entries
        int p = 0;
        for (int j = 0; j < n; ++j)
          if (j != tid) row[p++] = row[j];
        for (int a = 1; a < n - 1; ++a) {
          const float v = row[a];
          int b = a - 1;
          while (b >= 0 && row[b] > v) {
            row[b + 1] = row[b];
            --b;
          }
          row[b + 1] = v;
        }
        tau[tid] = static_cast<double>(np_pw32(m, [&](int q) { return row[q]; }));
      }
      __syncthreads();
      // drop the fp largest scores (ties: later index dropped first, like a
      // stable partition from the top)
      if (tid < FNP) active[tid] = tid < n ? 1 : 0;
      __syncthreads();
      if (tid == 0) {
        for (int r = 0; r < fp && r < n; ++r) {
          int best = -1;
          double bv = -1.0;
          for (int i = 0; i < n; ++i)
            if (active[i] && (best < 0 || tau[i] >= bv)) { bv = tau[i]; best = i; }
          if (best >= 0) active[best] = 0;
        }
        int cnt = 0;
        for (int i = 0; i < n; ++i) cnt += active[i];
        iscal[0] = cnt;
      }
      __syncthreads();
      n_keep = iscal[0];
      // max pairwise distance (fp32, from the unsorted definition) among kept
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
      const float sq32 = mdall * mdall;
      step = static_cast<double>(0.5f / sq32);
      if (tid < FNP) c[tid] = (tid < n && active[tid]) ? 1.0 : 0.0;
      __syncthreads();
    } else {
      if (tid < FNP) {
        active[tid] = tid < n ? 1 : 0;
        c[tid] = tid < n ? 1.0 : 0.0;
      }
      __syncthreads();
    }

    // ================= Phase C: iterations ==================================
    const int iters = MODE == 0 ? 2 * static_cast<int>(A.eps * n)
                                : static_cast<int>(2 * A.eps * n_keep);
    bool have_u = false;
    for (int it = 0; it < iters; ++it) {
      // weights
      const double csum = block_sum(tid < FNP && active[tid] ? c[tid] : 0.0, red);
      if (tid < FNP) {
        const double wi = active[tid] ? c[tid] / csum : 0.0;
        w[tid] = wi;
        sw[tid] = sqrt(wi > 0.0 ? wi : 0.0);
      }
      __syncthreads();
      gmv(w, gw);
      {
        const double s = block_sum(tid < FNP ? w[tid] * gw[tid] : 0.0, red);
        if (tid == 0) {
          scal[0] = s;
          if (dbg) { scal[4] = csum; scal[5] = s; scal[6] = gw[0]; scal[7] = sw[0]; }
        }
        __syncthreads();
      }
      // ---- Lanczos on M = W^1/2 C W^1/2 ----
      int nact = 0;
      {
        const double cnt = block_sum(tid < FNP && sw[tid] > 0.0 ? 1.0 : 0.0, red);
        nact = static_cast<int>(cnt);
      }
      int msteps = nact < LMAX ? nact : LMAX;
      if (msteps < 1) msteps = 1;
      double* V = reinterpret_cast<double*>(uni);   // [LMAX][FNP]
      double lam = 0.0, resid_last = 0.0;
      int rs_used = 0, m_last = 0;
#pragma unroll 1
      for (int rs = 0; rs < LRESTART; ++rs) {
      // start vector: previous Ritz vector (warm; perturbed towards sqrt-weights
      // on a new outer iteration so no active client is missed) or sqrt-weights
      if (tid < FNP)
        rv[tid] = (sw[tid] > 0.0) ? (rs > 0 ? uv[tid] : (have_u ? uv[tid] + 1e-3 * sw[tid] : sw[tid])) : 0.0;
      __syncthreads();
      {
        const double nrm = sqrt(block_sum(tid < FNP ? rv[tid] * rv[tid] : 0.0, red));
        if (tid < FNP) V[tid] = rv[tid] / nrm;
        if (dbg && tid == 0 && rs == 0) { scal[8] = nrm; scal[9] = rv[0]; }
        __syncthreads();
      }
      int mused = msteps;
      for (int j = 0; j < msteps; ++j) {
        double* qj = V + j * FNP;
        cop(qj, rv, true);     // rv = M q_j
        const double aj = block_sum(tid < FNP ? qj[tid] * rv[tid] : 0.0, red);
        if (tid < FNP) {
          double r = rv[tid] - aj * qj[tid];
          if (j > 0) r -= beta[j - 1] * V[(j - 1) * FNP + tid];
          rv[tid] = r;
        }
        if (tid == 0) alpha[j] = aj;
        if (dbg && tid == 0 && rs == 0 && j == 0) { scal[10] = aj; scal[11] = rv[0]; scal[12] = yv[0]; scal[13] = xv[0]; }
        __syncthreads();
        // full reorthogonalisation (classical Gram-Schmidt, twice)
        for (int pass = 0; pass < 2; ++pass) {
          if (tid <= j) {
            double h = 0.0;
            for (int i = 0; i < FNP; ++i) h += V[tid * FNP + i] * rv[i];
            svec[tid] = h;
          }
          __syncthreads();
          if (tid < FNP) {
            double r = rv[tid];
            for (int q = 0; q <= j; ++q) r -= svec[q] * V[q * FNP + tid];
            rv[tid] = r;
          }
          __syncthreads();
        }
        const double bj = sqrt(block_sum(tid < FNP ? rv[tid] * rv[tid] : 0.0, red));
        if (tid == 0) beta[j] = bj;
        if (dbg && tid == 0 && rs == 0 && j == 0) { scal[14] = bj; scal[15] = V[0]; }
        __syncthreads();
        if (j + 1 >= msteps || !(bj > 1e-300) || bj <= 1e-13 * (aj > 0 ? aj : -aj)) {
          mused = j + 1;
          break;
        }
        if (tid < FNP) V[(j + 1) * FNP + tid] = rv[tid] / bj;
        __syncthreads();
      }
      // ---- top eigenpair of the tridiagonal (alpha, beta[0..m-2]) ----
      if (wave == 0) {
        // Gershgorin bounds
        double lo = 1e300, hi = -1e300;
        for (int q = 0; q < mused; ++q) {
          const double rad = (q > 0 ? fabs(beta[q - 1]) : 0.0) + (q + 1 < mused ? fabs(beta[q]) : 0.0);
          lo = fmin(lo, alpha[q] - rad);
          hi = fmax(hi, alpha[q] + rad);
        }
        // multisection for the largest eigenvalue: count(x) = #eig < x;
        // the largest lies where count crosses from mused-1 to mused
        for (int round = 0; round < 12; ++round) {
          const double x = lo + (hi - lo) * (lane + 1) / 65.0;
          const int cnt = sturm_count(alpha, beta, mused, x);
          const unsigned long long ok = __builtin_amdgcn_ballot_w64(cnt >= mused);  // x above all
          // first lane whose x is above the top eigenvalue
          const int first = ok ? __builtin_ctzll(ok) : 64;
          const double nlo = lo + (hi - lo) * first / 65.0;
          const double nhi = first < 64 ? lo + (hi - lo) * (first + 1) / 65.0 : hi;
          lo = nlo;
          hi = nhi;
        }
        const double lam = 0.5 * (lo + hi);
        if (lane == 0) {
          scal[1] = lam;
          // inverse iteration on (T - lam I) with a tiny shift
          const int m = mused;
          double shift = lam + 1e-12 * (fabs(lam) + 1e-300);
          for (int q = 0; q < m; ++q) svec[q] = 1.0;
          for (int pass = 0; pass < 3; ++pass) {
            // Thomas algorithm on (T - shift I) x = svec
            double* cp = tcp;
            double* dp = tdp;
            double den = alpha[0] - shift;
            if (den == 0.0) den = 1e-300;
            cp[0] = (m > 1 ? beta[0] : 0.0) / den;
            dp[0] = svec[0] / den;
            for (int q = 1; q < m; ++q) {
              den = (alpha[q] - shift) - beta[q - 1] * cp[q - 1];
              if (den == 0.0) den = 1e-300;
              cp[q] = (q + 1 < m ? beta[q] : 0.0) / den;
              dp[q] = (svec[q] - beta[q - 1] * dp[q - 1]) / den;
            }
            svec[m - 1] = dp[m - 1];
            for (int q = m - 2; q >= 0; --q) svec[q] = dp[q] - cp[q] * svec[q + 1];
            double nn = 0.0;
            for (int q = 0; q < m; ++q) nn += svec[q] * svec[q];
            nn = sqrt(nn);
            for (int q = 0; q < m; ++q) svec[q] /= nn;
          }
          iscal[1] = m;
        }
      }
      __syncthreads();
      lam = scal[1];
      const int m = iscal[1];
      if (tid < FNP) {
        double u = 0.0;
        for (int q = 0; q < m; ++q) u += V[q * FNP + tid] * svec[q];
        uv[tid] = u;
      }
      __syncthreads();
      // Ritz residual |beta_m s_m|: stop when the pair is converged to fp64
      // level or the Krylov space is the whole active subspace
      const double resid = fabs(beta[m - 1] * svec[m - 1]);
      resid_last = resid;
      m_last = m;
      rs_used = rs + 1;
      if (m >= nact || resid <= 1e-13 * fabs(lam)) break;
      __syncthreads();
      }
      have_u = true;
      if (dbg && it < 256) {
        double* rec = A.dbg + FNP * FNP + static_cast<int64_t>(it) * kDbgRec;
        if (tid < FNP) rec[tid] = c[tid];
        if (tid == 0) {
          rec[FNP] = lam;
          rec[FNP + 1] = m_last;
          rec[FNP + 2] = resid_last;
          rec[FNP + 3] = rs_used;
          for (int q = 4; q < 16; ++q) rec[FNP + q] = scal[q];
        }
      }
      // ---- early exit ----
      if (lam * lam <= A.expansion * A.sigma * A.sigma) break;
      // ---- tau = (C W^1/2 u)^2 / lam ----
      cop(uv, rv, false);
      if (tid < FNP) tau[tid] = active[tid] ? rv[tid] * rv[tid] / lam : -1.0;
      __syncthreads();
      if constexpr (MODE == 0) {
        if (tid == 0) {
          int best = -1;
          double bv = 0.0;
          for (int i = 0; i < n; ++i)
            if (active[i] && (best < 0 || tau[i] > bv)) { bv = tau[i]; best = i; }
          iscal[2] = best;
          scal[2] = bv;
        }
        __syncthreads();
        const int p = iscal[2];
        const double tmax = scal[2];
        if (tid < FNP && active[tid]) c[tid] = c[tid] * (1.0 - tau[tid] / tmax);
        __syncthreads();
        if (tid == 0 && p >= 0) {
          active[p] = 0;
          c[p] = 0.0;
        }
        __syncthreads();
        const double l1 = block_sum(tid < FNP && active[tid] ? fabs(c[tid]) : 0.0, red);
        if (tid < FNP && active[tid]) c[tid] = c[tid] / l1;
        __syncthreads();
      } else {
        if (tid < FNP && active[tid]) c[tid] = c[tid] * (1.0 - step * tau[tid]);
        __syncthreads();
        // ---- KL projection onto {sum c = 1, c <= cap} (robust_estimator.py:77-99) ----
        // compact kept weights in client order: cc[0..nk)
        double* cc = rv;        // compacted c
        double* cand = yv;      // candidate KL per i (thread i)
        int* desc = reinterpret_cast<int*>(xv);   // ranks: desc[q] = compact index of q-th largest
        int* rank = desc + FNP;                   // rank of compact index
        if (tid == 0) {
          int q = 0;
          for (int i = 0; i < n; ++i)
            if (active[i]) cc[q++] = c[i];
          // descending order = np.flip(np.argsort(c)) ; insertion sort by value,
          // ties: later index first (flip of a stable ascending order)
          for (int a = 0; a < q; ++a) desc[a] = a;
          for (int a = 1; a < q; ++a) {
            const int v = desc[a];
            int b = a - 1;
            while (b >= 0 && (cc[desc[b]] < cc[v] || (cc[desc[b]] == cc[v] && desc[b] < v))) {
              desc[b + 1] = desc[b];
              --b;
            }
            desc[b + 1] = v;
          }
          for (int a = 0; a < q; ++a) rank[desc[a]] = a;
          iscal[3] = q;
        }
        __syncthreads();
        const int nk = iscal[3];
        const double cap = 1.0 / (1.0 - A.eps) / nk;
        // candidate i (thread i): cap the i+1 largest, rescale the rest
        double kl = __builtin_inf();
        int feasible = 0, stop = 0;
        if (tid < nk) {
          const int i = tid;
          const double clip = 1.0 - np_pw64(0, i + 1, [&](int) { return cap; });
          if (clip <= 0.0) {
            stop = 1;
          } else if (i + 1 < nk) {
            const double norm = np_pw64(0, nk - i - 1, [&](int q) { return cc[desc[i + 1 + q]]; });
            const double scale = clip / norm;
            if (!(cc[desc[i + 1]] * scale > cap)) {
              feasible = 1;
              kl = np_pw64(0, nk, [&](int q) {
                const double x = cc[q];
                const double y = rank[q] <= i ? cap : cc[q] * scale;
                return (x > 0.0 && y > 0.0) ? x * log(x / y) : (x == 0.0 && y >= 0.0 ? 0.0 : __builtin_inf());
              });
            }
          }
        }
        __syncthreads();
        if (tid < nk) {
          cand[tid] = feasible ? kl : __builtin_inf();
          reinterpret_cast<int*>(tau)[tid] = stop;   // reuse tau storage for flags
        }
        __syncthreads();
        if (tid == 0) {
          // the reference loops i upward and breaks at the first clip <= 0
          int best = -1;
          double bv = 0.0;
          for (int i = 0; i < nk; ++i) {
            if (reinterpret_cast<int*>(tau)[i]) break;
            if (cand[i] < __builtin_inf() && (best < 0 || cand[i] < bv)) { bv = cand[i]; best = i; }
          }
          iscal[4] = best;
          if (best < 0) *A.status = 2;   // projected_c None -> TypeError in the reference
        }
        __syncthreads();
        const int bi = iscal[4];
        if (bi >= 0) {
          // apply the chosen candidate (per compact index)
          const double clip = 1.0 - np_pw64(0, bi + 1, [&](int) { return cap; });
          const double norm = np_pw64(0, nk - bi - 1, [&](int q) { return cc[desc[bi + 1 + q]]; });
          const double scale = clip / norm;
          if (tid == 0) {
            int q = 0;
            for (int i2 = 0; i2 < n; ++i2)
              if (active[i2]) {
                c[i2] = rank[q] <= bi ? cap : cc[q] * scale;
                ++q;
              }
          }
        }
        __syncthreads();
        if (bi < 0) break;
      }
    }

    // ================= Phase D: weighted mean over the chunk ================
    {
      double cs = 0.0;
      if (tid == 0) {
        // np.average's scale: pairwise sum of the (kept) weights in order
        int q = 0;
        for (int i = 0; i < n; ++i)
          if (active[i]) rv[q++] = c[i];
        cs = np_pw64(0, q, [&](int z) { return rv[z]; });
        scal[3] = cs;
      }
      __syncthreads();
      cs = scal[3];
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
  return FilterShared::kUnionBytes + sizeof(double) * (9 * FNP + 5 * LMAX + 8 + 16) + sizeof(int) * (FNP + 16) + 64;
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
