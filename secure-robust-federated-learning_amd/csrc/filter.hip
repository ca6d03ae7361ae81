// k6 — spectral filters: filterL2 and ex_noregret (and, after k5 bucketing,
// mom_filterL2 / mom_ex_noregret).
//
// Replaces src/robust_estimator.py:42-133 (ex_noregret_, ex_noregret) and
// :144-208 (filterL2_, filterL2).  Each layer is cut into itv-wide chunks
// (restarting at every layer, last chunk partial); each chunk is filtered
// independently.  The reference forms the k x k (k <= itv = 1000) fp64
// weighted covariance from N outer products and calls eigh for its top
// eigenpair, 2*int(eps*N) times per chunk.  Here everything after one pass
// over the chunk runs in client space (n x n, n <= 128), in four launches per
// batch of chunks (the n x n Gram of every chunk of the batch lives in the
// caller's workspace between them):
//
//   chunk_gram_kernel   centred chunk Gram G = Z Z^T, Z = X_chunk - column
//                       mean, on the fp64 MFMA (v_mfma_f64_16x16x4_f64), one
//                       256-thread workgroup per chunk; HBM / MFMA bound.
//   noregret_pre_kernel ex_noregret only: Krum pre-filter of the chunk (fp32
//                       distances from G, numpy pairwise score sums, the
//                       ceil(eps*n) largest scores dropped) and the step size
//                       0.5 / max pairwise distance^2 in fp32.
//   wave_solve_kernel   (filter_wave.hip, round 5) the iterations, ONE wave
//                       per chunk, four per CU, C packed in the wave's
//                       registers and LDS and recentred in place; per
//                       iteration with w = c / sum(c), the covariance's
//                       nonzero spectrum is that of M = W^1/2 C W^1/2; top
//                       eigenpair (lambda, u) by Lanczos (plain for filterL2,
//                       partial re-orthogonalisation for ex_noregret) with
//                       checks at predicted convergence points;
//                       tau_j = (C W^1/2 u)_j^2 / lambda; early exit if
//                       lambda^2 <= expansion * sigma^2; filterL2:
//                       c *= 1 - tau/tau_max, drop argmax, c /= |c|_1;
//                       ex_noregret: c *= 1 - step*tau, KL projection onto the
//                       capped simplex.
//   filter_solve_kernel the rare chunk the one-wave solver lists (ghost after
//                       the retries): one 256-thread workgroup per chunk, G in
//                       registers, full re-orthogonalisation.
//   chunk_mean_kernel   mu_j = sum_i c_i x_ij / sum_i c_i in fp64 over the kept
//                       clients in client order (the reference's np.average),
//                       one lane per coordinate; HBM bound.
#include <cstdlib>
#include <type_traits>

#include "filter_common.hpp"
#include "sra_common.hpp"

namespace sra {


// ============================================================================
// chunk_gram_kernel
// ============================================================================
struct GramArgs {
  const float* X;
  int n;
  int64_t d;
  int64_t ldx;
  int itv;
  int64_t chunk0;   // first chunk of the batch
  int nb;           // chunks in the batch
  double* G;        // [nb][FNP][FNP]
  // MoM filters (round 5): bs > 0 -> X holds nsrc clients and row r of the
  // filtered matrix is the mean of clients [r bs, min((r+1) bs, nsrc)),
  // formed in the stage loads with bucket_mean_kernel's arithmetic (np.mean:
  // a sequential fp32 sum / the count) and written to Bout[r][col - chunk0 itv]
  // for the chunk-mean pass -- the separate bucket pass is gone
  int bs;
  int nsrc;
  float* Bout;
  int64_t ldb;
  int vec4;         // 16-byte fills: X, ldx, itv and d (and ldb on the bucket path) multiples of 4 floats
};

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

// wave W's 9 upper tiles (W + 4t) of the 36 16x16 tiles accumulate G over the
// chunk in 64-coordinate stages staged through LDS and centred by the stage's
// column means (fp64); the tile -> row block mapping is compile-time.
template <int W, bool BKT>
__device__ __forceinline__ void gram_tiles(const GramArgs& A, int64_t k0, int k, float* stage, double* smean,
                                           f64x4 (&acc)[9]) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int n = A.n;
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  static_assert(FST == 64, "one stage column per lane");
  const int cc_f = lane, r0_f = tid >> 6;   // the fill: column = lane, rows r0 + 4 i
  for (int s0 = 0; s0 < k; s0 += FST) {
    const int64_t col = k0 + s0 + cc_f;
    const bool cok = s0 + cc_f < k;
    // bucket rows unrolled by eight so that their loads are in flight
    // together (C5: 16.4 -> 12.6 ms)
    if (BKT && A.vec4) {
      // 16-byte loads: thread (rr, c4) forms columns 4 c4 .. + 3 of rows
      // rr + 16 i, every bucket row's float4 loads issued together
      const int c4 = tid & 15, rr = tid >> 4;
      const int64_t colv = k0 + s0 + 4 * c4;
      const int nvalid = k - s0 - 4 * c4;   // columns of this float4 inside the chunk (k % 4 == 0 here)
#pragma unroll 2
      for (int i = 0; i < FNP / 16; ++i) {
        const int r = rr + 16 * i;
        float4 v = {0.f, 0.f, 0.f, 0.f};
        if (r < n && nvalid > 0) {
          const int lo = r * A.bs, hi = lo + A.bs < A.nsrc ? lo + A.bs : A.nsrc;
          float4 acc = {0.f, 0.f, 0.f, 0.f};
          auto add = [&](const float4 x) {
            acc.x += x.x;
            acc.y += x.y;
            acc.z += x.z;
            acc.w += x.w;
          };
          if (hi - lo == 4) {   // a full bucket of four: its loads issued together (C5 Gram 9.67 -> 9.30 ms)
            const float* p = A.X + static_cast<int64_t>(lo) * A.ldx + colv;
            const float4 x0 = *reinterpret_cast<const float4*>(p);
            const float4 x1 = *reinterpret_cast<const float4*>(p + A.ldx);
            const float4 x2 = *reinterpret_cast<const float4*>(p + 2 * A.ldx);
            const float4 x3 = *reinterpret_cast<const float4*>(p + 3 * A.ldx);
            add(x0);
            add(x1);
            add(x2);
            add(x3);
          } else {
#pragma unroll 4
            for (int q = lo; q < hi; ++q) add(*reinterpret_cast<const float4*>(A.X + static_cast<int64_t>(q) * A.ldx + colv));
          }
          const float cnt = static_cast<float>(hi - lo);
          v = float4{acc.x / cnt, acc.y / cnt, acc.z / cnt, acc.w / cnt};
          *reinterpret_cast<float4*>(A.Bout + static_cast<int64_t>(r) * A.ldb + (colv - A.chunk0 * A.itv)) = v;
        }
        *reinterpret_cast<float4*>(stage + r * FROW + 4 * c4) = v;
      }
    } else if (BKT) {
#pragma unroll 8
      for (int i = 0; i < FNP / 4; ++i) {
        const int r = r0_f + 4 * i;
        float v = 0.f;
        if (r < n && cok) {
          const int lo = r * A.bs, hi = lo + A.bs < A.nsrc ? lo + A.bs : A.nsrc;
          float acc = 0.f;
#pragma unroll 4
          for (int q = lo; q < hi; ++q) acc += A.X[static_cast<int64_t>(q) * A.ldx + col];
          v = acc / static_cast<float>(hi - lo);
          A.Bout[static_cast<int64_t>(r) * A.ldb + (col - A.chunk0 * A.itv)] = v;
        }
        stage[r * FROW + cc_f] = v;
      }
    } else if (A.vec4) {
      // plain rows, 16-byte loads: thread (rr, c4) moves columns 4 c4 .. + 3
      // of rows rr + 16 i, the eight loads in flight together
      const int c4 = tid & 15, rr = tid >> 4;
      const bool vok = k - s0 - 4 * c4 > 0;   // k % 4 == 0: a float4 is wholly in or out
      const float* src = A.X + k0 + s0 + 4 * c4;
      float4 v[FNP / 16];
#pragma unroll
      for (int i = 0; i < FNP / 16; ++i) {
        const int r = rr + 16 * i;
        v[i] = (r < n && vok) ? *reinterpret_cast<const float4*>(src + static_cast<int64_t>(r) * A.ldx)
                              : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < FNP / 16; ++i) *reinterpret_cast<float4*>(stage + (rr + 16 * i) * FROW + 4 * c4) = v[i];
    } else {   // (the plain rows: a dynamic loop measured faster, 4.7 vs 7.3 ms at C4)
      for (int e = tid; e < FNP * FST; e += 256) {
        const int r = e / FST, cc = e - (e / FST) * FST;
        stage[r * FROW + cc] = (r < n && s0 + cc < k) ? A.X[static_cast<int64_t>(r) * A.ldx + k0 + s0 + cc] : 0.f;
      }
    }
    __syncthreads();
    {
      // column means: 4 lanes per column, interleaved rows, quad reduction
      const int cc = tid >> 2, part = tid & 3;
      double sm = 0.0;
      for (int r = part; r < n; r += 4) sm += static_cast<double>(stage[r * FROW + cc]);
      sm += dpp_f64<0xB1>(sm);
      sm += dpp_f64<0x4E>(sm);
      if (part == 0) smean[cc] = sm / n;
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
      for (int t = 0; t < 9; ++t)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[ftile_i(W + 4 * t)], fr[ftile_j(W + 4 * t)], acc[t], 0, 0, 0);
    }
    __syncthreads();
  }
}

template <int W>
__device__ __forceinline__ void gram_store(double* G, const f64x4 (&acc)[9]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int I = ftile_i(W + 4 * t), J = ftile_j(W + 4 * t);
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      // f64 16x16x4 C/D layout: col = lane & 15, row = (lane >> 4) + 4 * reg
      const int row = 16 * I + (lane >> 4) + 4 * rg;
      const int col = 16 * J + (lane & 15);
      G[row * FNP + col] = acc[t][rg];
      if (I != J) G[col * FNP + row] = acc[t][rg];
    }
  }
}

// three waves per SIMD (147 VGPRs plain, 168 with the bucket fill): the MoM
// Gram 10.7 -> 9.5 ms at C5; the plain Gram is bound by the fill's loads
// either way (same time at two waves)
template <bool BKT>   // the MoM forms' bucket rows (a separate instantiation: the plain fill's codegen unchanged)
__global__ void __launch_bounds__(256, 3) chunk_gram_kernel(GramArgs A) {
  __shared__ __attribute__((aligned(16))) float stage[FNP * FROW];
  __shared__ double smean[FST];
  const int b = blockIdx.x;
  const int64_t k0 = (A.chunk0 + b) * static_cast<int64_t>(A.itv);
  const int k = static_cast<int>((k0 + A.itv < A.d ? k0 + A.itv : A.d) - k0);
  double* G = A.G + static_cast<size_t>(b) * FNP * FNP;
  f64x4 acc[9];
  switch (threadIdx.x >> 6) {
    case 0: gram_tiles<0, BKT>(A, k0, k, stage, smean, acc); gram_store<0>(G, acc); break;
    case 1: gram_tiles<1, BKT>(A, k0, k, stage, smean, acc); gram_store<1>(G, acc); break;
    case 2: gram_tiles<2, BKT>(A, k0, k, stage, smean, acc); gram_store<2>(G, acc); break;
    default: gram_tiles<3, BKT>(A, k0, k, stage, smean, acc); gram_store<3>(G, acc); break;
  }
}

// ============================================================================
// noregret_pre_kernel: ex_noregret's Krum pre-filter (robust_estimator.py:47-58)
// ============================================================================
struct PreArgs {
  const double* G;
  int* act;        // [nb][FNP] out: kept clients
  double* misc;    // [nb][kMisc] out: [1] step
  int n;
  int nb;
  double eps;
};

__global__ void __launch_bounds__(256) noregret_pre_kernel(PreArgs A) {
  __shared__ float drow[FNP * FNP];   // fp32 distances, rows sorted in place
  __shared__ double diag[FNP];
  __shared__ double score[FNP];
  __shared__ int keep[FNP];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = A.n;
  const int b = blockIdx.x;
  const double* G = A.G + static_cast<size_t>(b) * FNP * FNP;
  const int fp = static_cast<int>(ceil(A.eps * n));
  if (tid < FNP) diag[tid] = G[tid * FNP + tid];
  __syncthreads();
  // krum_'s np.linalg.norm in fp32: sqrt of the centred-Gram squared distance
  for (int e = tid; e < FNP * FNP; e += 256) {
    const int i = e >> 7, j = e & (FNP - 1);
    if (i < n && j < n) {
      const double sq = diag[i] + diag[j] - 2.0 * G[e];
      drow[e] = i == j ? 0.f : static_cast<float>(sqrt(sq > 0.0 ? sq : 0.0));
    }
  }
  __syncthreads();
  // one wave per row: its n-1 off-diagonal distances (+inf padded to 128)
  // sorted by a register bitonic network, 2 elements per lane
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
    __builtin_amdgcn_wave_barrier();
    drow[row * FNP + 2 * lane] = v0;
    drow[row * FNP + 2 * lane + 1] = v1;
  }
  __syncthreads();
  // score = numpy pairwise fp32 sum of the m smallest (Python slice semantics)
  const int m = n - fp - 2 >= 0 ? (n - fp - 2 < n - 1 ? n - fp - 2 : n - 1)
                                : ((n - 1) + (n - fp - 2) > 0 ? (n - 1) + (n - fp - 2) : 0);
  if (tid < n) {
    const float* rw = drow + tid * FNP;
    score[tid] = static_cast<double>(np_pw32(m, [&](int q) { return rw[q]; }));
  }
  __syncthreads();
  // argpartition(metric, -f)[:-f]: drop the fp largest scores (ties: the later
  // index is dropped first; numpy's introselect order on exact ties is not
  // pinned by any fixture)
  if (tid < FNP) {
    int kp = 0;
    if (tid < n) {
      const double si = score[tid];
      int above = 0;
      for (int j = 0; j < n; ++j) above += (score[j] > si || (score[j] == si && j > tid)) ? 1 : 0;
      kp = above >= fp ? 1 : 0;
    }
    keep[tid] = kp;
    A.act[static_cast<size_t>(b) * FNP + tid] = kp;
  }
  __syncthreads();
  // step = 0.5 / max pairwise fp32 distance^2 among the kept clients (fp32
  // arithmetic: numpy 2 keeps the float32 scalar)
  float md = 0.f;
  for (int e = tid; e < FNP * FNP; e += 256) {
    const int i = e >> 7, j = e & (FNP - 1);
    if (i < n && j < n && i < j && keep[i] && keep[j]) {
      const double sq = diag[i] + diag[j] - 2.0 * G[e];
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
  if (tid == 0) {
    float mx = red[0];
    for (int q = 1; q < 4; ++q) mx = red[q] > mx ? red[q] : mx;
    A.misc[static_cast<size_t>(b) * kMisc + 1] = static_cast<double>(0.5f / (mx * mx));
  }
}

// ============================================================================
// filter_solve_kernel
// ============================================================================

constexpr size_t kSolveLds =
    sizeof(double) * (static_cast<size_t>(LMAX) * VST + 2 * XLEN + 64 + 32 + 4 * TRI + 4 * FNP) +
    sizeof(int) * (3 * FNP + 16);
static_assert(2 * kSolveLds <= 163840, "two solver workgroups must fit one CU's LDS");

// Top eigenpair of the Lanczos tridiagonal T_m (alpha in trw[0, m), beta^2 in
// trw[64, 64 + m - 1)), evaluated identically by every wave of the block:
// multisection on Sturm counts (the division-free recurrence of the leading
// principal minors, rescaled every 4 steps; the previous check's Ritz value
// theta_lb is a lower bound by interlacing, so the first round's points are
// geometric above it), then the eigenvector from a twisted factorisation of
// T - lambda I (forward and backward pivots in one wave-uniform loop held in
// registers, the twist is the smallest |gamma|).  The normalised eigenvector goes to
// trw[128, 128 + m); returns lambda and its last component.  Kept out of line:
// it runs a few times per filter iteration and its registers would otherwise
// compete with the 64 Gram values per lane of the solver's hot loop.
__device__ __attribute__((noinline)) void tri_top(double* trw, int m, double tscale, double theta_lb, double* lam_out,
                                                  double* zlast_out) {
  m = __builtin_amdgcn_readfirstlane(m);   // wave-uniform: scalar loop control
  const int lane = threadIdx.x & 63;
  const double al = lane < m ? trw[lane] : 0.0;
  const double b2l = lane + 1 < m ? trw[64 + lane] : 0.0;
  const double bl = lane + 1 < m ? sqrt(trw[64 + lane]) : 0.0;
  const double bp = (lane >= 1 && lane < m) ? sqrt(trw[64 + lane - 1]) : 0.0;
  const double rad = fabs(bp) + fabs(bl);
  double lo = wave_min(lane < m ? al - rad : 1e300);
  double hi = wave_max(lane < m ? al + rad : -1e300);
  // multisection on Sturm counts: the division-free recurrence of the
  // leading principal minors, rescaled by powers of two every 4
  // steps; the previous check's Ritz value is a lower bound
  // (interlacing), so the first round's points are geometric above it
  // T_00 = alpha_0 is a lower bound too (the start vector's Rayleigh quotient;
  // after a restart, the previous Ritz value)
  theta_lb = fmax(theta_lb, readlane_f64(al, 0));
  const bool geo = theta_lb > lo && theta_lb < hi;
  if (geo) lo = theta_lb;
  constexpr double kInv65 = 1.0 / 65.0;
  for (int round = 0; round < 16; ++round) {
    const double fr = (geo && round == 0) ? __builtin_amdgcn_ldexp(1.0, lane - 63) : (lane + 1) * kInv65;
    const double x = lo + (hi - lo) * fr;
    double p2 = 1.0;
    double p1 = readlane_f64(al, 0) - x;
    int cntb = __builtin_signbit(p1) ? 1 : 0;
    // one step: only the fma depends on the previous step (beta^2 * p2 uses
    // the value of two steps back); alpha / beta^2 broadcast from registers
    auto step = [&](int q) __attribute__((always_inline)) {
      const double pk = fma(readlane_f64(al, q) - x, p1, -(readlane_f64(b2l, q - 1) * p2));
      cntb += (__builtin_signbit(pk) ? 1 : 0) != (__builtin_signbit(p1) ? 1 : 0);
      p2 = p1;
      p1 = pk;
    };
    int q = 1;
    for (; q + 4 <= m; q += 4) {   // unrolled by hand: the rescale runs once per 4 steps
      step(q);
      step(q + 1);
      step(q + 2);
      step(q + 3);
      const int e = __builtin_amdgcn_frexp_exp(p1);
      p1 = __builtin_amdgcn_ldexp(p1, -e);
      p2 = __builtin_amdgcn_ldexp(p2, -e);
    }
    for (; q < m; ++q) step(q);
    const unsigned long long ok = __builtin_amdgcn_ballot_w64(cntb >= m);
    const int first = ok ? __builtin_ctzll(ok) : 64;
    const double flo = first == 0 ? 0.0
                                  : ((geo && round == 0) ? __builtin_amdgcn_ldexp(1.0, first - 64)
                                                         : first * kInv65);
    const double fhi = (geo && round == 0) ? __builtin_amdgcn_ldexp(1.0, first - 63) : (first + 1) * kInv65;
    const double nlo = lo + (hi - lo) * flo;
    const double nhi = first < 64 ? lo + (hi - lo) * fhi : hi;
    const bool stalled = nlo == lo && nhi == hi;   // a bracket of a few ulps no longer splits
    lo = nlo;
    hi = nhi;
    // two ulps: one ulp is up to 2.2e-16 relative, so a 2e-16 test could
    // never pass just above a power of two and every check ran all 16 rounds
    if (stalled || hi - lo <= 4.5e-16 * fmax(fabs(lo), fabs(hi))) break;
  }
  const double lm = 0.5 * (lo + hi);
  // eigenvector of T - lm I by a twisted factorisation.  The forward pivots
  // dp_q (q = k) and the backward pivots dm_q (q = m - 1 - k) run in one
  // wave-uniform serial loop on alpha / beta^2 broadcast from registers; lane
  // q keeps dp_q and dm_q (no LDS round trip on the chain); the twist is the
  // smallest |gamma|
  const double tiny = 1e-300 + 1e-30 * tscale;
  double dpl = 0.0, dml = 0.0;
  {
    double pf = 0.0, pb = 0.0;
    for (int k = 0; k < m; ++k) {
      const int qf = k, qb = m - 1 - k;
      double vf = readlane_f64(al, qf) - lm;
      double vb = readlane_f64(al, qb) - lm;
      if (k > 0) {
        vf -= fdiv(readlane_f64(b2l, qf - 1), pf);
        vb -= fdiv(readlane_f64(b2l, qb), pb);
      }
      if (fabs(vf) < tiny) vf = -tiny;
      if (fabs(vb) < tiny) vb = -tiny;
      pf = vf;
      pb = vb;
      dpl = lane == qf ? vf : dpl;
      dml = lane == qb ? vb : dml;
    }
  }
  // the shuffle runs with every lane active (a disabled source lane reads 0)
  const double dmx = __shfl_down(dml, 1);
  const double dmn = lane + 1 < m ? dmx : 1.0;
  double gam = lane < m ? fabs(dpl + dml - (al - lm)) : 1e308;
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
  // z_tw = 1; z_q = -(b_q / dp_q) z_{q+1} below the twist,
  // z_{q+1} = -(b_q / dm_{q+1}) z_q above it: ratios per lane, then both
  // walks in one wave-uniform loop (lane q keeps z_q)
  const double rat = lane < tw ? -bl / dpl : (lane + 1 < m ? -bl / dmn : 0.0);
  double zv = lane == tw ? 1.0 : 0.0;
  {
    double zd = 1.0, zu = 1.0;
    const int sd = tw, su = m - 1 - tw;
    const int steps = sd > su ? sd : su;
    for (int k = 0; k < steps; ++k) {
      if (k < sd) {
        const int q = tw - 1 - k;
        zd *= readlane_f64(rat, q);
        if (fabs(zd) > 1e150) zd = copysign(1e150, zd);   // z_tw = 1 is the largest in exact arithmetic
        zv = lane == q ? zd : zv;
      }
      if (k < su) {
        const int q = tw + k;
        zu *= readlane_f64(rat, q);
        if (fabs(zu) > 1e150) zu = copysign(1e150, zu);
        zv = lane == q + 1 ? zu : zv;
      }
    }
  }
  const double amax = wave_max(fabs(zv));
  const double zs = zv / amax;
  zv = zs / sqrt(wave_sum(zs * zs));
  if (lane < m) trw[128 + lane] = zv;
  __builtin_amdgcn_wave_barrier();
  *lam_out = lm;
  *zlast_out = readlane_f64(zv, m - 1);
}

// ex_noregret's projection (robust_estimator.py:77-99) onto {sum c = 1,
// c <= cap} over the nk kept clients: candidate i caps the i+1 largest weights
// and rescales the rest; the feasible candidate with the smallest
// KL(c || c_) = sum_{q<=i} c_q log(c_q / cap) - log(scale) * sum_{q>i} c_q wins
// (first on ties); the reference's loop stops at the first infeasible clip.
// Once per filter iteration, so it is kept out of line: the solver's 64 Gram
// registers per lane stay put while this runs.  Returns false when no
// candidate is feasible.  Block-wide (all 256 lanes), barriers inside.
// NP: row capacity of the scratch, NW: waves of the block (needs red[NW],
// ibuf[3 NP + 2 NW], vscr[3 NP]).
template <int NP, int NW>
__device__ __attribute__((noinline)) bool kl_project_t(double* ci_io, bool ai, int row, bool own, int nk, double cap,
                                                       double* cvec, double* vscr, int* ibuf, double* red,
                                                       double* hbuf, int* capped) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int* kidx = ibuf;            // compact -> client row
  int* irank = ibuf + NP;      // descending rank of a compact entry
  int* flag = ibuf + 2 * NP;   // active flags
  int* islot = ibuf + 3 * NP;  // argmax indices
  double* cc = vscr;           // compact weights
  double* sv = vscr + NP;      // weights in descending order
  double* hl = vscr + 2 * NP;  // sv * log(sv / cap)
  const double ci = *ci_io;
  if (own) flag[row] = ai ? 1 : 0;
  __syncthreads();
  if (own && ai) {
    int pos = 0;
    for (int q2 = 0; q2 < row; ++q2) pos += flag[q2];
    kidx[pos] = row;
    cc[pos] = ci;
  }
  __syncthreads();
  // descending rank; ties: later compact index first (flip of a stable ascending argsort)
  if (tid < nk) {
    const double v = cc[tid];
    int rk = 0;
    for (int q2 = 0; q2 < nk; ++q2) rk += (cc[q2] > v || (cc[q2] == v && q2 > tid)) ? 1 : 0;
    irank[tid] = rk;
    sv[rk] = v;
    hl[rk] = v * log(v / cap);
  }
  __syncthreads();
  double negkl = -__builtin_inf(), scale = 0.0;
  int stop = 1 << 30;
  if (tid < nk) {
    const int i = tid;
    auto pw = [&](int lo, int cnt, auto&& g) -> double {
      if constexpr (NP > 512) return np_pw64_rec<4>(lo, cnt, g);
      else return np_pw64(lo, cnt, g);
    };
    const double clip = 1.0 - pw(0, i + 1, [&](int) { return cap; });
    if (clip <= 0.0) {
      stop = i;
    } else if (i + 1 < nk) {
      const double norm = pw(i + 1, nk - i - 1, [&](int q2) { return sv[q2]; });
      scale = clip / norm;
      if (!(sv[i + 1] * scale > cap)) {
        double head = 0.0;
        for (int q2 = 0; q2 <= i; ++q2) head += hl[q2];
        negkl = -(head - norm * log(scale));
      }
    }
  }
  // first infeasible clip (block min of stop), then the first best candidate before it
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int o2 = __shfl_xor(stop, off);
    stop = o2 < stop ? o2 : stop;
  }
  if (lane == 0) islot[wave] = stop;
  __syncthreads();
  int istop = islot[0];
  for (int q2 = 1; q2 < NW; ++q2) istop = islot[q2] < istop ? islot[q2] : istop;
  if (tid >= istop) negkl = -__builtin_inf();
  double v = negkl;
  int bi = tid;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ov = __shfl_xor(v, off);
    const int oi = __shfl_xor(bi, off);
    if (ov > v || (ov == v && oi < bi)) {
      v = ov;
      bi = oi;
    }
  }
  if (lane == 0) {
    red[wave] = v;
    islot[NW + wave] = bi;
  }
  __syncthreads();
  double bv = red[0];
  bi = islot[NW];
  for (int q2 = 1; q2 < NW; ++q2)
    if (red[q2] > bv || (red[q2] == bv && islot[NW + q2] < bi)) {
      bv = red[q2];
      bi = islot[NW + q2];
    }
  const bool ok = bv > -__builtin_inf();
  *capped = ok ? bi + 1 : 0;
  if (ok && tid == bi) hbuf[0] = scale;
  __syncthreads();
  if (ok && tid < nk) cvec[kidx[tid]] = irank[tid] <= bi ? cap : cc[tid] * hbuf[0];
  __syncthreads();
  if (ok && ai) *ci_io = cvec[row];
  return ok;
}
__device__ __forceinline__ bool kl_project(double* ci_io, bool ai, int row, bool own, int nk, double cap, double* cvec,
                                           double* vscr, int* ibuf, double* red, double* hbuf, int* capped) {
  return kl_project_t<FNP, 4>(ci_io, ai, row, own, nk, cap, cvec, vscr, ibuf, red, hbuf, capped);
}

// MODE 0: filterL2, 1: ex_noregret; DBG: diagnostics of chunk 0.  Since round
// 2 this re-orthogonalising solver is the fallback: it runs only the chunks
// that wave_solve_kernel listed in A.fb_list (A.fb_count on the device).
template <int MODE, bool DBG>
__global__ void __launch_bounds__(256, 2) filter_solve_kernel(SolveArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* V = reinterpret_cast<double*>(smem);   // [LMAX][VST] Lanczos basis
  double* xbuf = V + LMAX * VST;                 // [XLEN] operator input
  double* rbuf = xbuf + XLEN;                    // [XLEN] residual before re-orthogonalisation
  double* hbuf = rbuf + XLEN;                    // [64] Gram-Schmidt coefficients (+ |r'|^2)
  double* red = hbuf + 64;                       // [2][16] block reductions (parity slots)
  double* tri = red + 32;                        // [4][TRI] per-wave tridiagonal record
  double* cvec = tri + 4 * TRI;                  // [FNP] weights (projection / final scale)
  double* vscr = cvec + FNP;                     // [3][FNP] projection scratch
  int* ibuf = reinterpret_cast<int*>(vscr + 3 * FNP);   // [3][FNP] int scratch + [16] argmax slots

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int row = tid >> 1;   // client row of this lane pair
  const int half = tid & 1;   // which 64 columns of the row
  const bool own = half == 0; // the even lane speaks for the pair
  const int n = A.n;
  double* trw = tri + wave * TRI;   // this wave's copy: alpha [0,64), beta^2 [64,128), s [128,192), scratch [192,256)
  const int xi = row < 64 ? row : XOFF + row - 64;   // this row's slot in xbuf / rbuf

  int rslot = 0;
  // block sum of up to 4 owner contributions with one barrier (parity slots:
  // a slot's reads happen before the barrier of the next reduction)
  auto reduce4 = [&](double v0, double v1, double v2, double v3, double (&o)[4], int nv) __attribute__((always_inline)) {
    // nv: how many of the four values are live (wave-uniform)
    v0 = wave_sum(v0);
    if (nv > 1) v1 = wave_sum(v1);
    if (nv > 2) v2 = wave_sum(v2);
    if (nv > 3) v3 = wave_sum(v3);
    double* R = red + 16 * rslot;
    if (lane == 0) {
      R[4 * wave + 0] = v0;
      if (nv > 1) R[4 * wave + 1] = v1;
      if (nv > 2) R[4 * wave + 2] = v2;
      if (nv > 3) R[4 * wave + 3] = v3;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nv) o[k] = (R[k] + R[4 + k]) + (R[8 + k] + R[12 + k]);
    rslot ^= 1;
  };
  // first index of the largest v over the block (-inf for no candidate); one barrier
  auto argmax_first = [&](double v, int i, double* vbest) __attribute__((always_inline)) -> int {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ov = __shfl_xor(v, off);
      const int oi = __shfl_xor(i, off);
      if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
      }
    }
    double* R = red + 16 * rslot;
    int* I = ibuf + 3 * FNP + 8 * rslot;
    if (lane == 0) {
      R[wave] = v;
      I[wave] = i;
    }
    __syncthreads();
    double bv = R[0];
    int bi = I[0];
    for (int q = 1; q < 4; ++q)
      if (R[q] > bv || (R[q] == bv && I[q] < bi)) {
        bv = R[q];
        bi = I[q];
      }
    rslot ^= 1;
    *vbest = bv;
    return bi;
  };

  const int nlisted = *A.fb_count;
  for (int li = blockIdx.x; li < nlisted; li += gridDim.x) {
    const int ch = A.fb_list[li];
    // ---- G rows into registers: lane pair (row, half) holds G[row][64 half + c]
    double g[64];
    {
      const double2* Gr = reinterpret_cast<const double2*>(A.G + static_cast<size_t>(ch) * FNP * FNP + row * FNP +
                                                           64 * half);
#pragma unroll
      for (int c = 0; c < 32; ++c) {
        const double2 v = Gr[c];
        g[2 * c] = v.x;
        g[2 * c + 1] = v.y;
      }
    }
    // y = G x for x in xbuf; both lanes of the pair get the row value
    auto gmv = [&]() __attribute__((always_inline)) -> double {
      const double2* xh = reinterpret_cast<const double2*>(xbuf + XOFF * half);
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
      for (int c = 0; c < 32; c += 2) {
        const double2 a = xh[c], b = xh[c + 1];
        p0 = fma(g[2 * c], a.x, p0);
        p1 = fma(g[2 * c + 1], a.y, p1);
        p2 = fma(g[2 * c + 2], b.x, p2);
        p3 = fma(g[2 * c + 3], b.y, p3);
        // at most 8 x pieces in flight: the compiler would otherwise hoist all
        // 32 loads (128 VGPRs beside the 128 of G) and spill
        if ((c & 6) == 6) asm volatile("" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)::"memory");
      }
      const double p = (p0 + p1) + (p2 + p3);
      return p + dpp_f64<0xB1>(p);
    };

    const bool dbg = DBG && ch == 0;
    bool ai;     // this row is an active client
    if constexpr (MODE == 1) ai = A.act[static_cast<size_t>(ch) * FNP + row] != 0;
    else ai = row < n;
    double ci = ai ? 1.0 : 0.0;
    const int fdrop = static_cast<int>(ceil(A.eps * n));
    const int n_keep = MODE == 1 ? n - (fdrop < n ? fdrop : n) : n;
    const double step = MODE == 1 ? A.misc[static_cast<size_t>(ch) * kMisc + 1] : 0.0;
    const int iters = MODE == 0 ? 2 * static_cast<int>(A.eps * n) : static_cast<int>(2 * A.eps * n_keep);
    double ui = 0.0;          // Ritz vector (warm start of the next iteration)
    bool have_u = false;
    int m_hint = 12;          // Lanczos steps the previous iteration needed
    double rate_hint = 0.0;   // last measured log-decay of the Ritz residual per step (0: none yet)
    int done = 0;             // filter iterations completed (decision trace)
    int* tr = A.trace != nullptr ? A.trace + static_cast<size_t>(ch) * kTraceStride : nullptr;
    // ex_noregret: projected_c is None (no feasible candidate, :99): the next
    // iteration runs with weights=None -- the plain mean and covariance
    // (:65-67) -- and either exits with that mean (:71-72) or fails at
    // c * (1 - step * tau) (:75, TypeError); at the last iteration the final
    // np.average(weights=None) returns it (:101).  unweighted: the chunk's
    // result is the plain fp32 mean of the kept clients.
    bool none = false, unweighted = false;

    for (int it = 0; it < iters; ++it) {
      const long long t_it = dbg ? clock64() : 0;
      if (MODE == 1 && none) ci = ai ? 1.0 : 0.0;
      // ---- weights, g = G w, s = w^T G w, active count
      double o[4];
      reduce4(own && ai ? ci : 0.0, own && ai ? 1.0 : 0.0, 0.0, 0.0, o, 2);
      const double csum = o[0];
      const int nact = static_cast<int>(o[1]);
      const double wi = ai ? ci / csum : 0.0;
      const double swi = sqrt(wi > 0.0 ? wi : 0.0);
      if (own) xbuf[xi] = wi;
      __syncthreads();
      const double gwi = gmv();
      reduce4(own ? wi * gwi : 0.0, 0.0, 0.0, 0.0, o, 1);
      const double sgw = o[0];

      // ---- top eigenpair of M = W^1/2 C W^1/2: Lanczos with full re-orthogonalisation
      double lam = 0.0, resid = 0.0;
      int m_conv = 0, nchecks = 0, restarts = 0, passes2 = 0;
      long long tph[4] = {0, 0, 0, 0};   // cycle probes (diagnostics only): check, matvec+alpha, dots, update
      long long tq = 0;
      double rt;   // unnormalised next basis vector (this row's entry)
      {
        // warm start from the previous Ritz vector (perturbed), else sqrt-weights
        // times a fixed non-uniform pattern (sqrt-weights alone span M's null
        // vector: M W^1/2 1 = W^1/2 C w = 0)
        const double hh = 0.5 + (row * 0.6180339887498949 - floor(row * 0.6180339887498949));
        rt = swi > 0.0 ? (have_u ? ui + 1e-3 * swi * hh : swi * hh) : 0.0;
      }
      for (;;) {   // explicit restarts from the Ritz vector when the basis is full
        double xt = swi * rt;
        if (own) xbuf[xi] = xt;
        reduce4(own ? rt * rt : 0.0, own ? xt : 0.0, own ? gwi * xt : 0.0, 0.0, o, 3);
        double nrm2 = o[0], S1 = o[1], GY = o[2];
        double qprev = 0.0, tscale = 0.0, theta_lb = -1e300;
        int next_check = m_hint - 1 > 4 ? m_hint - 1 : 4;
        int m_a = -1;
        double res_a = 0.0;
        bool converged = false;
        for (int j = 0;; ++j) {
          const double bet = sqrt(nrm2);   // beta_{j-1} (the start norm at j = 0)
          if (dbg) tq = clock64();
          if (j > 0) {
            if (lane == 0) trw[64 + j - 1] = bet * bet;
            tscale = fmax(tscale, bet);
            const bool breakdown = !(bet > 1e-14 * tscale);
            if (breakdown || j >= nact || j == LMAX || j >= next_check) {
              // ---- top eigenpair of T_j, identically in every wave
              const int m = j;
              ++nchecks;
              __builtin_amdgcn_wave_barrier();
              double lm, zlast;
              tri_top(trw, m, tscale, theta_lb, &lm, &zlast);
              lam = lm;
              resid = fabs(bet * zlast);
              theta_lb = lm;
              if (resid <= kResTol * fabs(lm) || breakdown || j >= nact) {
                converged = true;
                m_conv = m;
                break;
              }
              if (j == LMAX) break;   // restart from the Ritz vector
              // next check: extrapolate the residual's geometric decay (this
              // cycle's two last checks, else the last rate measured); a check
              // costs about two Lanczos steps, so no cap short of the basis size
              int adv = 4;
              double rate = rate_hint;
              if (m_a >= 0 && res_a > resid && resid > 0.0) rate = rate_hint = log(resid / res_a) / (m - m_a);
              if (rate < 0.0 && resid > 0.0) {
                const double need = log(kResTol * fabs(lm) / resid) / rate;
                adv = need < 1.0 ? 1 : (need > LMAX ? LMAX : static_cast<int>(ceil(need)));
              }
              m_a = m;
              res_a = resid;
              next_check = m + adv;
            }
          }
          if (dbg) { const long long t = clock64(); tph[0] += t - tq; tq = t; }
          // ---- (1) y = G x~, M q_j = W^1/2 C x~ / beta, r' = M q_j - beta q_{j-1},
          // alpha_j = q_j^T M q_j = x~^T C x~ / beta^2 (one block sum)
          const double y = gmv();
          const double cx = y - gwi * S1 - GY + sgw * S1;
          const double ib = 1.0 / bet;
          const double q = rt * ib;
          if (own) V[j * VST + row] = q;
          const double rp = swi * cx * ib - (j > 0 ? bet * qprev : 0.0);
          if (own) rbuf[xi] = rp;
          qprev = q;
          reduce4(own ? swi * rt * y : 0.0, 0.0, 0.0, 0.0, o, 1);
          const double aj = (o[0] - 2.0 * S1 * GY + sgw * S1 * S1) * (ib * ib);
          // r'' = r' - alpha_j q_j before the re-orthogonalisation: without it the
          // coefficients carry alpha_j and one classical pass loses ~3x of
          // orthogonality per step (|r''| << |r'|)
          double r = rp - aj * q;
          double alpha = aj;
          if (dbg) { const long long t = clock64(); tph[1] += t - tq; tq = t; }
#pragma unroll 1
          for (int pass = 0; pass < 2; ++pass) {
            // ---- (2) coefficients h_q = q_q . r (q <= j) and |r|^2 (first pass):
            // 4 lanes per basis vector, 16-byte pieces interleaved; the first
            // pass subtracts alpha_j q_j from r' on the fly
            {
              const int qq = tid >> 2, part = tid & 3;
              const int top = pass == 0 ? j + 1 : j;
              const double asub = pass == 0 ? aj : 0.0;
              if (qq <= top) {
                const bool isv = qq <= j;
                const double* vb = V + (isv ? qq : 0) * VST;
                const double* vj = V + j * VST;
                double h0 = 0.0, h1 = 0.0;
#pragma unroll
                for (int e = 0; e < 16; e += 2) {
                  const int i0 = 2 * (part + 4 * e), i1 = 2 * (part + 4 * (e + 1));
                  const int r0 = i0 < 64 ? i0 : XOFF + i0 - 64, r1 = i1 < 64 ? i1 : XOFF + i1 - 64;
                  const double2 b0 = *reinterpret_cast<const double2*>(rbuf + r0);
                  const double2 c0 = *reinterpret_cast<const double2*>(vj + i0);
                  const double2 b1 = *reinterpret_cast<const double2*>(rbuf + r1);
                  const double2 c1 = *reinterpret_cast<const double2*>(vj + i1);
                  const double s0x = fma(-asub, c0.x, b0.x), s0y = fma(-asub, c0.y, b0.y);
                  const double s1x = fma(-asub, c1.x, b1.x), s1y = fma(-asub, c1.y, b1.y);
                  double2 a0, a1;
                  if (isv) {
                    a0 = *reinterpret_cast<const double2*>(vb + i0);
                    a1 = *reinterpret_cast<const double2*>(vb + i1);
                  } else {
                    a0 = double2{s0x, s0y};
                    a1 = double2{s1x, s1y};
                  }
                  h0 = fma(a0.x, s0x, fma(a0.y, s0y, h0));
                  h1 = fma(a1.x, s1x, fma(a1.y, s1y, h1));
                  if ((e & 2) == 2) asm volatile("" : "+v"(h0), "+v"(h1)::"memory");
                }
                double h = h0 + h1;
                h += dpp_f64<0xB1>(h);
                h += dpp_f64<0x4E>(h);
                if (part == 0) hbuf[qq] = h;
              }
            }
            __syncthreads();
            if (dbg) { const long long t = clock64(); tph[2] += t - tq; tq = t; }
            // ---- (3) r -= sum_q h_q q_q: the lane pair splits q = 0..j into two
            // contiguous halves, 4 coefficients per batch (loads issued together)
            double hn2 = 0.0, upd = 0.0;
            {
              const int nq = j + 1, hq0 = (nq + 1) >> 1;
              const int qlo = half ? hq0 : 0, qhi = half ? nq : hq0;
              double u[4] = {0.0, 0.0, 0.0, 0.0}, e2[4] = {0.0, 0.0, 0.0, 0.0};
              int qq = qlo;
              for (; qq + 4 <= qhi; qq += 4) {
                double hv[4], vv[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                  hv[t] = hbuf[qq + t];
                  vv[t] = V[(qq + t) * VST + row];
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                  u[t] = fma(hv[t], vv[t], u[t]);
                  e2[t] = fma(hv[t], hv[t], e2[t]);
                }
              }
              for (; qq < qhi; ++qq) {
                const double hv = hbuf[qq];
                u[0] = fma(hv, V[qq * VST + row], u[0]);
                e2[0] = fma(hv, hv, e2[0]);
              }
              upd = (u[0] + u[1]) + (u[2] + u[3]);
              hn2 = (e2[0] + e2[1]) + (e2[2] + e2[3]);
              upd += dpp_f64<0xB1>(upd);
              hn2 += dpp_f64<0xB1>(hn2);
            }
            r -= upd;
            alpha += hbuf[j];
            if (pass == 1) break;
            const double rr2 = hbuf[j + 1];
            if (!(rr2 - hn2 < kDgks * rr2)) break;
            // heavy cancellation: one more classical Gram-Schmidt pass
            ++passes2;
            if (own) rbuf[xi] = r;
            __syncthreads();
          }
          if (lane == 0) trw[j] = alpha;
          tscale = fmax(tscale, fabs(alpha));
          // ---- (4) next unnormalised vector and its sums (deferred normalisation)
          rt = r;
          xt = swi * r;
          if (own) xbuf[xi] = xt;
          reduce4(own ? r * r : 0.0, own ? xt : 0.0, own ? gwi * xt : 0.0, 0.0, o, 3);
          nrm2 = o[0];
          S1 = o[1];
          GY = o[2];
          if (dbg) { const long long t = clock64(); tph[3] += t - tq; tq = t; }
        }
        // ---- Ritz vector u = V s
        {
          const int m = converged ? m_conv : LMAX;
          double u0 = 0.0, u1 = 0.0;
          int qq = 0;
          for (; qq + 1 < m; qq += 2) {
            u0 = fma(trw[128 + qq], V[qq * VST + row], u0);
            u1 = fma(trw[128 + qq + 1], V[(qq + 1) * VST + row], u1);
          }
          if (qq < m) u0 = fma(trw[128 + qq], V[qq * VST + row], u0);
          ui = u0 + u1;
        }
        if (converged || restarts == kMaxRestarts) break;
        ++restarts;
        rt = ui;
        __syncthreads();   // every wave's reads of V before the restart overwrites it
      }
      m_hint = m_conv > 4 ? m_conv : 4;
      have_u = true;
      if (dbg && it < 256) {
        double* rec = A.dbg + FNP * FNP + static_cast<int64_t>(it) * kDbgRec;
        if (own) rec[row] = ci;
        if (tid == 0) {
          rec[FNP] = lam;
          rec[FNP + 1] = m_conv;
          rec[FNP + 2] = resid;
          rec[FNP + 3] = nchecks;
          rec[FNP + 4] = nact;
          rec[FNP + 5] = sgw;
          rec[FNP + 6] = restarts;
          rec[FNP + 7] = passes2;
          rec[FNP + 8] = static_cast<double>(clock64() - t_it);
          for (int k = 0; k < 4; ++k) rec[FNP + 9 + k] = static_cast<double>(tph[k]);
        }
      }
      // ---- early exit (robust_estimator.py:163-164 / :71-72)
      if (lam * lam <= A.expansion * A.sigma * A.sigma) {
        unweighted = none;
        break;
      }
      if (MODE == 1 && none) {
        if (tid == 0) *A.status = 2;   // c * (1 - step * tau) with c None: TypeError (:75)
        break;
      }
      // ---- tau_j = ((x_j - mu).v)^2 = (C W^1/2 u)_j^2 / lambda
      {
        const double xt = swi * ui;
        if (own) xbuf[xi] = xt;
        reduce4(own ? xt : 0.0, own ? gwi * xt : 0.0, 0.0, 0.0, o, 2);
      }
      const double cu = gmv() - gwi * o[0] - o[1] + sgw * o[0];
      const double ti = cu * cu / lam;
      if constexpr (MODE == 0) {
        // c *= 1 - tau/tau_max; drop the argmax (first index); c /= |c|_1
        double tmax = 0.0;
        const int p = argmax_first(own && ai ? ti : -__builtin_inf(), row, &tmax);
        const double cn = (ai && row != p) ? ci * (1.0 - ti / tmax) : 0.0;
        reduce4(own ? fabs(cn) : 0.0, 0.0, 0.0, 0.0, o, 1);
        ci = cn / o[0];
        if (row == p) ai = false;
        if (tr != nullptr && tid == 0) tr[1 + it] = p;
      } else {
        // c *= 1 - step*tau, then the KL projection onto {sum c = 1, c <= cap}
        // (robust_estimator.py:74-99) over the n_keep kept clients
        const int nk = n_keep;
        const double cap = 1.0 / (1.0 - A.eps) / nk;
        if (ai) ci = ci * (1.0 - step * ti);
        int capped = 0;
        if (!kl_project(&ci, ai, row, own, nk, cap, cvec, vscr, ibuf, red, hbuf, &capped)) {
          none = true;   // projected_c = None (:99)
          unweighted = it + 1 == iters;
          if (unweighted && ai) ci = 1.0;
        }
        if (tr != nullptr && tid == 0) tr[1 + it] = capped;
      }
      done = it + 1;
    }
    if (tr != nullptr) {
      if (tid == 0) tr[0] = done;
      if (own) tr[1 + FNP + row] = ai ? 1 : 0;
    }

    // ---- final weights and np.average's scale (pairwise sum of the kept weights in order)
    __syncthreads();
    if (own) {
      cvec[row] = ai ? ci : 0.0;
      ibuf[2 * FNP + row] = ai ? 1 : 0;
      A.c[static_cast<size_t>(ch) * FNP + row] = ai ? ci : 0.0;
      A.act[static_cast<size_t>(ch) * FNP + row] = ai ? 1 : 0;
    }
    __syncthreads();
    if (tid == 0) {
      int q2 = 0;
      double* kept = vscr;
      for (int i = 0; i < n; ++i)
        if (ibuf[2 * FNP + i]) kept[q2++] = cvec[i];
      A.misc[static_cast<size_t>(ch) * kMisc] = np_pw64(0, q2, [&](int z) { return kept[z]; });
      A.misc[static_cast<size_t>(ch) * kMisc + 2] = unweighted ? 1.0 : 0.0;
      if (unweighted) atomicAdd(A.status + 1, 1);
    }
    __syncthreads();
  }
}

// (round 5: the four-wave lanczos_solve_kernel with its block_check /
// fast_check checks was replaced by wave_solve_kernel, filter_wave.hip;
// DESIGN.md k6 keeps its measurements)

// ============================================================================
// chunk_mean_kernel: the weighted mean of every coordinate of the batch
// ============================================================================
__global__ void __launch_bounds__(256) chunk_mean_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                         int64_t jx0, int itv, int64_t chunk0, int nb,
                                                         const double* __restrict__ c, const int* __restrict__ act,
                                                         const double* __restrict__ misc, double* __restrict__ out,
                                                         int cs, int unw) {
  const int64_t j0 = chunk0 * itv;
  const int64_t jend = (chunk0 + nb) * static_cast<int64_t>(itv);
  const int64_t j1 = jend < d ? jend : d;
  const int64_t j = j0 + static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (j >= j1) return;
  const int b = static_cast<int>((j - j0) / itv);
  if (cs == FNP && misc[static_cast<size_t>(b) * kMisc + 3] != 0.0) return;   // written by wave_solve_kernel
  const double* cb = c + static_cast<size_t>(b) * cs;
  const int* ab = act + static_cast<size_t>(b) * cs;
  if (unw && misc[static_cast<size_t>(b) * kMisc + 2] != 0.0) {
    // ex_noregret's np.average(samples, weights=None) of fp32 samples: the
    // sequential fp32 sum over the kept clients / their count, in fp32.
    // Deviation: the sum runs in client-index order; the reference's kept
    // list is in np.argpartition's order (robust_estimator.py:49-50, an
    // introselect detail of numpy), so the two fp32 sums can differ in the
    // last ulps (the unweighted outcome itself only exists in the fp32
    // window of tests/golden/gen_none_sides.py; the tests bound it by tolerance)
    float s32 = 0.f;
    int cnt = 0;
    for (int i = 0; i < n; ++i)
      if (ab[i]) {
        s32 += X[static_cast<int64_t>(i) * ldx + (j - jx0)];
        ++cnt;
      }
    out[j] = static_cast<double>(s32 / static_cast<float>(cnt));
    return;
  }
  double s = 0.0;
  for (int i = 0; i < n; ++i)
    if (ab[i]) s += static_cast<double>(X[static_cast<int64_t>(i) * ldx + (j - jx0)]) * cb[i];
  out[j] = s / misc[static_cast<size_t>(b) * kMisc];
}

// ============================================================================
// N in (128, NBIG]: the same filters with the client-space objects out of
// registers (the reference has no client limit, robust_estimator.py:42-218).
//   chunk_colmean_kernel + chunk_gram_big_kernel: the centred chunk Gram on the
//     fp64 MFMA in 64 x 64 output blocks (each block stages its two row blocks
//     through LDS and centres them by the chunk's fp64 column means);
//   noregret_pre_big_kernel: ex_noregret's Krum pre-filter, one wave per
//     distance row, the row bitonic-sorted in the wave's LDS slice;
//   filter_big_kernel<MODE>: filter_solve_kernel's re-orthogonalising Lanczos
//     with G read from global memory (column i of the symmetric G: coalesced),
//     the basis in a per-workgroup global slot (each entry read back only by
//     the thread that wrote it), 1024 threads = two per client row (the two
//     halves of every matvec).
// A correctness path: the BASELINE configurations all have N <= 128 per
// filter (C5 filters 128 bucket means).
// ============================================================================
constexpr int NBIG = 512;
constexpr int NBIG2 = 1024;        // N in (512, 1024]: one thread per row (filter_big_kernel<MODE, NBIG2>)
constexpr int kBigThreads = 1024;
constexpr int kBigWaves = kBigThreads / 64;
constexpr int kBatchBig = 256;     // chunks per workspace batch
constexpr int kBigGrid = 256;      // filter_big_kernel workgroups (one per CU), each owns a basis slot
constexpr int kBigTile = 64;       // Gram output block

__global__ void __launch_bounds__(256) chunk_colmean_kernel(const float* __restrict__ X, int n, int64_t d,
                                                            int64_t ldx, int itv, int64_t chunk0, int nb,
                                                            double* __restrict__ mu) {
  const int64_t j0 = chunk0 * itv;
  const int64_t jend = (chunk0 + nb) * static_cast<int64_t>(itv);
  const int64_t j1 = jend < d ? jend : d;
  const int64_t j = j0 + static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (j >= j1) return;
  double sm = 0.0;
  for (int i = 0; i < n; ++i) sm += static_cast<double>(X[static_cast<int64_t>(i) * ldx + j]);
  mu[j - j0] = sm / n;
}

// block (I, J), I <= J, of chunk blockIdx.y: wave w owns rows 16 w .. + 15 of
// I against the four 16-row groups of J
__global__ void __launch_bounds__(256) chunk_gram_big_kernel(const float* __restrict__ X, int n, int64_t d,
                                                             int64_t ldx, int itv, int64_t chunk0,
                                                             const double* __restrict__ mu, double* __restrict__ Gb) {
  __shared__ __attribute__((aligned(16))) float sa[kBigTile * FROW];
  __shared__ __attribute__((aligned(16))) float sb[kBigTile * FROW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.y;
  int I = 0, J = 0;
  {
    const int nbk = static_cast<int>(cdiv(n, kBigTile));
    int p = blockIdx.x;
    while (p >= nbk - I) {
      p -= nbk - I;
      ++I;
    }
    J = I + p;
  }
  const int64_t k0 = (chunk0 + b) * static_cast<int64_t>(itv);
  const int k = static_cast<int>((k0 + itv < d ? k0 + itv : d) - k0);
  const double* mub = mu + static_cast<int64_t>(b) * itv;
  f64x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int s0 = 0; s0 < k; s0 += FST) {
    for (int e = tid; e < kBigTile * FST; e += 256) {
      const int r = e / FST, cc = e - (e / FST) * FST;
      const int ra = kBigTile * I + r, rb = kBigTile * J + r;
      const bool okc = s0 + cc < k;
      sa[r * FROW + cc] = (ra < n && okc) ? X[static_cast<int64_t>(ra) * ldx + k0 + s0 + cc] : 0.f;
      sb[r * FROW + cc] = (rb < n && okc) ? X[static_cast<int64_t>(rb) * ldx + k0 + s0 + cc] : 0.f;
    }
    __syncthreads();
    for (int ks = 0; ks < FST / 4; ++ks) {
      const int cc = 4 * ks + (lane >> 4);
      const double m = s0 + cc < k ? mub[s0 + cc] : 0.0;
      const int ra = 16 * w + (lane & 15);
      const double fa = (kBigTile * I + ra < n && s0 + cc < k) ? static_cast<double>(sa[ra * FROW + cc]) - m : 0.0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int rb = 16 * t + (lane & 15);
        const double fb = (kBigTile * J + rb < n && s0 + cc < k) ? static_cast<double>(sb[rb * FROW + cc]) - m : 0.0;
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  double* G = Gb + static_cast<size_t>(b) * n * n;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int row = kBigTile * I + 16 * w + (lane >> 4) + 4 * rg;
      const int col = kBigTile * J + 16 * t + (lane & 15);
      if (row < n && col < n) {
        G[static_cast<size_t>(row) * n + col] = acc[t][rg];
        if (I != J) G[static_cast<size_t>(col) * n + row] = acc[t][rg];
      }
    }
  }
}

// numpy pairwise fp32 sum of f(0..m), m <= 512: numpy splits while a piece
// holds more than 128 elements; from m <= 512 the largest piece after three
// splits is <= 76, so three levels are exact (m = 505: 248 + (128 + (64 + 65)))
template <typename F>
__device__ float np_pw32_big(int m, F&& f) {
  auto blk = [&](int lo, int mm) -> float {
    if (mm < 8) {
      float r = 0.f;
      for (int i = 0; i < mm; ++i) r += f(lo + i);
      return r;
    }
    float r0 = f(lo), r1 = f(lo + 1), r2 = f(lo + 2), r3 = f(lo + 3), r4 = f(lo + 4), r5 = f(lo + 5),
          r6 = f(lo + 6), r7 = f(lo + 7);
    int i = 8;
    for (; i < mm - (mm % 8); i += 8) {
      r0 += f(lo + i); r1 += f(lo + i + 1); r2 += f(lo + i + 2); r3 += f(lo + i + 3);
      r4 += f(lo + i + 4); r5 += f(lo + i + 5); r6 += f(lo + i + 6); r7 += f(lo + i + 7);
    }
    float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < mm; ++i) res += f(lo + i);
    return res;
  };
  auto quarter = [&](int lo, int mm) -> float {
    if (mm <= 128) return blk(lo, mm);
    int q = mm / 2;
    q -= q % 8;
    return blk(lo, q) + blk(lo + q, mm - q);
  };
  auto half = [&](int lo, int mm) -> float {
    if (mm <= 128) return blk(lo, mm);
    int q = mm / 2;
    q -= q % 8;
    return quarter(lo, q) + quarter(lo + q, mm - q);
  };
  if (m <= 128) return blk(0, m);
  int m2 = m / 2;
  m2 -= m2 % 8;
  return half(0, m2) + half(m2, m - m2);
}

template <int NB>
__global__ void __launch_bounds__(kBigThreads) noregret_pre_big_kernel(const double* __restrict__ Gb, int n, double eps,
                                                                       int* __restrict__ act, double* __restrict__ misc) {
  __shared__ float srt[kBigWaves][NB];
  __shared__ double diag[NB];
  __shared__ double score[NB];
  __shared__ int keep[NB];
  __shared__ float red[kBigWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const double* G = Gb + static_cast<size_t>(b) * n * n;
  const int fp = static_cast<int>(ceil(eps * n));
  if (tid < n) diag[tid] = G[static_cast<size_t>(tid) * n + tid];
  __syncthreads();
  auto dist = [&](int i, int j) -> float {
    const double sq = diag[i] + diag[j] - 2.0 * G[static_cast<size_t>(i) * n + j];
    return static_cast<float>(sqrt(sq > 0.0 ? sq : 0.0));
  };
  const int m = n - fp - 2 >= 0 ? (n - fp - 2 < n - 1 ? n - fp - 2 : n - 1)
                                : ((n - 1) + (n - fp - 2) > 0 ? (n - 1) + (n - fp - 2) : 0);
  const int pn = next_pow2(n - 1 > 1 ? n - 1 : 1);
  float* sr = srt[wave];
  for (int row = wave; row < n; row += kBigWaves) {
    for (int p = lane; p < pn; p += 64) sr[p] = p < n - 1 ? dist(row, p < row ? p : p + 1) : __builtin_inff();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int kk = 2; kk <= pn; kk <<= 1) {
      for (int st = kk >> 1; st > 0; st >>= 1) {
        for (int h = lane; h < pn / 2; h += 64) {
          const int a = (h / st) * (2 * st) + (h % st);
          const float va = sr[a], vb = sr[a + st];
          const float lo = fminf(va, vb), hi = fmaxf(va, vb);
          const bool up = (a & kk) == 0;
          sr[a] = up ? lo : hi;
          sr[a + st] = up ? hi : lo;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    if (lane == 0) {
      if constexpr (NB > NBIG) score[row] = static_cast<double>(np_pw32_rec<4>(0, m, [&](int q) { return sr[q]; }));
      else score[row] = static_cast<double>(np_pw32_big(m, [&](int q) { return sr[q]; }));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __syncthreads();
  // argpartition(metric, -f)[:-f]: drop the fp largest (ties: the later index first)
  if (tid < NB) {
    int kp = 0;
    if (tid < n) {
      const double si = score[tid];
      int above = 0;
      for (int j = 0; j < n; ++j) above += (score[j] > si || (score[j] == si && j > tid)) ? 1 : 0;
      kp = above >= fp ? 1 : 0;
    }
    keep[tid] = kp;
    act[static_cast<size_t>(b) * NB + tid] = kp;
  }
  __syncthreads();
  float md = 0.f;
  for (int e = tid; e < n * n; e += kBigThreads) {
    const int i = e / n, j = e - (e / n) * n;
    if (i < j && keep[i] && keep[j]) {
      const float dd = dist(i, j);
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
  if (tid == 0) {
    float mx = red[0];
    for (int q = 1; q < kBigWaves; ++q) mx = red[q] > mx ? red[q] : mx;
    misc[static_cast<size_t>(b) * kMisc + 1] = static_cast<double>(0.5f / (mx * mx));
  }
}

struct BigArgs {
  const double* G;   // [nb][n][n]
  double* c;         // [nb][NB]
  int* act;          // [nb][NB]
  double* misc;      // [nb][kMisc]
  int* status;
  int n;
  int nb;
  double eps;
  double sigma;
  double expansion;
  double* Vg;        // [grid][LMAX][NB]
  int* trace;        // optional [nb][1 + 2 n] decision trace (batch-relative), the small path's layout
};

constexpr int kHStride = LMAX + 2;
constexpr size_t big_lds(int nb) {
  return sizeof(double) * (4 * nb + kBigWaves * kHStride + kHStride + 2 * 4 * kBigWaves + kBigWaves * TRI + 4 * nb) +
         sizeof(int) * (3 * nb + 4 * kBigWaves + 16);
}
constexpr size_t kBigLds = big_lds(NBIG);
static_assert(big_lds(NBIG2) <= 163840, "the big solver's LDS must fit one CU");

// NB = NBIG: 1024 threads = two per row (the two column halves of every
// matvec); NB = NBIG2: one thread per row, the matvec over all columns.
template <int MODE, int NB = NBIG>
__global__ void __launch_bounds__(kBigThreads) filter_big_kernel(BigArgs A) {
  constexpr int HALVES = kBigThreads / NB;
  static_assert(HALVES == 1 || HALVES == 2, "one or two threads per row");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* xbuf = reinterpret_cast<double*>(smem);   // [NB] operator input
  double* ysum = xbuf + NB;                         // [2][NB] matvec halves
  double* rbuf = ysum + 2 * NB;                     // [NB] scratch
  double* hpart = rbuf + NB;                        // [kBigWaves][kHStride] per-wave dot products
  double* hbuf = hpart + kBigWaves * kHStride;      // [kHStride] Gram-Schmidt coefficients (+ |r''|^2)
  double* red = hbuf + kHStride;                    // [2][4 kBigWaves] block reductions
  double* tri = red + 2 * 4 * kBigWaves;            // [kBigWaves][TRI] per-wave tridiagonal record
  double* cvec = tri + kBigWaves * TRI;             // [NB]
  double* vscr = cvec + NB;                         // [3][NB]
  int* ibuf = reinterpret_cast<int*>(vscr + 3 * NB);   // [3][NB] + [4][kBigWaves] + [16]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = tid & (NB - 1);
  const int half = tid / NB;       // which half of every matvec's columns (HALVES == 2)
  const bool own = half == 0;      // the first NB threads speak for their row
  const int n = A.n;
  double* trw = tri + wave * TRI;
  double* Vb = A.Vg + static_cast<size_t>(blockIdx.x) * LMAX * NB;

  int rslot = 0;
  auto reduce4 = [&](double v0, double v1, double v2, double v3, double (&o)[4], int nv) {
    v0 = wave_sum(v0);
    if (nv > 1) v1 = wave_sum(v1);
    if (nv > 2) v2 = wave_sum(v2);
    if (nv > 3) v3 = wave_sum(v3);
    double* R = red + 4 * kBigWaves * rslot;
    if (lane == 0) {
      R[4 * wave + 0] = v0;
      if (nv > 1) R[4 * wave + 1] = v1;
      if (nv > 2) R[4 * wave + 2] = v2;
      if (nv > 3) R[4 * wave + 3] = v3;
    }
    __syncthreads();
    for (int kk = 0; kk < nv; ++kk) {
      double acc = R[kk];
      for (int q = 1; q < kBigWaves; ++q) acc += R[4 * q + kk];
      o[kk] = acc;
    }
    rslot ^= 1;
  };
  auto argmax_first = [&](double v, int i, double* vbest) -> int {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ov = __shfl_xor(v, off);
      const int oi = __shfl_xor(i, off);
      if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
      }
    }
    double* R = red + 4 * kBigWaves * rslot;
    int* I = ibuf + 3 * NB + 2 * kBigWaves * rslot;
    if (lane == 0) {
      R[wave] = v;
      I[wave] = i;
    }
    __syncthreads();
    double bv = R[0];
    int bi = I[0];
    for (int q = 1; q < kBigWaves; ++q)
      if (R[q] > bv || (R[q] == bv && I[q] < bi)) {
        bv = R[q];
        bi = I[q];
      }
    rslot ^= 1;
    *vbest = bv;
    return bi;
  };
  // y_row = sum_j G[j][row] x_j (G symmetric): each half sums its columns in
  // order, the halves are added in a fixed order
  auto gmv = [&](const double* G) -> double {
    const int hn = (n + HALVES - 1) / HALVES;
    const int j0 = half * hn, j1 = j0 + hn < n ? j0 + hn : n;
    double p0 = 0.0, p1 = 0.0;
    if (row < n) {
      int j = j0;
      for (; j + 1 < j1; j += 2) {
        p0 = fma(G[static_cast<size_t>(j) * n + row], xbuf[j], p0);
        p1 = fma(G[static_cast<size_t>(j + 1) * n + row], xbuf[j + 1], p1);
      }
      if (j < j1) p0 = fma(G[static_cast<size_t>(j) * n + row], xbuf[j], p0);
    }
    // ysum is rewritten by the next gmv only after a reduction's barrier
    if constexpr (HALVES == 1) {
      __syncthreads();   // every thread has read xbuf before it is rewritten
      return p0 + p1;
    } else {
      ysum[half * NB + row] = p0 + p1;
      __syncthreads();
      return ysum[row] + ysum[NB + row];
    }
  };

  for (int ch = blockIdx.x; ch < A.nb; ch += gridDim.x) {
    const double* G = A.G + static_cast<size_t>(ch) * n * n;
    bool ai;
    if constexpr (MODE == 1) ai = own && row < n && A.act[static_cast<size_t>(ch) * NB + row] != 0;
    else ai = own && row < n;
    double ci = ai ? 1.0 : 0.0;
    const int fdrop = static_cast<int>(ceil(A.eps * n));
    const int n_keep = MODE == 1 ? n - (fdrop < n ? fdrop : n) : n;
    const double step = MODE == 1 ? A.misc[static_cast<size_t>(ch) * kMisc + 1] : 0.0;
    const int iters = MODE == 0 ? 2 * static_cast<int>(A.eps * n) : static_cast<int>(2 * A.eps * n_keep);
    double ui = 0.0;
    bool have_u = false;
    int m_hint = 12;
    double rate_hint = 0.0;
    int done = 0;
    int* tr = A.trace != nullptr ? A.trace + static_cast<size_t>(ch) * (1 + 2 * n) : nullptr;
    bool none = false, unweighted = false;   // projected_c None: see filter_solve_kernel

    for (int it = 0; it < iters; ++it) {
      if (MODE == 1 && none) ci = ai ? 1.0 : 0.0;
      double o[4];
      reduce4(ai ? ci : 0.0, ai ? 1.0 : 0.0, 0.0, 0.0, o, 2);
      const double csum = o[0];
      const int nact = static_cast<int>(o[1]);
      const double wi = ai ? ci / csum : 0.0;
      const double swi = sqrt(wi > 0.0 ? wi : 0.0);
      if (own) xbuf[row] = wi;
      __syncthreads();
      const double gwi = gmv(G);
      reduce4(own ? wi * gwi : 0.0, 0.0, 0.0, 0.0, o, 1);
      const double sgw = o[0];

      double lam = 0.0;
      int m_conv = 0, restarts = 0;
      double rt;
      {
        const double hh = 0.5 + (row * 0.6180339887498949 - floor(row * 0.6180339887498949));
        rt = swi > 0.0 ? (have_u ? ui + 1e-3 * swi * hh : swi * hh) : 0.0;
      }
      for (;;) {
        double xt = swi * rt;
        if (own) xbuf[row] = xt;
        reduce4(own ? rt * rt : 0.0, own ? xt : 0.0, own ? gwi * xt : 0.0, 0.0, o, 3);
        double nrm2 = o[0], S1 = o[1], GY = o[2];
        double qprev = 0.0, tscale = 0.0, theta_lb = -1e300;
        int next_check = m_hint - 1 > 4 ? m_hint - 1 : 4;
        int m_a = -1;
        double res_a = 0.0;
        bool converged = false;
        for (int j = 0;; ++j) {
          const double bet = sqrt(nrm2);
          if (j > 0) {
            if (lane == 0) trw[64 + j - 1] = bet * bet;
            tscale = fmax(tscale, bet);
            const bool breakdown = !(bet > 1e-14 * tscale);
            if (breakdown || j >= nact || j == LMAX || j >= next_check) {
              const int m = j;
              __builtin_amdgcn_wave_barrier();
              double lm, zlast;
              tri_top(trw, m, tscale, theta_lb, &lm, &zlast);
              lam = lm;
              const double resid = fabs(bet * zlast);
              theta_lb = lm;
              if (resid <= kResTol * fabs(lm) || breakdown || j >= nact) {
                converged = true;
                m_conv = m;
                break;
              }
              if (j == LMAX) break;
              int adv = 4;
              double rate = rate_hint;
              if (m_a >= 0 && res_a > resid && resid > 0.0) rate = rate_hint = log(resid / res_a) / (m - m_a);
              if (rate < 0.0 && resid > 0.0) {
                const double need = log(kResTol * fabs(lm) / resid) / rate;
                adv = need < 1.0 ? 1 : (need > LMAX ? LMAX : static_cast<int>(ceil(need)));
              }
              m_a = m;
              res_a = resid;
              next_check = m + adv;
            }
          }
          // (1) y = G x~, alpha_j, r' = M q_j - beta q_{j-1}
          const double y = gmv(G);
          const double cx = y - gwi * S1 - GY + sgw * S1;
          const double ib = 1.0 / bet;
          const double q = rt * ib;
          if (own && row < n) Vb[static_cast<size_t>(j) * NB + row] = q;
          const double rp = swi * cx * ib - (j > 0 ? bet * qprev : 0.0);
          qprev = q;
          reduce4(own ? swi * rt * y : 0.0, 0.0, 0.0, 0.0, o, 1);
          const double aj = (o[0] - 2.0 * S1 * GY + sgw * S1 * S1) * (ib * ib);
          double r = own && row < n ? rp - aj * q : 0.0;
          double alpha = aj;
#pragma unroll 1
          for (int pass = 0; pass < 2; ++pass) {
            // (2) h_q = q_q . r (q <= j), and |r|^2 in the first pass
            const int nh = pass == 0 ? j + 2 : j + 1;
            for (int qq = 0; qq < nh; ++qq) {
              double v = 0.0;
              if (own && row < n) v = qq <= j ? Vb[static_cast<size_t>(qq) * NB + row] * r : r * r;
              v = wave_sum(v);
              if (lane == 0) hpart[wave * kHStride + qq] = v;
            }
            __syncthreads();
            if (tid < nh) {
              double hs = hpart[tid];
              for (int w2 = 1; w2 < kBigWaves; ++w2) hs += hpart[w2 * kHStride + tid];
              hbuf[tid] = hs;
            }
            __syncthreads();
            // (3) r -= sum_q h_q q_q
            double upd = 0.0, hn2 = 0.0;
            for (int qq = 0; qq <= j; ++qq) {
              const double hv = hbuf[qq];
              if (own && row < n) upd = fma(hv, Vb[static_cast<size_t>(qq) * NB + row], upd);
              hn2 = fma(hv, hv, hn2);
            }
            r -= upd;
            alpha += hbuf[j];
            if (pass == 1) break;
            const double rr2 = hbuf[j + 1];
            if (!(rr2 - hn2 < kDgks * rr2)) break;
            __syncthreads();   // hbuf is rewritten by the second pass
          }
          if (lane == 0) trw[j] = alpha;
          tscale = fmax(tscale, fabs(alpha));
          rt = r;
          xt = swi * r;
          if (own) xbuf[row] = xt;
          reduce4(own ? r * r : 0.0, own ? xt : 0.0, own ? gwi * xt : 0.0, 0.0, o, 3);
          nrm2 = o[0];
          S1 = o[1];
          GY = o[2];
        }
        {
          const int m = converged ? m_conv : LMAX;
          double u0 = 0.0;
          if (own && row < n)
            for (int qq = 0; qq < m; ++qq) u0 = fma(trw[128 + qq], Vb[static_cast<size_t>(qq) * NB + row], u0);
          ui = u0;
        }
        if (converged || restarts == kMaxRestarts) break;
        ++restarts;
        rt = ui;
        __syncthreads();
      }
      m_hint = m_conv > 4 ? m_conv : 4;
      have_u = true;
      if (lam * lam <= A.expansion * A.sigma * A.sigma) {   // robust_estimator.py:163-164 / :71-72
        unweighted = none;
        break;
      }
      if (MODE == 1 && none) {
        if (tid == 0) *A.status = 2;   // c * (1 - step * tau) with c None: TypeError (:75)
        break;
      }
      {
        const double xt = swi * ui;
        if (own) xbuf[row] = xt;
        reduce4(own ? xt : 0.0, own ? gwi * xt : 0.0, 0.0, 0.0, o, 2);
      }
      const double cu = gmv(G) - gwi * o[0] - o[1] + sgw * o[0];
      const double ti = cu * cu / lam;
      if constexpr (MODE == 0) {
        double tmax = 0.0;
        const int p = argmax_first(ai ? ti : -__builtin_inf(), row, &tmax);
        const double cn = (ai && row != p) ? ci * (1.0 - ti / tmax) : 0.0;
        reduce4(own ? fabs(cn) : 0.0, 0.0, 0.0, 0.0, o, 1);
        ci = cn / o[0];
        if (row == p) ai = false;
        if (tr != nullptr && tid == 0) tr[1 + it] = p;
      } else {
        const int nk = n_keep;
        const double cap = 1.0 / (1.0 - A.eps) / nk;
        if (ai) ci = ci * (1.0 - step * ti);
        int capped = 0;
        if (!kl_project_t<NB, kBigWaves>(&ci, ai, row, own && row < n, nk, cap, cvec, vscr, ibuf, red, hbuf,
                                            &capped)) {
          none = true;   // projected_c = None (:99)
          unweighted = it + 1 == iters;
          if (unweighted && ai) ci = 1.0;
        }
        if (tr != nullptr && tid == 0) tr[1 + it] = capped;
      }
      done = it + 1;
    }
    if (tr != nullptr) {
      if (tid == 0) tr[0] = done;
      if (own && row < n) tr[1 + n + row] = ai ? 1 : 0;
    }
    __syncthreads();
    if (own) {
      cvec[row] = ai ? ci : 0.0;
      ibuf[2 * NB + row] = ai ? 1 : 0;
      A.c[static_cast<size_t>(ch) * NB + row] = ai ? ci : 0.0;
      A.act[static_cast<size_t>(ch) * NB + row] = ai ? 1 : 0;
    }
    __syncthreads();
    if (tid == 0) {
      int q2 = 0;
      double* kept = vscr;
      for (int i = 0; i < n; ++i)
        if (ibuf[2 * NB + i]) kept[q2++] = cvec[i];
      auto kz = [&](int z) { return kept[z]; };
      if constexpr (NB > NBIG) A.misc[static_cast<size_t>(ch) * kMisc] = np_pw64_rec<4>(0, q2, kz);
      else A.misc[static_cast<size_t>(ch) * kMisc] = np_pw64(0, q2, kz);
      A.misc[static_cast<size_t>(ch) * kMisc + 2] = unweighted ? 1.0 : 0.0;
      if (unweighted) atomicAdd(A.status + 1, 1);
    }
    __syncthreads();
  }
}

// ============================================================================
// host side
// ============================================================================
// per chunk of a batch: G, weights, scalars, kept flags, fallback list slot
constexpr size_t kChunkWsBytes = sizeof(double) * (FNP * FNP + FNP + kMisc) + sizeof(int) * (FNP + 1);
constexpr int kLanczosGrid = 1024;   // waves of wave_solve_kernel: 4 per CU, each owns a basis slot

// N > FNP: [G nb n n][c nb NB][misc nb kMisc][mu nb itv][V grid LMAX NB][act nb NB], NB = NBIG or NBIG2
static int big_rows(int n) { return n > NBIG ? NBIG2 : NBIG; }
static size_t filter_big_workspace_bytes(int n, int64_t d, int itv) {
  const int64_t nchunks = cdiv(d, itv);
  const int64_t b = nchunks < kBatchBig ? nchunks : kBatchBig;
  const int64_t grid = b < kBigGrid ? b : kBigGrid;
  const size_t NB = big_rows(n);
  return 256 + static_cast<size_t>(b) * (sizeof(double) * (static_cast<size_t>(n) * n + NB + kMisc + itv) +
                                         sizeof(int) * NB) +
         static_cast<size_t>(grid) * LMAX * NB * sizeof(double) + 256;
}

int launch_filter_big(int mode, const float* X, int n, int64_t d, int64_t ldx, int itv, double eps, double sigma,
                      double expansion, double* out, int* status, int* trace, void* ws, hipStream_t s) {
  const int64_t nchunks = cdiv(d, itv);
  const int64_t bmax = nchunks < kBatchBig ? nchunks : kBatchBig;
  const int grid_max = static_cast<int>(bmax < kBigGrid ? bmax : kBigGrid);
  const int NB = big_rows(n);
  const bool wide = NB == NBIG2;
  const size_t lds = wide ? big_lds(NBIG2) : kBigLds;
  char* base = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  double* Gws = reinterpret_cast<double*>(base);
  double* cws = Gws + static_cast<size_t>(bmax) * n * n;
  double* mws = cws + static_cast<size_t>(bmax) * NB;
  double* muws = mws + static_cast<size_t>(bmax) * kMisc;
  double* Vws = muws + static_cast<size_t>(bmax) * itv;
  int* aws = reinterpret_cast<int*>(Vws + static_cast<size_t>(grid_max) * LMAX * NB);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&filter_big_kernel<0>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     static_cast<int>(kBigLds));
  static const hipError_t attr1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&filter_big_kernel<1>),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      static_cast<int>(kBigLds));
  static const hipError_t attr2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&filter_big_kernel<0, NBIG2>),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      static_cast<int>(big_lds(NBIG2)));
  static const hipError_t attr3 = hipFuncSetAttribute(reinterpret_cast<const void*>(&filter_big_kernel<1, NBIG2>),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      static_cast<int>(big_lds(NBIG2)));
  SRA_REQUIRE(attr == hipSuccess && attr1 == hipSuccess && attr2 == hipSuccess && attr3 == hipSuccess,
              SRA_ERR_UNSUPPORTED, "filter_big_kernel: cannot reserve %zu bytes of LDS", lds);
  const int nbk = static_cast<int>(cdiv(n, kBigTile));
  for (int64_t c0 = 0; c0 < nchunks; c0 += bmax) {
    const int nb = static_cast<int>(nchunks - c0 < bmax ? nchunks - c0 : bmax);
    const int64_t jend = (c0 + nb) * static_cast<int64_t>(itv);
    const int64_t ncols = (jend < d ? jend : d) - c0 * static_cast<int64_t>(itv);
    hipLaunchKernelGGL(chunk_colmean_kernel, dim3(cdiv(ncols, 256)), dim3(256), 0, s, X, n, d, ldx, itv, c0, nb, muws);
    int rc = launch_status("chunk_colmean_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(chunk_gram_big_kernel, dim3(nbk * (nbk + 1) / 2, nb), dim3(256), 0, s, X, n, d, ldx, itv, c0,
                       muws, Gws);
    rc = launch_status("chunk_gram_big_kernel");
    if (rc) return rc;
    if (mode == 1) {
      if (wide)
        hipLaunchKernelGGL(noregret_pre_big_kernel<NBIG2>, dim3(nb), dim3(kBigThreads), 0, s, Gws, n, eps, aws, mws);
      else
        hipLaunchKernelGGL(noregret_pre_big_kernel<NBIG>, dim3(nb), dim3(kBigThreads), 0, s, Gws, n, eps, aws, mws);
      rc = launch_status("noregret_pre_big_kernel");
      if (rc) return rc;
    }
    BigArgs ba{Gws, cws, aws, mws, status, n, nb, eps, sigma, expansion, Vws,
               trace != nullptr ? trace + static_cast<size_t>(c0) * (1 + 2 * n) : nullptr};
    const int grid = nb < grid_max ? nb : grid_max;
    if (wide) {
      if (mode == 0) hipLaunchKernelGGL((filter_big_kernel<0, NBIG2>), dim3(grid), dim3(kBigThreads), lds, s, ba);
      else hipLaunchKernelGGL((filter_big_kernel<1, NBIG2>), dim3(grid), dim3(kBigThreads), lds, s, ba);
    } else {
      if (mode == 0) hipLaunchKernelGGL(filter_big_kernel<0>, dim3(grid), dim3(kBigThreads), kBigLds, s, ba);
      else hipLaunchKernelGGL(filter_big_kernel<1>, dim3(grid), dim3(kBigThreads), kBigLds, s, ba);
    }
    rc = launch_status("filter_big_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(chunk_mean_kernel, dim3(cdiv(ncols, 256)), dim3(256), 0, s, X, n, d, ldx, int64_t(0), itv, c0,
                       nb, cws, aws, mws, out, NB, mode);
    rc = launch_status("chunk_mean_kernel");
    if (rc) return rc;
  }
  return SRA_OK;
}

// bucketed: the MoM form's bucket rows of one batch (n x batch columns fp32)
size_t filter_workspace_bytes(int n, int64_t d, int itv, bool bucketed) {
  if (n > FNP) return filter_big_workspace_bytes(n, d, itv);
  const int64_t nchunks = cdiv(d, itv);
  const int64_t b = nchunks < kBatch ? nchunks : kBatch;
  const int64_t grid = b < kLanczosGrid ? b : kLanczosGrid;
  return static_cast<size_t>(b) * kChunkWsBytes + static_cast<size_t>(grid) * (MMAX + 1) * FNP * sizeof(double) + 528 +
         (bucketed ? static_cast<size_t>(n) * b * itv * sizeof(float) + 256 : 0);
}

// bs > 0: the MoM forms -- X holds nsrc clients, n = the bucket count (<= FNP)
int launch_filter(int mode, const float* X, int n, int64_t d, int64_t ldx, int itv, double eps, double sigma,
                  double expansion, double* out, int* status, double* dbg, int* trace, void* ws, size_t ws_bytes,
                  hipStream_t s, int bs = 0, int nsrc = 0) {
  SRA_REQUIRE(n >= 1 && n <= NBIG2, SRA_ERR_UNSUPPORTED, "spectral filters support 1 <= N <= %d (got %d)", NBIG2, n);
  SRA_REQUIRE(itv >= 1, SRA_ERR_ARG, "itv must be >= 1");
  const int64_t nchunks = cdiv(d, itv);
  SRA_REQUIRE(nchunks < (int64_t(1) << 31), SRA_ERR_ARG, "too many chunks");
  SRA_REQUIRE(ws != nullptr && ws_bytes >= filter_workspace_bytes(n, d, itv, bs > 0), SRA_ERR_WORKSPACE,
              "filter workspace too small: need %zu bytes", filter_workspace_bytes(n, d, itv, bs > 0));
  SRA_REQUIRE(bs == 0 || n <= FNP, SRA_ERR_UNSUPPORTED, "fused MoM filters take <= %d buckets (got %d)", FNP, n);
  if (n > FNP) {
    SRA_REQUIRE(dbg == nullptr, SRA_ERR_UNSUPPORTED, "filter debug records support N <= %d (got %d)", FNP, n);
    return launch_filter_big(mode, X, n, d, ldx, itv, eps, sigma, expansion, out, status, trace, ws, s);
  }
  const int64_t bmax = nchunks < kBatch ? nchunks : kBatch;
  const int lgrid_max = static_cast<int>(bmax < kLanczosGrid ? bmax : kLanczosGrid);
  char* base = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  double* Gws = reinterpret_cast<double*>(base);
  double* cws = Gws + static_cast<size_t>(bmax) * FNP * FNP;
  double* mws = cws + static_cast<size_t>(bmax) * FNP;
  double* Vws = mws + static_cast<size_t>(bmax) * kMisc;
  int* aws = reinterpret_cast<int*>(Vws + static_cast<size_t>(lgrid_max) * (MMAX + 1) * FNP);   // wave_solve_kernel: MMAX + 1 basis slots per wave
  int* fbl = aws + static_cast<size_t>(bmax) * FNP;
  int* fbc = fbl + bmax;   // [0] listed chunks, [1] ghost after the retry, [2] out of steps, [3] retries,
                           // [4] the solver's chunk queue
  const int64_t ldb = bmax * itv;   // bucket rows of a batch (MoM forms)
  float* Bws = bs > 0 ? reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(fbc + 8) + 255) & ~uintptr_t(255))
                      : nullptr;
  const void* solve = mode == 0 ? (dbg ? reinterpret_cast<const void*>(&filter_solve_kernel<0, true>)
                                       : reinterpret_cast<const void*>(&filter_solve_kernel<0, false>))
                                : (dbg ? reinterpret_cast<const void*>(&filter_solve_kernel<1, true>)
                                       : reinterpret_cast<const void*>(&filter_solve_kernel<1, false>));
  SRA_HIP(hipFuncSetAttribute(solve, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kSolveLds)));
  for (int64_t c0 = 0; c0 < nchunks; c0 += bmax) {
    const int nb = static_cast<int>(nchunks - c0 < bmax ? nchunks - c0 : bmax);
    // 16-byte fills when X, ldx, itv and d (and the bucket rows) allow them:
    // the plain C4 Gram 5.28 -> 3.56 ms
    const bool al4 = ldx % 4 == 0 && itv % 4 == 0 && d % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
    const int vec4 = bs > 0 ? al4 && ldb % 4 == 0 && (reinterpret_cast<uintptr_t>(Bws) & 15) == 0 : al4;
    GramArgs ga{X, n, d, ldx, itv, c0, nb, Gws, bs, nsrc, Bws, ldb, vec4};
    if (bs > 0) hipLaunchKernelGGL(chunk_gram_kernel<true>, dim3(nb), dim3(256), 0, s, ga);
    else hipLaunchKernelGGL(chunk_gram_kernel<false>, dim3(nb), dim3(256), 0, s, ga);
    int rc = launch_status("chunk_gram_kernel");
    if (rc) return rc;
    if (dbg != nullptr && c0 == 0)
      SRA_HIP(hipMemcpyAsync(dbg, Gws, sizeof(double) * FNP * FNP, hipMemcpyDeviceToDevice, s));
    if (mode == 1) {
      PreArgs pa{Gws, aws, mws, n, nb, eps};
      hipLaunchKernelGGL(noregret_pre_kernel, dim3(nb), dim3(256), 0, s, pa);
      rc = launch_status("noregret_pre_kernel");
      if (rc) return rc;
    }
    // check schedule of the one-wave solver: first check 12 steps before the
    // previous iteration's step count -- a check (~25k cycles) costs ~6 steps,
    // a late first check a ghost and a dense retry (C4 filterL2: -8 106.0 ms,
    // -12 91.0, -16 92.4, -20 93.5; 0 221, DESIGN k6)
    constexpr int first_off = -12;
    SolveArgs sa{Gws, cws, aws, mws, status, n, nb, eps, sigma, expansion, c0 == 0 ? dbg : nullptr, Vws, fbl, fbc,
                 trace != nullptr ? trace + static_cast<size_t>(c0) * kTraceStride : nullptr, first_off,
                 kMaxAdvance, 0, bs > 0 ? Bws : X, bs > 0 ? ldb : ldx, bs > 0 ? c0 * itv : int64_t(0), itv, d, c0,
                 out};
    SRA_HIP(hipMemsetAsync(fbc, 0, 8 * sizeof(int), s));
    const int lgrid = nb < lgrid_max ? nb : lgrid_max;
    // both filters on the one-wave solver (ex_noregret re-orthogonalising
    // from the first step, wave_solve_kernel<1>)
    rc = launch_wave_solve(mode, dbg != nullptr, sa, lgrid, s);
    if (rc) return rc;
    // the listed chunks (not converged / ghost) on the re-orthogonalising solver
    const int grid = nb < 512 ? nb : 512;
    if (mode == 0 && dbg) hipLaunchKernelGGL((filter_solve_kernel<0, true>), dim3(grid), dim3(256), kSolveLds, s, sa);
    else if (mode == 0) hipLaunchKernelGGL((filter_solve_kernel<0, false>), dim3(grid), dim3(256), kSolveLds, s, sa);
    else if (dbg) hipLaunchKernelGGL((filter_solve_kernel<1, true>), dim3(grid), dim3(256), kSolveLds, s, sa);
    else hipLaunchKernelGGL((filter_solve_kernel<1, false>), dim3(grid), dim3(256), kSolveLds, s, sa);
    rc = launch_status("filter_solve_kernel");
    if (rc) return rc;
    // diagnostics: the first batch's fallback count, as an int32 in the low
    // word of the last record's last slot
    if (dbg != nullptr && c0 == 0)
      SRA_HIP(hipMemcpyAsync(dbg + FNP * FNP + 255 * kDbgRec + kDbgRec - 3, fbc, 6 * sizeof(int), hipMemcpyDeviceToDevice, s));
    const int64_t jend = (c0 + nb) * static_cast<int64_t>(itv);
    const int64_t ncols = (jend < d ? jend : d) - c0 * static_cast<int64_t>(itv);
    // the chunk means read the filtered rows: X itself, or the batch's bucket rows
    hipLaunchKernelGGL(chunk_mean_kernel, dim3(cdiv(ncols, 256)), dim3(256), 0, s, bs > 0 ? Bws : X, n, d,
                       bs > 0 ? ldb : ldx, bs > 0 ? c0 * itv : int64_t(0), itv, c0, nb, cws, aws, mws, out, FNP, mode);
    rc = launch_status("chunk_mean_kernel");
    if (rc) return rc;
  }
  return SRA_OK;
}

static int filter_checks(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, double eps, double* out,
                         int32_t* status) {
  SRA_REQUIRE(X != nullptr && out != nullptr && status != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx");
  SRA_REQUIRE(mode == 0 || mode == 1, SRA_ERR_ARG, "mode must be 0 (filterL2) or 1 (ex_noregret)");
  // ex_noregret drops ceil(eps*n) clients and takes the max over the pairwise
  // distances of the rest: the reference raises (amax of an empty list) below 2
  SRA_REQUIRE(mode == 0 || n - static_cast<int64_t>(std::ceil(eps * n)) >= 2, SRA_ERR_ARG,
              "ex_noregret needs at least 2 clients after dropping ceil(eps*n)");
  // f = ceil(eps*n) = 0: argpartition(metric, -0)[:-0] keeps nothing and the
  // reference's np.amax of the empty distance list raises ValueError
  SRA_REQUIRE(mode == 0 || std::ceil(eps * n) >= 1.0, SRA_ERR_ARG,
              "ex_noregret with ceil(eps*n) = 0 keeps no client (the reference raises ValueError)");
  return SRA_OK;
}

}  // namespace sra

extern "C" int sra_filter_workspace_bytes(int64_t n, int64_t d, int32_t itv, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && d >= 1 && itv >= 1, SRA_ERR_SHAPE, "bad shape");
  *bytes = sra::filter_workspace_bytes(static_cast<int>(n), d, itv, false);
  return SRA_OK;
}

extern "C" int sra_mom_filter_workspace_bytes(int64_t nbuckets, int64_t d, int32_t itv, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(nbuckets >= 1 && nbuckets <= sra::FNP && d >= 1 && itv >= 1, SRA_ERR_SHAPE, "bad shape");
  *bytes = sra::filter_workspace_bytes(static_cast<int>(nbuckets), d, itv, true);
  return SRA_OK;
}

extern "C" int sra_mom_filter_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                                  int32_t bucket_size, int32_t nbuckets, double eps, double sigma, double expansion,
                                  double* out, int32_t* status, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(n >= 1, SRA_ERR_SHAPE, "bad shape");
  SRA_REQUIRE(bucket_size >= 1 && nbuckets >= 1 && nbuckets <= sra::FNP, SRA_ERR_UNSUPPORTED,
              "fused MoM filters take 1 <= nbuckets <= %d (got %d)", sra::FNP, nbuckets);
  SRA_REQUIRE(static_cast<int64_t>(nbuckets - 1) * bucket_size < n, SRA_ERR_EMPTY_BUCKET,
              "bucket %d of size %d is empty for N=%lld (the reference's np.mean of an empty slice)",
              (int)((n + bucket_size - 1) / bucket_size), bucket_size, (long long)n);
  const int rc = sra::filter_checks(X, nbuckets, d, ldx, mode, eps, out, status);
  if (rc) return rc;
  return sra::launch_filter(mode, X, nbuckets, d, ldx, itv, eps, sigma, expansion, out, status, nullptr, nullptr, ws,
                            ws_bytes, static_cast<hipStream_t>(stream), bucket_size, static_cast<int>(n));
}

extern "C" int sra_filter_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                              double eps, double sigma, double expansion, double* out, int32_t* status, void* ws,
                              size_t ws_bytes, void* stream) {
  const int rc = sra::filter_checks(X, n, d, ldx, mode, eps, out, status);
  if (rc) return rc;
  return sra::launch_filter(mode, X, static_cast<int>(n), d, ldx, itv, eps, sigma, expansion, out, status, nullptr,
                            nullptr, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int sra_filter_trace_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                                    double eps, double sigma, double expansion, double* out, int32_t* status,
                                    int32_t* trace, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(trace != nullptr, SRA_ERR_ARG, "null trace pointer");
  const int rc = sra::filter_checks(X, n, d, ldx, mode, eps, out, status);
  if (rc) return rc;
  return sra::launch_filter(mode, X, static_cast<int>(n), d, ldx, itv, eps, sigma, expansion, out, status, nullptr,
                            trace, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int sra_filter_debug_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                                    double eps, double sigma, double expansion, double* out, int32_t* status,
                                    double* dbg, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(dbg != nullptr, SRA_ERR_ARG, "null pointer");
  const int rc = sra::filter_checks(X, n, d, ldx, mode, eps, out, status);
  if (rc) return rc;
  return sra::launch_filter(mode, X, static_cast<int>(n), d, ldx, itv, eps, sigma, expansion, out, status, dbg,
                            nullptr, ws, ws_bytes, static_cast<hipStream_t>(stream));
}
