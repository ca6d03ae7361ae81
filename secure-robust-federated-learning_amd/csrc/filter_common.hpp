// Declarations shared by the spectral-filter solvers (k6): filter.hip
// (chunk Gram, Krum pre-filter, the four-wave solvers, the N > 128 paths,
// the chunk means and the host side) and filter_wave.hip (the one-wave
// solver, round 5).  Replaces nothing on its own; see filter.hip's header
// for the reference lines (src/robust_estimator.py:42-218).
#pragma once
#include <type_traits>

#include "sra_common.hpp"

namespace sra {

constexpr int FNP = 128;           // padded client count
constexpr int FST = 64;            // coordinates per Gram stage
constexpr int FROW = FST + 4;      // stage row stride (floats)
constexpr int LMAX = 59;           // Lanczos basis capacity (LDS)
constexpr int VST = 136;           // basis row stride (doubles): the 4 rows one ds_read_b128 lane group
                                   // touches start 16 banks apart
constexpr int XOFF = 66;           // vector buffers: entries [64, 128) start at XOFF (bank-disjoint halves)
constexpr int XLEN = XOFF + 64 + 2;
constexpr int TRI = 256;           // per-wave tridiagonal record: alpha[64] beta^2[64] s / dp[64] dm[64]
constexpr double kResTol = 1e-16;  // converged when the Ritz residual <= kResTol * lambda
constexpr double kDgks = 0.5;      // second Gram-Schmidt pass when |r|^2 < kDgks * |r'|^2 (DGKS)
constexpr int kMaxRestarts = 8;
constexpr int kBatch = 16384;      // chunks per workspace batch (a d = 1e7 layer at itv 1000 in one)
constexpr int kMisc = 8;           // per-chunk scalars: [0] np.average scale, [1] ex_noregret step

// per-iteration diagnostics of chunk 0 (sra_filter_debug_f32): FNP weights
// before the update, then lambda, Lanczos steps, Ritz residual, checks, active
// clients, w'Gw, restarts, second Gram-Schmidt passes, cycles of the iteration
constexpr int kDbgRec = FNP + 16;

// ----- wave helpers ---------------------------------------------------------
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

// a / b from the hardware reciprocal with one Newton step and one residual
// correction (within an ulp or two; pivots of the tridiagonal only)
__device__ __forceinline__ double fdiv(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = fma(fma(-b, r, 1.0), r, r);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}

// numpy pairwise fp32 sum of f(0..n) (n <= 255 via one split)
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

struct SolveArgs {
  const double* G;   // [nb][FNP][FNP]
  double* c;         // [nb][FNP] out: final weights
  int* act;          // [nb][FNP] in (ex_noregret: the pre-filter's kept set) / out: kept
  double* misc;      // [nb][kMisc]
  int* status;
  int n;
  int nb;
  double eps;
  double sigma;
  double expansion;
  double* dbg;       // optional diagnostics of the batch's chunk 0
  double* Vg;        // lanczos_solve_kernel: [grid][MMAX][FNP] Lanczos basis per workgroup
  int* fb_list;      // chunks handed to the re-orthogonalising fallback
  int* fb_count;
  int* trace;        // optional [nb][1 + 2 FNP] decision trace (sra_filter_trace_f32), batch-relative
  int first_off;     // first check at (previous iteration's steps) + first_off
  int max_adv;       // checks at most this many steps apart
  int warm;          // (unused since round 5)
  // round 5: wave_solve_kernel writes the chunk means itself once a chunk's
  // weights are final (chunk_mean_kernel's arithmetic and order) and flags the
  // chunk in misc[kMisc * ch + 3]; chunk_mean_kernel then covers only the
  // chunks the fallback solver finished.  Xm = X or the batch's bucket rows.
  const float* Xm;
  int64_t ldxm;
  int64_t jx0;       // column of Xm holding the batch's first coordinate
  int itv;
  int64_t d;
  int64_t chunk0;    // the batch's first chunk
  double* out;
};

// Decision trace of one chunk (sra_filter_trace_f32): [0] iterations completed
// (< T after the early exit), [1 + it] the decision of iteration it -- the
// removed client (filterL2, robust_estimator.py:166-172) or the capped count of
// the kept projection candidate (ex_noregret, :78-99) -- and [1 + FNP + row]
// whether the client is still active at the end (ex_noregret: kept by the
// Krum pre-filter, :49-51).
constexpr int kTraceStride = 1 + 2 * FNP;

constexpr int MMAX = 128;          // plain Lanczos steps per eigenproblem (two lane slots of the check)
constexpr int kMaxAdvance = 8;     // checks at most this far apart (a ghost forms ~15-20 steps past convergence)
constexpr double kAccept = 2.5e-16;  // plain Lanczos: accept the Ritz pair at residual <= kAccept * lambda

__device__ __forceinline__ double rl_any(const double (&v)[2], int q) {
  // q wave-uniform: both readlanes land in SGPRs, the select is scalar
  const double a = readlane_f64(v[0], q & 63), b = readlane_f64(v[1], q & 63);
  return q < 64 ? a : b;
}

__device__ __forceinline__ double rcp_nr(double b) {   // 1/b within ~1 ulp
  const double r = __builtin_amdgcn_rcp(b);
  return fma(fma(-b, r, 1.0), r, r);
}

// filter_wave.hip: the one-wave filterL2 solver (round 5)
size_t wave_solve_lds();
int wave_solve_grid();
int launch_wave_solve(int mode, bool dbg, const SolveArgs& sa, int grid, hipStream_t s);

}  // namespace sra
