// k4 — Bulyan (src/robust_estimator.py:259-332).
//
// Selection (theta = N - 2f rounds, :286-322):
//   krum        -> k3 krum rounds on the k2 Gram (krum.hip), the chosen clients
//                  themselves are the selected vectors;
//   median /    -> per round: k-select over the remaining clients (row list) ->
//   trimmedmean    aggregate vector (row t of S); squared distance of every
//                  remaining client to it; the first strict minimum is removed
//                  from the (order-preserving) device row list.  No host sync
//                  between rounds.
// Per-coordinate stage (:324-330, bulyan_one_coordinate/bulyan_median), one
// lane per coordinate, beta = theta - 2f:
//   1. sort the theta selected values (register network);
//   2. the Bulyan median m = argmin_i sum_j |a_i - a_j| (first index) is a
//      middle order statistic; for even theta the lower and upper middles tie
//      in exact arithmetic and numpy's fp64 pairwise row sum (8 accumulators,
//      in selection order) decides -- emulated exactly here;
//   3. the `keep` values nearest a_m (np.argsort(row)[:beta] with Python slice
//      semantics: keep = min(beta, theta) for beta >= 0, max(theta + beta, 0)
//      for beta < 0, e.g. N=100, f=30 keeps 20) form a contiguous window of
//      the sorted values, grown left on <= ties;
//   4. their mean, summed in that (distance) order with numpy's pairwise
//      scheme in fp64, is the output (float64, like the reference); keep = 0
//      is the mean of an empty slice (NaN).
//   A NaN among a coordinate's theta values makes every total distance NaN,
//   so the reference's argmin picks index 0: the centre is then the first
//   selected value, NaN distances sort last, and the result is NaN only when
//   a NaN is among the kept values.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "sra_common.hpp"

namespace sra {

int launch_krum(const float* X, int n, int64_t d, int64_t ldx, int f, int rounds, int* order, float* scores0,
                void* ws, size_t ws_bytes, hipStream_t s);
size_t krum_workspace_bytes(int n, int64_t d);

enum BulyanMode { kBulyanKrum = 0, kBulyanMedian = 1, kBulyanTrimmed = 2 };

// ---------------------------------------------------------------------------
// k-select over a device row list (median / trimmed mean of the remaining set)
// ---------------------------------------------------------------------------
__device__ __forceinline__ const char* uniform_ptr(const char* p) {
  const uint64_t r = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r >> 32));
  return reinterpret_cast<const char*>((static_cast<uint64_t>(hi) << 32) | lo);
}

// Row indices taken from device row lists (by readlane from the list held in
// VGPRs, or loaded) go through checked_row (sra_common.hpp): round 2's one GPU
// fault was a readlane of a register slot the compiler had written under a
// partial exec mask.
unsigned int bulyan_row_faults(bool reset) { return tu_row_faults(reset); }

__device__ __forceinline__ float ld_lane(const char* row, unsigned off) {
  typedef const __attribute__((address_space(1))) float gfloat;
  return __builtin_nontemporal_load(reinterpret_cast<gfloat*>(reinterpret_cast<uint64_t>(row) + off));
}

// One round of the median / trimmed-mean modes as ONE pass over the remaining
// rows (robust_estimator.py:297-322).  Per 256-coordinate block tile:
//   1. each wave loads the column of every listed row (one lane per
//      coordinate; row bases formed per tile as one 64-bit pointer per lane
//      and broadcast by two readlanes, fetched two rows ahead of their load)
//      and runs the k-select network -> the round's aggregate for its 64
//      coordinates (written out: it is the t-th selected vector);
//   2. the listed rows' columns go, 32 rows at a time, into an LDS tile (from
//      the step-1 copy in LDS or registers, or re-read: L2 / Infinity Cache
//      lines, all re-reads issued at once), read back transposed -- lanes l
//      and l + 32 hold row l's two 32-coordinate halves -- and each row's
//      squared distance over the wave's 64 coordinates is an in-order fp32
//      fma chain of (agg - x)^2 per half plus one cross-half add;
//   3. the block's four waves are added in order (fp32), into a per-block,
//      per-row partial; bulyan_dist_reduce_kernel sums the blocks in order in
//      fp64.  Deterministic for a given d (sharded or not: a shard's dist is
//      its own columns' share).
// Blocks take runs of consecutive tiles (one tile each up to d = 16.7M), so
// the partial table is at most kRoundMaxBlocks x n floats.
// Round 6 (C3, N = 128, f = 20, d = 1e7; profiles/r06_bulyan_rounds_ab.txt):
// per-round kernel 1.82 -> 1.45 ms at P = 128 (trimmed mean), 1.53 -> 1.40
// (median).  PMC before the change: VALU ~55-60 % busy, as many scalar
// instructions as vector ones (the per-row index, clamp and 64-bit multiply,
// twice), and four cache-latency waits per tile in step 2.
constexpr int kRoundMaxBlocks = 65536;

// Where step 2 takes each listed row's column from (template KL, KU):
//   rows [0, KL)   copied into this wave's LDS tile in step 1 (KL = 0 or >= 32);
//   rows [KL, KU)  kept in VGPRs across the network;
//   rows [KU, P)   re-read (L2 / Infinity Cache).
// Step 2 stages every row that is not already in LDS at tile row r % 32 (the
// first 32 rows' slots, consumed by then), then reads the tile transposed and
// forms res - x there: the same fp32 operations in the same order whatever
// the split, so the distances do not depend on it.  W: waves per SIMD.
template <int P, int MODE, int KL, int KU, int W>  // MODE: 0 median, 1 trimmed; n in (P-16, P] (P=16: 1..16)
__global__ void __launch_bounds__(256, W) select_dist_rows_kernel(const float* __restrict__ X, int64_t ldx,
                                                               const int* __restrict__ rows, int nrows_x, int n_arg,
                                                               int64_t d,
                                                               int lo, int hi, int nan_all, float* __restrict__ out,
                                                               float* __restrict__ bpart, int nb, int tpb) {
  constexpr int P2 = next_pow2(P);
  const unsigned t = threadIdx.x;
  const unsigned lane = t & 63u;
  const unsigned w = t >> 6;
  // the row list in VGPRs (lane l holds rows[l], rows[64 + l], ...): each
  // row index is then a readlane, not a dependent scalar load per row
  // -- as 64-bit byte offsets (row * ldx * 4, the row checked and clamped
  // once here): a row's base is then two readlanes and one 64-bit scalar add
  // per tile (the index, clamp and multiply per row and pass were ~12 scalar
  // instructions and a branch each, as many as the network's VALU work)
  // (formed per tile from the list: nothing but the list pointer stays live
  // across tiles, which the 256-VGPR copy variants need)
  constexpr int RW = (P + 63) / 64;
  static_assert(KL == 0 || (KL >= 32 && KL <= P), "LDS copy rows");
  static_assert(KU == 0 || (KU >= KL && KU <= P), "register copy rows");
  constexpr int KR = KL > 32 ? KL : 32;
  __shared__ float dl[4][KR][68];   // row stride 68 words: the transposed b128 reads spread over the banks
  __shared__ float rsl[4][64];      // the round's aggregate of each wave's 64 coordinates
  __shared__ float wsum[4][P];
  float bs = 0.f;
  const int n_out = n_arg;
  const int64_t ntiles = cdiv(d, 256);
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * tpb;
  const int64_t t1 = t0 + tpb < ntiles ? t0 + tpb : ntiles;
  for (int64_t tile = t0; tile < t1; ++tile) {
    const int64_t base = tile * 256;
    const int64_t rem = d - base;
    const unsigned last = rem < 256 ? static_cast<unsigned>(rem - 1) : 255u;
    const unsigned off = (t < last ? t : last) * 4u;
    // this tile's row bases, one per lane (per tile: hoisted out of the tile
    // loop they would be held, spilled, across it)
    const uint64_t xa = reinterpret_cast<uint64_t>(X + base);
    uint32_t plo[RW], phi[RW];
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      const int li = 64 * q + static_cast<int>(lane);
      const int row = checked_row(rows[li < n_arg ? li : n_arg - 1], nrows_x);
      const uint64_t pa = xa + static_cast<uint64_t>(row) * static_cast<uint64_t>(ldx) * 4u;
      plo[q] = static_cast<uint32_t>(pa);
      phi[q] = static_cast<uint32_t>(pa >> 32);
    }
    // n per tile as well: the ~2P row-count conditions (64-bit masks) would
    // otherwise be hoisted and spilled to VGPR lanes (a v_readlane each)
    int n = n_arg;
    asm volatile("" : "+s"(n));
    const int k_bottom = MODE == 0 ? (P - n) / 2 : 0;
    // row i's base (two readlanes into an SGPR pair, opaque: the second pass
    // recomputes it -- kept from the first pass, the 128 64-bit bases would be
    // held in spilled SGPRs across the network -- and the address stays an
    // SGPR base + the lane's offset)
    auto rowptr = [&](int i) -> uint64_t {
      const uint32_t lo32 = __builtin_amdgcn_readlane(plo[i / 64], i % 64);
      const uint32_t hi32 = __builtin_amdgcn_readlane(phi[i / 64], i % 64);
      uint64_t rp = (static_cast<uint64_t>(hi32) << 32) | lo32;
      asm volatile("" : "+s"(rp));
      return rp;
    };
    // default cache policy (not nt): step 2 re-reads these lines.  A/B at
    // N=128, d=1e7: 2.06 ms (default) vs 2.14 (nt) per P=128 round; keeping
    // an unsorted copy in registers instead (AGPR-backed): 2.63 ms
    auto ldp = [&](uint64_t rp) -> float {
      typedef const __attribute__((address_space(1))) float gfloat;
      return *reinterpret_cast<gfloat*>(rp + off);   // global_load, SGPR base
    };
    // rows [first, first + count) in order, each base read two rows ahead of
    // its load (a readlane-written SGPR read by the load right away costs a
    // 5-cycle s_nop per row)
    auto load_rows = [&](auto&& put, auto first_c, auto count_c) {
      constexpr int first = decltype(first_c)::value, count = decltype(count_c)::value;
      if constexpr (count > 0) {
        uint64_t pa = rowptr(first);
        uint64_t pb = count > 1 ? rowptr(first + 1) : 0;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < count; ++k) {
          const uint64_t pc = k + 2 < count ? rowptr(first + k + 2) : 0;
          __builtin_amdgcn_sched_barrier(0);
          put(first + k, ldp(pa));
          __builtin_amdgcn_sched_barrier(0);
          pa = pb;
          pb = pc;
        }
      }
    };
    constexpr int kFirstPad = P > 16 ? P - 16 : 0;   // rows below this are always real (n > P - 16)
    float v[P2];
    // lane i % 64 of block i / 64 holds rows[min(i, n - 1)] (clamped above);
    // slots past n are padded
    load_rows([&](int i, float x) { v[i] = x; }, std::integral_constant<int, 0>{}, std::integral_constant<int, P>{});
    // after every load is in flight (a select right behind its load would
    // wait for it there)
#pragma unroll
    for (int i = kFirstPad; i < P; ++i) {
      const float pad = (i - n < k_bottom) ? -__builtin_inff() : __builtin_inff();
      v[i] = i < n ? v[i] : pad;
    }
    const bool valid = t < rem;   // lanes past d contribute 0 to the distances
    // the unsorted column for step 2: rows [0, KL) into LDS (zero past d),
    // rows [KL, KU) stay in registers
    if constexpr (KL > 0) {
#pragma unroll
      for (int i = 0; i < KL; ++i) dl[w][i][lane] = v[i];
      if (rem < 256 && !valid) {   // ragged last tile only
#pragma unroll
        for (int i = 0; i < KL; ++i) dl[w][i][lane] = 0.f;
      }
    }
    constexpr int NU = KU > KL ? KU - KL : 0;
    float u[NU > 0 ? NU : 1];
#pragma unroll
    for (int i = 0; i < NU; ++i) u[i] = v[KL + i];
    // NaN detection over all slots (pads are +-inf, never NaN)
    float m = v[0];
#pragma unroll
    for (int i = 1; i < P; ++i) m = __builtin_elementwise_maximum(m, v[i]);
    int nan_cnt = 0;
    if (__builtin_amdgcn_ballot_w64(__builtin_isnan(m)) != 0) {
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const bool isn = __builtin_isnan(v[i]);
        nan_cnt += isn ? 1 : 0;
        v[i] = isn ? __builtin_inff() : v[i];
      }
    }
    float res;
    if constexpr (MODE == 0) {
      network_fast<P2, P, P / 2 - 1, P / 2 + 1>(v);
      res = (n & 1) ? v[P / 2 - 1] : (v[P / 2 - 1] + v[P / 2]) * 0.5f;
      if (nan_cnt > 0) res = qnan();
    } else {
      // lo = int(0.1 n), hi = n - lo over n in (P-16, P]: the kept window is
      // always inside [int(0.1 (P-15)), P - int(0.1 P)) -> prune the cone to it
      constexpr int OLO = (P > 16 ? P - 15 : 1) / 10;
      constexpr int OHI = P - P / 10;
      network_fast<P2, P, OLO, OHI>(v);
      // lo / hi re-materialised per tile: hoisted out of the tile loop, the
      // ~100 per-slot conditions would be kept as SGPR masks (and spilled)
      int lo_t = lo, hi_t = hi;
      asm volatile("" : "+s"(lo_t), "+s"(hi_t));
      float acc_s = 0.f;
      // the trimmed mean's window, lo = int(0.1 n) <= A and hi = n - lo >= B
      // for every n in (P - 16, P]: slots [A, B) are always summed, only the
      // edges are conditional, and an edge slot outside the window adds -0
      // (x + -0 == x for every x: the sum is bit-identical).  Any other
      // window (the DBA lower median is one slot) takes the general loop.
      constexpr int A = P / 10;
      constexpr int B = (P > 16 ? P - 15 : 1) - (P > 16 ? P - 15 : 1) / 10;
      if (lo_t <= A && hi_t >= B) {
#pragma unroll
        for (int p = OLO; p < A; ++p) acc_s += p >= lo_t ? v[p] : -0.0f;
#pragma unroll
        for (int p = A; p < B; ++p) acc_s += v[p];
#pragma unroll
        for (int p = B > A ? B : A; p < OHI; ++p) acc_s += p < hi_t ? v[p] : -0.0f;
      } else {
#pragma unroll
        for (int p = OLO; p < OHI; ++p) {
          if (p >= lo_t && p < hi_t) {
            asm volatile("");
            acc_s += v[p];
          }
        }
      }
      res = acc_s / static_cast<float>(hi - lo);
      // NaN sorts last (torch.sort / np.sort): the window sees it when it
      // reaches past n - hi; torch.median (nan_all, the DBA lower median)
      // propagates any NaN
      if (nan_cnt > (nan_all ? 0 : n - hi)) res = qnan();
    }
    if (t < rem) out[base + t] = res;
    // step 2: squared distances of the listed rows over this wave's 64 coordinates
    rsl[w][lane] = valid ? res : 0.f;
    // fresh copies of the row list: the first pass's 128 readlane results
    // (SGPRs) must not stay live across the network
#pragma unroll
    for (int q = 0; q < RW; ++q) asm volatile("" : "+v"(plo[q]), "+v"(phi[q]));
    // every re-read in flight at once, before the first chunk (the network's
    // registers are free now): one cache latency per tile instead of one per
    // chunk.  Rows past n are clamped copies of row n - 1 (sums never read).
    constexpr int NR = P - (KU > KL ? KU : KL);
    float xr[NR > 0 ? NR : 1];
    load_rows([&](int i, float x) { xr[i - (P - NR)] = x; }, std::integral_constant<int, P - NR>{},
              std::integral_constant<int, NR>{});
    const unsigned ti = lane & 31u, th = lane >> 5;
#pragma unroll
    for (int c = 0; c < RW * 2; ++c) {
      if (32 * c >= n) break;   // wave-uniform
      constexpr int kChunkRows = 32;
#pragma unroll
      for (int i = 0; i < kChunkRows; ++i) {
        const int r = 32 * c + i;
        if (r < P && r >= KL) dl[w][i][lane] = r < P - NR ? u[r - KL] : xr[r - (P - NR)];
      }
      if (rem < 256 && !valid) {   // ragged last tile only: lanes past d add 0
#pragma unroll
        for (int i = 0; i < kChunkRows; ++i) {
          const int r = 32 * c + i;
          if (r < P && r >= KL) dl[w][i][lane] = 0.f;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int rr = 32 * c + static_cast<int>(ti);
      const int lrow = rr < KL ? rr : static_cast<int>(ti);
      float sh = 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(&dl[w][lrow][32 * th + 4 * u]);
        const f32x4 a = *reinterpret_cast<const f32x4*>(&rsl[w][32 * th + 4 * u]);
        const float q0 = a[0] - x[0], q1 = a[1] - x[1], q2 = a[2] - x[2], q3 = a[3] - x[3];
        sh = __builtin_fmaf(q0, q0, sh);
        sh = __builtin_fmaf(q1, q1, sh);
        sh = __builtin_fmaf(q2, q2, sh);
        sh = __builtin_fmaf(q3, q3, sh);
      }
      const float so = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(static_cast<int>((lane ^ 32u) * 4u),
                                                                              __builtin_bit_cast(int, sh)));
      const float st = th == 0 ? sh + so : so + sh;   // same value in both halves
      if (th == 0 && 32 * c + static_cast<int>(ti) < n) wsum[w][32 * c + ti] = st;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();   // dl is rewritten by the next chunk only after every lane read it
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
    if (static_cast<int>(t) < n) bs += (wsum[0][t] + wsum[1][t]) + (wsum[2][t] + wsum[3][t]);
    __syncthreads();   // wsum / dl reuse by the next tile
  }
  if (static_cast<int>(t) < n_out) bpart[static_cast<int64_t>(t) * nb + blockIdx.x] = bs;
}

// dist[r] = the per-block partials of listed row r summed in fp64 in a fixed
// order: strided chains per thread, then a fixed tree
__global__ void __launch_bounds__(256) bulyan_dist_reduce_kernel(const float* __restrict__ bpart, int nb,
                                                                 double* __restrict__ dist) {
  const int r = blockIdx.x;
  const float* p = bpart + static_cast<int64_t>(r) * nb;
  // eight independent strided chains per thread (loads in flight), combined
  // in a fixed order
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int g = threadIdx.x;
  for (; g + 7 * 256 < nb; g += 8 * 256) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += static_cast<double>(p[g + 256 * u]);
  }
  for (; g < nb; g += 256) a[0] += static_cast<double>(p[g]);
  double s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < static_cast<unsigned>(k)) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) dist[r] = red[0];
}

static int64_t round_tiles_per_block(int64_t d) { return cdiv(cdiv(d, 256), kRoundMaxBlocks); }
static int64_t round_blocks(int64_t d) { return cdiv(cdiv(d, 256), round_tiles_per_block(d)); }
static size_t round_partial_bytes(int n, int64_t d) {
  return sizeof(float) * static_cast<size_t>(n) * static_cast<size_t>(round_blocks(d));
}

// argmin (first strict minimum, NaN never chosen) of the listed rows'
// distances; removes it from the list (order preserved) into rows_next.
__global__ void __launch_bounds__(256) bulyan_pick_kernel(const double* __restrict__ dist, const int* __restrict__ rows,
                                                         int nr, int* __restrict__ rows_next, int* __restrict__ status,
                                                         int* __restrict__ picked = nullptr) {
  __shared__ int pick;
  if (threadIdx.x == 0) {
    int best = -1;
    double bv = __builtin_inf();
    for (int r = 0; r < nr; ++r) {
      // the reference compares fp32 norms: sqrt is monotone, compare squares
      if (dist[r] < bv) { bv = dist[r]; best = r; }
    }
    pick = best;
    if (best < 0 && status) *status = 1;  // AssertionError in the reference (all NaN / inf)
  }
  __syncthreads();
  const int p = pick < 0 ? 0 : pick;
  if (picked != nullptr && threadIdx.x == 0) *picked = rows[p];
  for (int r = threadIdx.x; r < nr - 1; r += blockDim.x) rows_next[r] = rows[r < p ? r : r + 1];
}

// ---------------------------------------------------------------------------
// Rounds with more than 128 remaining clients (N up to kBigMaxClients): two
// passes per round instead of the fused one.
//   select_rows_lds_kernel: a tile of `tile` coordinates x pn slots (pn =
//     next_pow2(nr), [slot][coordinate] so a wave's compare-exchanges hit
//     distinct banks) filled through the row list, bitonic-sorted by the
//     whole workgroup (NaN-last order, padding NaN), then one lane per
//     coordinate forms the round's aggregate exactly as the register kernel
//     does (numpy's median / the ascending sequential fp32 window sum).
//   dist_rows_kernel: the listed rows' squared distances to that aggregate
//     with the fused kernel's arithmetic -- fp32 fma chains over the two
//     32-coordinate halves of each wave, the four waves added in order, fp32
//     across a block's tiles, the same per-block partial table for
//     bulyan_dist_reduce_kernel -- so the pick sees the same distances
//     whichever path a round took.
// Row indices are clamped to the matrix (a bad list cannot fault).
// ---------------------------------------------------------------------------
constexpr int kBigMaxClients = 8192;   // as Krum (krum.hip kKrumMaxClients)
constexpr int kBigLdsFloats = 16384;   // 64 KiB tile
constexpr int kDistRowGroup = 1024;    // dist_rows_kernel<4>: rows per launch above 512

__global__ void __launch_bounds__(256) select_rows_lds_kernel(const float* __restrict__ X, int64_t ldx,
                                                              const int* __restrict__ rows, int nrows_x, int n, int pn,
                                                              int tile, int64_t d, int median, int lo, int hi,
                                                              int nan_all, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * tile;
  const int tid = threadIdx.x;
  const int lt = __builtin_ctz(static_cast<unsigned>(tile));
  for (int e = tid; e < pn * tile; e += blockDim.x) {
    const int r = e >> lt, c = e & (tile - 1);   // tile: a power of two
    const int64_t j = j0 + c;
    float x = qnan();
    if (r < n && j < d) {
      x = X[static_cast<int64_t>(checked_row(rows[r], nrows_x)) * ldx + j];
    }
    lds[e] = x;
  }
  __syncthreads();
  const int pairs = (pn / 2) * tile;
  for (int k = 2; k <= pn; k <<= 1) {
    for (int s = k >> 1; s > 0; s >>= 1) {
      for (int q = tid; q < pairs; q += blockDim.x) {
        const int c = q & (tile - 1);
        const int h = q >> lt;
        const int i = h + (h & ~(s - 1));   // (h / s) * 2s + h % s, s a power of two
        const int l = i + s;
        float a = lds[i * tile + c], b = lds[l * tile + c];
        if ((i & k) == 0) ce(a, b); else ce(b, a);
        lds[i * tile + c] = a;
        lds[l * tile + c] = b;
      }
      __syncthreads();
    }
  }
  if (tid < tile) {
    const int64_t j = j0 + tid;
    if (j < d) {
      float res;
      if (median) {   // np.median: NaN anywhere -> NaN (NaN sorts last, so slot n-1 is NaN)
        if (n & 1) res = lds[((n - 1) / 2) * tile + tid];
        else res = (lds[(n / 2 - 1) * tile + tid] + lds[(n / 2) * tile + tid]) * 0.5f;
        if (__builtin_isnan(lds[(n - 1) * tile + tid])) res = qnan();
      } else {        // window [lo, hi) of the sorted column, summed in ascending order
        float acc = 0.f;
        for (int p = lo; p < hi; ++p) acc += lds[p * tile + tid];
        res = acc / static_cast<float>(hi - lo);
        if (nan_all && __builtin_isnan(lds[(n - 1) * tile + tid])) res = qnan();   // torch.median
      }
      out[j] = res;
    }
  }
}

template <int MAXR>   // rows per thread-slot bound: nr <= 256 * MAXR
__global__ void __launch_bounds__(256) dist_rows_kernel(const float* __restrict__ X, int64_t ldx,
                                                        const int* __restrict__ rows, int nrows_x, int nr, int64_t d,
                                                        const float* __restrict__ agg, float* __restrict__ bpart,
                                                        int nb, int tpb) {
  const unsigned t = threadIdx.x;
  const unsigned lane = t & 63u;
  const unsigned w = t >> 6;
  __shared__ float dl[4][32][68];
  __shared__ float wsum[4][256 * MAXR];
  float bs[MAXR];
#pragma unroll
  for (int q = 0; q < MAXR; ++q) bs[q] = 0.f;
  const int64_t ntiles = cdiv(d, 256);
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * tpb;
  const int64_t t1 = t0 + tpb < ntiles ? t0 + tpb : ntiles;
  const unsigned ti = lane & 31u, th = lane >> 5;
  for (int64_t tile = t0; tile < t1; ++tile) {
    const int64_t base = tile * 256;
    const int64_t rem = d - base;
    const bool valid = static_cast<int64_t>(t) < rem;
    const int64_t j = valid ? base + t : d - 1;
    const float a = agg[j];
    for (int c = 0; 32 * c < nr; ++c) {
      // this chunk's 32 row indices, loaded by the whole wave (full exec) and
      // broadcast by readlane right here
      const int li = 32 * c + static_cast<int>(lane & 31u);
      const int rv = rows[li < nr ? li : nr - 1];
      float xs[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const int row = checked_row(__builtin_amdgcn_readlane(rv, i), nrows_x);
        xs[i] = X[static_cast<int64_t>(row) * ldx + j];
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) dl[w][i][lane] = valid ? a - xs[i] : 0.f;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float sh = 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(&dl[w][ti][32 * th + 4 * u]);
        sh = __builtin_fmaf(q[0], q[0], sh);
        sh = __builtin_fmaf(q[1], q[1], sh);
        sh = __builtin_fmaf(q[2], q[2], sh);
        sh = __builtin_fmaf(q[3], q[3], sh);
      }
      const float so = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(static_cast<int>((lane ^ 32u) * 4u),
                                                                              __builtin_bit_cast(int, sh)));
      const float st = th == 0 ? sh + so : so + sh;
      if (th == 0 && 32 * c + static_cast<int>(ti) < nr) wsum[w][32 * c + ti] = st;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < MAXR; ++q) {
      const int r = static_cast<int>(t) + 256 * q;
      if (r < nr) bs[q] += (wsum[0][r] + wsum[1][r]) + (wsum[2][r] + wsum[3][r]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < MAXR; ++q) {
    const int r = static_cast<int>(t) + 256 * q;
    if (r < nr) bpart[static_cast<int64_t>(r) * nb + blockIdx.x] = bs[q];
  }
}

// ---------------------------------------------------------------------------
// per-coordinate Bulyan stage
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// The per-coordinate stage by definition, O(theta^2) per lane and no sort:
//   T_i  = numpy pairwise fp64 sum of the distance row i (|a_i - a_k|, diagonal
//          0 as np.zeros leaves it); m = np.argmin(T): the first NaN if any,
//          else the first strict minimum;
//   row  = distances[m]; argsort(row)[:beta] keeps `keep` values (slice
//          semantics), NaN distances last, equal distances smaller value first
//          (the left-first rule of the fast path), then index;
//   res  = their numpy pairwise mean in that order.
// Serves the drop-in's scalar helpers (any float64 input) and the columns of
// the fused stage that hold a NaN or an infinity (NaN anywhere makes every T
// NaN -> m = 0; one infinity makes every T infinite -> m = 0; two equal
// infinities are at NaN distance -> m = the first of them).  `slot(p)` is
// per-lane scratch for the rank -> value-index map.
// ---------------------------------------------------------------------------
// DEEP: theta may exceed 512 (the N > 512 stage and the scalar helpers), so
// the pairwise sums take numpy's split to seven levels there (exact to 16368).
template <int DEPTH, typename F>
__device__ __attribute__((noinline)) double np_pw64_deep(int lo, int n, F f) {
  if constexpr (DEPTH == 0) {
    return np_pw_block64(n, [&](int i) { return f(lo + i); });
  } else {
    if (n <= 128) return np_pw_block64(n, [&](int i) { return f(lo + i); });
    int q = n / 2;
    q -= q % 8;
    const double l = np_pw64_deep<DEPTH - 1>(lo, q, f);
    return l + np_pw64_deep<DEPTH - 1>(lo + q, n - q, f);
  }
}

template <bool DEEP = false, typename A, typename Slot>
__device__ double bulyan_stage_generic(A&& a, int theta, int keep, Slot&& slot, int* m_out) {
  auto pw = [&](int n, auto&& g) -> double {
    if constexpr (DEEP) {
      if (n > 512) return np_pw64_deep<7>(0, n, g);
    }
    return np_pw64(0, n, g);
  };
  int m = 0;
  double best = 0.0;
  for (int i = 0; i < theta; ++i) {
    const double ai = a(i);
    const double T = pw(theta, [&](int k) { return k == i ? 0.0 : __builtin_fabs(ai - a(k)); });
    if (__builtin_isnan(T)) {
      m = i;
      break;
    }
    if (i == 0 || T < best) {
      best = T;
      m = i;
    }
  }
  *m_out = m;
  const double am = a(m);
  auto dist = [&](int k) -> double { return k == m ? 0.0 : __builtin_fabs(am - a(k)); };
  auto before = [&](int q, int k) -> bool {
    const double dq = dist(q), dk = dist(k);
    const bool nq = __builtin_isnan(dq), nk = __builtin_isnan(dk);
    if (nq != nk) return nk;
    if (!nq && dq != dk) return dq < dk;
    if (!nq) {
      const double vq = a(q), vk = a(k);
      if (vq != vk) return vq < vk;
    }
    return q < k;
  };
  for (int k = 0; k < theta; ++k) {
    int r = 0;
    for (int q = 0; q < theta; ++q) r += (q != k && before(q, k)) ? 1 : 0;
    slot(r) = k;
  }
  if (keep <= 0) return __builtin_nan("");
  return pw(keep, [&](int p) { return a(slot(p)); }) / static_cast<double>(keep);
}

// numpy's pairwise fp64 sum (np_pw_block64) of f(0..n) for n in (P - 16, P],
// unrolled over static indices so that f may read registers; n is wave-uniform
template <int P, typename F>
__device__ __forceinline__ double np_pw_static64(int n, F&& f) {
  static_assert(P <= 128, "one pairwise block");
  if (n < 8) {
    double res = 0.0;
#pragma unroll
    for (int i = 0; i < (P < 8 ? P : 8); ++i)
      if (i < n) res += f(i);
    return res;
  }
  const int nb = n - (n % 8);
  double r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = f(k);
#pragma unroll
  for (int i = 8; i + 8 <= P; i += 8)
    if (i < nb) {
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] += f(i + k);
    }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
  for (int i = (P > 16 ? P - 16 : 8); i < P; ++i)
    if (i >= nb && i < n) res += f(i);
  return res;
}

// The mean of the keep values nearest the centre c = s(p0) of a sorted column
// (s(p), p < theta), for a column whose partial sums are all exact in fp64:
// the order of summation is then immaterial, and the window is
// [pl - a, pr + k - a] around the run [pl, pr] of values equal to c, with a
// found by bisection (left element i is taken iff the (k - i + 1)-th right
// element is not strictly nearer: robust_estimator.py:272-275 takes the run
// first, then grows left on <= ties).
template <typename Col>
__device__ double bulyan_window_mean(Col&& s, int theta, int keep, int p0) {
  const double c = s(p0);
  int pl = p0, pr = p0;
  while (pl > 0 && static_cast<double>(s(pl - 1)) == c) --pl;
  while (pr + 1 < theta && static_cast<double>(s(pr + 1)) == c) ++pr;
  const int run = pr - pl + 1;
  if (keep <= run) return c;   // keep copies of c
  const int k = keep - run, nl = pl, nr = theta - 1 - pr;
  int lo = k - nr > 0 ? k - nr : 0, hi = k < nl ? k : nl;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int jr = k - mid + 1;
    const bool taken = jr > nr || static_cast<double>(s(pr + jr)) - c >= c - static_cast<double>(s(pl - mid));
    if (taken) lo = mid;
    else hi = mid - 1;
  }
  // every partial sum is exact (the caller's span test), so the window is
  // summed as four independent chains: the order is immaterial
  double a0 = static_cast<double>(run) * c, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  const int w0 = pl - lo, w1 = pr + k - lo;   // the window minus the run: [w0, pl) and (pr, w1]
  int p = w0;
  for (; p + 3 < pl; p += 4) {
    a0 += static_cast<double>(s(p));
    a1 += static_cast<double>(s(p + 1));
    a2 += static_cast<double>(s(p + 2));
    a3 += static_cast<double>(s(p + 3));
  }
  for (; p < pl; ++p) a0 += static_cast<double>(s(p));
  p = pr + 1;
  for (; p + 3 <= w1; p += 4) {
    a0 += static_cast<double>(s(p));
    a1 += static_cast<double>(s(p + 1));
    a2 += static_cast<double>(s(p + 2));
    a3 += static_cast<double>(s(p + 3));
  }
  for (; p <= w1; ++p) a1 += static_cast<double>(s(p));
  return ((a0 + a1) + (a2 + a3)) / static_cast<double>(keep);
}

constexpr int kFinalMaxTheta = 128;

// value v[i] of a register array at a wave-uniform runtime index i in
// [(P - 16) / 2 - 1, P / 2] (theta in (P - 16, P]): a select chain; the empty
// asm keeps the optimiser from folding it back into an indexed (scratch) load
template <int P, int P2>
__device__ __forceinline__ float pick_hi(const float (&v)[P2], int i) {   // i in [P - 16, P)
  float r = v[P - 1];
#pragma unroll
  for (int q = (P > 16 ? P - 16 : 0); q < P - 1; ++q) {
    r = i == q ? v[q] : r;
    asm volatile("" : "+v"(r));
  }
  return r;
}
template <int P, int P2>
__device__ __forceinline__ float pick_mid(const float (&v)[P2], int i) {
  constexpr int lo = (P > 16 ? (P - 16) / 2 - 1 : 0);
  float r = v[P / 2];
#pragma unroll
  for (int q = lo; q < P / 2; ++q) {
    r = i == q ? v[q] : r;
    asm volatile("" : "+v"(r));
  }
  return r;
}

// Columns the final kernel lists, entry = 2 j + kind:
//   kind 1 -- a NaN or an infinity among the values: the per-coordinate stage
//             by definition (bulyan_stage_generic), LDS rank scratch;
//   kind 0 -- finite, but the magnitude span lets fp64 rounding decide: the
//             centre from numpy's pairwise totals of the two middle values
//             (first index on a tie), then the window walked in argsort order
//             (run first, grow left on <= ties) and summed with numpy's
//             eight-accumulator scheme, as robust_estimator.py:259-275 does.
// One lane per listed column, any number of columns per lane (the count is
// only known on the device); a few per million columns in practice.
template <int P>
__global__ void __launch_bounds__(64) bulyan_listed_kernel(const float* __restrict__ S, int64_t lds_,
                                                           const int* __restrict__ rows, int nrows_s, int theta,
                                                           int keep,
                                                           const int* __restrict__ nf_count,
                                                           const int64_t* __restrict__ nf_list,
                                                           double* __restrict__ out) {
  constexpr int P2 = next_pow2(P);
  __shared__ float col[P][64];
  const int t = threadIdx.x;
  const int cnt = *nf_count;
  for (int e = blockIdx.x * 64 + t; e < cnt; e += gridDim.x * 64) {
    const int64_t j = nf_list[e] >> 1;
    auto a = [&](int i) -> float { return S[static_cast<int64_t>(checked_row(rows[i], nrows_s)) * lds_ + j]; };
    if (nf_list[e] & 1) {
      int m;
      out[j] = keep == 0 ? __builtin_nan("")
                         : bulyan_stage_generic([&](int i) -> double { return a(i); }, theta, keep,
                                                [&](int p) -> int& { return *reinterpret_cast<int*>(&col[p][t]); },
                                                &m);
      continue;
    }
    if (keep == 0) {
      out[j] = __builtin_nan("");
      continue;
    }
    float o[P2], v[P2];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      o[i] = i < theta ? a(i) : __builtin_inff();
      v[i] = o[i];
    }
    network_fast<P2, P, 0, P>(v);
#pragma unroll
    for (int i = 0; i < P; ++i) col[i][t] = v[i];
    double am;
    if (theta & 1) {
      am = col[(theta - 1) / 2][t];
    } else {
      const float L = col[theta / 2 - 1][t], U = col[theta / 2][t];
      if (L == U) {
        am = L;
      } else {
        const double TL = np_pw_static64<P>(theta, [&](int i) { return __builtin_fabs(static_cast<double>(L) - o[i]); });
        const double TU = np_pw_static64<P>(theta, [&](int i) { return __builtin_fabs(static_cast<double>(U) - o[i]); });
        int fl = theta, fu = theta;
#pragma unroll
        for (int i = P - 1; i >= 0; --i) {
          fl = o[i] == L ? i : fl;
          fu = o[i] == U ? i : fu;
        }
        am = (TL < TU || (TL == TU && fl < fu)) ? L : U;
      }
    }
    // run of values equal to am in the sorted column, then the walk
    int pl = (theta - 1) / 2;
    while (pl > 0 && static_cast<double>(col[pl][t]) > am) --pl;
    while (pl < theta - 1 && static_cast<double>(col[pl][t]) < am) ++pl;
    while (pl > 0 && static_cast<double>(col[pl - 1][t]) == am) --pl;
    int pr = pl;
    while (pr + 1 < theta && static_cast<double>(col[pr + 1][t]) == am) ++pr;
    int l = pl, r = pr, taken = 0;
    auto next = [&]() -> double {
      if (taken < pr - pl + 1) {
        ++taken;
        return am;
      }
      const double dl = l > 0 ? am - static_cast<double>(col[l - 1][t]) : __builtin_inf();
      const double dr = r < theta - 1 ? static_cast<double>(col[r + 1][t]) - am : __builtin_inf();
      ++taken;
      if (dl <= dr) {
        --l;
        return static_cast<double>(col[l][t]);
      }
      ++r;
      return static_cast<double>(col[r][t]);
    };
    double res;
    if (keep < 8) {
      res = 0.0;
      for (int i = 0; i < keep; ++i) res += next();
    } else {
      double r0 = next(), r1 = next(), r2 = next(), r3 = next(), r4 = next(), r5 = next(), r6 = next(), r7 = next();
      int i = 8;
      for (; i < keep - (keep % 8); i += 8) {
        r0 += next(); r1 += next(); r2 += next(); r3 += next();
        r4 += next(); r5 += next(); r6 += next(); r7 += next();
      }
      res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
      for (; i < keep; ++i) res += next();
    }
    out[j] = res / static_cast<double>(keep);
  }
}

// Four waves per block, one lane per coordinate.  The theta selected values
// are gathered in selection order (row indices broadcast from VGPRs by
// readlane) and sorted in registers.  The sorted column goes through ONE LDS
// tile per block that the four waves take in turn (a barrier per turn), so
// LDS does not cap the occupancy (round 1's per-wave tile allowed 6 waves per
// CU: 5.3 ms at theta = 88, d = 1e7).  In its turn a wave checks the column's
// magnitude span -- when every partial sum of values and of |differences| is
// exact in fp64 the result does not depend on summation order -- and finds
// the windows of the centre candidates by bisection.  The even-theta
// tie-break between the two middle values re-reads the column in selection
// order: their totals are then equal, so the first index holding either
// value decides, as np.argmin does.  Columns failing the span test, or
// holding a NaN or an infinity, go to bulyan_listed_kernel.
template <int P>  // theta in (P - 16, P]
__global__ void __launch_bounds__(256, P <= 96 ? 4 : 2) bulyan_final_kernel(const float* __restrict__ S, int64_t lds_,
                                                           const int* __restrict__ rows, int nrows_s, int theta,
                                                           int keep,
                                                           int64_t d, double* __restrict__ out,
                                                           int* __restrict__ nf_count, int64_t* __restrict__ nf_list) {
  constexpr int P2 = next_pow2(P);
  __shared__ float col[P][64];
  const int t = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 + wave * 64;
  const int64_t rem = d - base;   // may be <= 0 for the last block's trailing waves
  const int tl = rem <= 0 ? 0 : (t < rem ? t : static_cast<int>(rem - 1));
  const int64_t j = rem <= 0 ? d - 1 : base + tl;
  constexpr int RW = (P + 63) / 64;
  const int64_t jb = j - tl;   // this wave's first coordinate (clamped)
  const unsigned off = static_cast<unsigned>(tl) * 4u;
  // the selected rows' bases for this wave's coordinates, one 64-bit pointer
  // per lane (lane l: rows[64 q + l], checked and clamped once); a row's base
  // is then two readlanes, fetched two rows ahead of its load (see
  // select_dist_rows_kernel)
  uint32_t plo[RW], phi[RW];
  auto row_bases = [&]() __attribute__((always_inline)) {
    const uint64_t sa = reinterpret_cast<uint64_t>(S + jb);
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      const int li = 64 * q + t;
      const int row = checked_row(rows[li < theta ? li : theta - 1], nrows_s);
      const uint64_t pa = sa + static_cast<uint64_t>(row) * static_cast<uint64_t>(lds_) * 4u;
      plo[q] = static_cast<uint32_t>(pa);
      phi[q] = static_cast<uint32_t>(pa >> 32);
      asm volatile("" : "+v"(plo[q]), "+v"(phi[q]));
    }
  };
  row_bases();
  auto rowptr = [&](int i) -> uint64_t {
    const uint32_t lo32 = __builtin_amdgcn_readlane(plo[i / 64], i % 64);
    const uint32_t hi32 = __builtin_amdgcn_readlane(phi[i / 64], i % 64);
    uint64_t rp = (static_cast<uint64_t>(hi32) << 32) | lo32;
    asm volatile("" : "+s"(rp));
    return rp;
  };
  constexpr int kFirstPad = P > 16 ? P - 16 : 0;
  auto load_col = [&](float (&v)[P2], bool& nonfinite) __attribute__((always_inline)) {
    uint64_t pa = rowptr(0), pb = P > 1 ? rowptr(1) : 0;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const uint64_t pc = i + 2 < P ? rowptr(i + 2) : 0;
      __builtin_amdgcn_sched_barrier(0);
      v[i] = ld_lane(reinterpret_cast<const char*>(pa), off);
      __builtin_amdgcn_sched_barrier(0);
      pa = pb;
      pb = pc;
    }
    // after every load is in flight: rows below P - 16 always exist
    // (theta > P - 16), the rest are padded
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const bool real = i < kFirstPad || i < theta;
      nonfinite |= real && !__builtin_isfinite(v[i]);
      v[i] = real ? v[i] : __builtin_inff();
    }
  };

  const bool even = (theta & 1) == 0;
  float cl, cu;            // centre candidates: the two middle values (even theta) or the median (cl)
  bool nonfinite = false;
  {
    float v[P2];
    load_col(v, nonfinite);
    if (__builtin_amdgcn_ballot_w64(nonfinite) != 0) {
#pragma unroll
      for (int i = 0; i < P; ++i) v[i] = __builtin_isnan(v[i]) ? __builtin_inff() : v[i];
    }
    network_fast<P2, P, 0, P>(v);
    cl = pick_mid<P, P2>(v, even ? theta / 2 - 1 : (theta - 1) / 2);
    cu = pick_mid<P, P2>(v, theta / 2);
    // magnitude span: every value, |x - y| and partial sum of <= 128 of them
    // is a multiple of ulp(smallest nonzero |value|) below 256 max|value|;
    // exact in fp64 when that spans <= 53 bits.  |value| bits compare as
    // unsigned integers; the +inf padding never wins the minimum, and the
    // maximum magnitude is at one end of the sorted column.
    bool exact = true;   // all sums exact in fp64
    {
      unsigned mnb = 0xffffffffu;   // (smallest nonzero |value| bits) - 1
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const unsigned ab = (__builtin_bit_cast(unsigned, v[i]) & 0x7fffffffu) - 1u;   // 0 wraps: ignored
        mnb = ab < mnb ? ab : mnb;
      }
      const unsigned mxb = fmaxf(-v[0], pick_hi<P, P2>(v, theta - 1)) < 0.f
                               ? 0u : __builtin_bit_cast(unsigned, fmaxf(-v[0], pick_hi<P, P2>(v, theta - 1)));
      if (mnb != 0xffffffffu) {
        const int emx = static_cast<int>(mxb >> 23) - 126;   // max|x| < 2^emx
        const int ebn = static_cast<int>((mnb + 1u) >> 23);
        const int ulp = (ebn > 0 ? ebn : 1) - 150;          // ulp(min nonzero |x|) = 2^ulp
        exact = (emx + 8) - ulp <= 53;
      }
    }
    // this wave's turn with the LDS tile: wave w works between the block's
    // barriers w + 1 and w + 2 (every wave passes four), so the sorted values
    // are dead once stored and do not share registers with the window search
    double res_l = 0.0, res_u = 0.0;
#pragma unroll 1
    for (int w = 0; w <= wave; ++w) __syncthreads();
#pragma unroll
    for (int i = 0; i < P; ++i) col[i][t] = v[i];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    auto s = [&](int p) -> float { return col[p][t]; };
    if (keep == 0) {
      // the mean of an empty slice: NaN for every column, written below
    } else if (nonfinite) {
      // a NaN or an infinity changes which value is the centre (see
      // bulyan_stage_generic): listed for bulyan_listed_kernel
      if (rem > 0 && t < rem) nf_list[atomicAdd(nf_count, 1)] = 2 * j + 1;
    } else {
      if (exact) {
        res_l = bulyan_window_mean(s, theta, keep, even ? theta / 2 - 1 : (theta - 1) / 2);
        if (even && cu != cl) res_u = bulyan_window_mean(s, theta, keep, theta / 2);
      } else if (rem > 0 && t < rem) {
        // rounding decides the centre and the order of the sums
        nf_list[atomicAdd(nf_count, 1)] = 2 * j;
      }
    }
#pragma unroll 1
    for (int w = wave + 1; w < 4; ++w) __syncthreads();
    // no early return from here on: the tie-break's gather broadcasts row
    // indices across lanes (readlane), which must not read the register
    // slots of lanes that left (the compiler may have copied the row list
    // under a partial exec mask, leaving stale values there)
    bool write = rem > 0 && t < rem && (keep == 0 || (!nonfinite && exact));   // else listed for bulyan_listed_kernel
    double result = res_l;
    bool tie = false;
    if (keep == 0) result = __builtin_nan("");   // mean of an empty slice
    else if (even && cu != cl) tie = true;
    if (__builtin_amdgcn_ballot_w64(write && tie) != 0) {   // wave-uniform: every lane active
      // even theta, two distinct middle values: np.argmin over the totals.
      // The row list is reloaded here, with every lane active, and kept opaque
      // (the first gather's row addresses are then not held live for reuse)
      row_bases();
      float o[P2];
      bool dummy = false;
      load_col(o, dummy);
      int fl = theta, fu = theta;
#pragma unroll
      for (int i = P - 1; i >= 0; --i) {
        // padding slots hold +inf, never a (finite) centre value
        fl = o[i] == cl ? i : fl;
        fu = o[i] == cu ? i : fu;
      }
      // exact sums: the two totals are equal (the middle values split the
      // column in halves), so np.argmin takes the first index holding either
      if (tie) result = fl < fu ? res_l : res_u;
    }
    if (write) out[base + t] = result;
  }
}

// ---------------------------------------------------------------------------
// The stage for theta in (128, kBigMaxClients]: a TW-coordinate tile (TW = 64
// up to theta = 512, halved with every doubling of pn above) of pn =
// next_pow2(theta) slots in LDS per 256-thread block, filled in selection
// order through the row list, bitonic-sorted by the block; then one lane per
// coordinate runs the register kernel's logic on its sorted column: the
// exact-span test (every partial sum of <= theta values and |differences|
// exact in fp64: 2 theta max|x| / ulp(min nonzero |x|) <= 2^53), the windows
// of the centre candidates by bisection, the even-theta tie decided by the
// first selection-order index holding either middle value (re-read from
// global memory).  NaN / inf columns and inexact ones are listed for
// bulyan_listed_big_kernel (the stage by definition).
// ---------------------------------------------------------------------------
template <int TW>
__global__ void __launch_bounds__(256) bulyan_final_lds_kernel(const float* __restrict__ S, int64_t lds_,
                                                               const int* __restrict__ rows, int nrows_s, int theta,
                                                               int pn, int keep, int64_t d, double* __restrict__ out,
                                                               int* __restrict__ nf_count,
                                                               int64_t* __restrict__ nf_list) {
  static_assert(TW >= 1 && TW <= 64 && (TW & (TW - 1)) == 0, "tile width: a power of two <= 64");
  constexpr int LG = __builtin_ctz(TW);
  extern __shared__ __attribute__((aligned(16))) float colt[];   // [pn][TW]
  __shared__ unsigned mnb_s[64], mxb_s[64];
  __shared__ int nonfin_s[64];
  const int tid = threadIdx.x;
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * TW;
  if (tid < 64) {
    mnb_s[tid] = 0xffffffffu;
    mxb_s[tid] = 0u;
    nonfin_s[tid] = 0;
  }
  __syncthreads();
  for (int e = tid; e < pn * TW; e += blockDim.x) {
    const int p = e >> LG, c = e & (TW - 1);
    const int64_t j = j0 + c;
    float x = __builtin_inff();
    if (p < theta && j < d) {
      x = S[static_cast<int64_t>(checked_row(rows[p], nrows_s)) * lds_ + j];
      if (!__builtin_isfinite(x)) {
        atomicOr(&nonfin_s[c], 1);
        x = __builtin_isnan(x) ? __builtin_inff() : x;
      } else {
        const unsigned ab = __builtin_bit_cast(unsigned, x) & 0x7fffffffu;
        if (ab != 0u) atomicMin(&mnb_s[c], ab);
        atomicMax(&mxb_s[c], ab);
      }
    }
    colt[e] = x;
  }
  __syncthreads();
  const int pairs = (pn / 2) * TW;
  for (int k = 2; k <= pn; k <<= 1) {
    for (int s = k >> 1; s > 0; s >>= 1) {
      for (int q = tid; q < pairs; q += blockDim.x) {
        const int c = q & (TW - 1);
        const int h = q >> LG;
        const int i = h + (h & ~(s - 1));   // (h / s) * 2s + h % s, s a power of two
        const int l = i + s;
        float a = colt[i * TW + c], b = colt[l * TW + c];
        if ((i & k) == 0) ce(a, b); else ce(b, a);
        colt[i * TW + c] = a;
        colt[l * TW + c] = b;
      }
      __syncthreads();
    }
  }
  if (tid >= TW) return;
  const int64_t j = j0 + tid;
  if (j >= d) return;
  if (keep == 0) {   // the mean of an empty slice
    out[j] = __builtin_nan("");
    return;
  }
  if (nonfin_s[tid]) {
    nf_list[atomicAdd(nf_count, 1)] = 2 * j + 1;
    return;
  }
  bool exact = true;
  if (mnb_s[tid] != 0xffffffffu) {
    const int emx = static_cast<int>(mxb_s[tid] >> 23) - 126;   // max|x| < 2^emx
    const int ebn = static_cast<int>(mnb_s[tid] >> 23);
    const int ulp = (ebn > 0 ? ebn : 1) - 150;                   // ulp(min nonzero |x|) = 2^ulp
    int lg = 0;
    while ((1 << lg) < 2 * theta) ++lg;
    exact = (emx + lg) - ulp <= 53;
  }
  if (!exact) {
    nf_list[atomicAdd(nf_count, 1)] = 2 * j;
    return;
  }
  auto s = [&](int p) -> float { return colt[p * TW + tid]; };
  const bool even = (theta & 1) == 0;
  const int pl = even ? theta / 2 - 1 : (theta - 1) / 2;
  const float cl = s(pl), cu = s(theta / 2);
  double res = bulyan_window_mean(s, theta, keep, pl);
  if (even && cu != cl) {
    // exact totals tie: np.argmin takes the first selection-order index
    // holding either middle value
    const double res_u = bulyan_window_mean(s, theta, keep, theta / 2);
    for (int p = 0; p < theta; ++p) {
      const float x = S[static_cast<int64_t>(checked_row(rows[p], nrows_s)) * lds_ + j];
      if (x == cl) break;
      if (x == cu) {
        res = res_u;
        break;
      }
    }
  }
  out[j] = res;
}

// Listed columns of the big stage: the stage by definition
// (bulyan_stage_generic), one lane per column, the rank map in LDS
// ([theta][blockDim.x]: 32 lanes up to theta = 1024, fewer above).
__global__ void __launch_bounds__(32) bulyan_listed_big_kernel(const float* __restrict__ S, int64_t lds_,
                                                               const int* __restrict__ rows, int nrows_s, int theta,
                                                               int keep, const int* __restrict__ nf_count,
                                                               const int64_t* __restrict__ nf_list,
                                                               double* __restrict__ out) {
  extern __shared__ int rank_slots[];   // [theta][L]
  const int t = threadIdx.x;
  const int L = blockDim.x;
  const int cnt = *nf_count;
  for (int e = blockIdx.x * L + t; e < cnt; e += gridDim.x * L) {
    const int64_t j = nf_list[e] >> 1;
    auto a = [&](int i) -> double {
      return S[static_cast<int64_t>(checked_row(rows[i], nrows_s)) * lds_ + j];
    };
    int m;
    out[j] = keep == 0 ? __builtin_nan("")
                       : bulyan_stage_generic<true>(a, theta, keep, [&](int p) -> int& { return rank_slots[p * L + t]; },
                                              &m);
  }
}

// arr[np.argsort(distances)[:beta]] keeps min(beta, theta) values for beta >= 0
// and max(theta + beta, 0) for beta < 0 (Python slice semantics,
// robust_estimator.py:274; torch slicing at src/DBA/helper.py:939 likewise)
inline int bulyan_keep(int theta, int beta) {
  if (beta >= 0) return beta < theta ? beta : theta;
  return theta + beta > 0 ? theta + beta : 0;
}

// the drop-in's scalar helpers: one lane per column of a float64 theta x d
// matrix; the rank slots [theta][L] in dynamic LDS, L = min(64, 32768 / theta)
// lanes per block (128 KiB at most)
constexpr int kCoordMaxTheta = kBigMaxClients;
constexpr int kCoordSlots = 512 * 64;

__global__ void __launch_bounds__(64) bulyan_coord_f64_kernel(const double* __restrict__ A, int theta, int64_t d,
                                                              int64_t lda, int keep, double* __restrict__ out,
                                                              int64_t* __restrict__ midx, double* __restrict__ mrow,
                                                              int64_t ldr) {
  extern __shared__ int order_slots[];   // [theta][blockDim.x]
  const int t = threadIdx.x;
  const int L = blockDim.x;
  const int64_t j = static_cast<int64_t>(blockIdx.x) * L + t;
  if (j >= d) return;
  auto a = [&](int i) -> double { return A[static_cast<int64_t>(i) * lda + j]; };
  int m;
  out[j] = bulyan_stage_generic<true>(a, theta, keep, [&](int p) -> int& { return order_slots[p * L + t]; }, &m);
  if (midx) midx[j] = m;
  if (mrow) {
    const double am = a(m);
    for (int k = 0; k < theta; ++k)
      mrow[static_cast<int64_t>(k) * ldr + j] = k == m ? 0.0 : __builtin_fabs(am - a(k));
  }
}

// ---------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------

// workspace: [0, 256) nonfinite-column count | order, row lists, status |
// krum workspace or (S, partial sums) | the nonfinite-column list (int64 x d)
static size_t bulyan_body_bytes(int n, int64_t d, int mode, int f) {
  const int theta = n - 2 * f;
  size_t b = 4096 + 4 * static_cast<size_t>(n) * 4 + 256;
  if (mode == kBulyanKrum) {
    b += krum_workspace_bytes(n, d);
  } else {
    b += sizeof(float) * static_cast<size_t>(theta > 0 ? theta : 0) * static_cast<size_t>(d) + 256;
    b += round_partial_bytes(n, d) + sizeof(double) * static_cast<size_t>(n) + 512;
  }
  return (b + 255) / 256 * 256;
}

size_t bulyan_workspace_bytes(int n, int64_t d, int mode, int f) {
  return bulyan_body_bytes(n, d, mode, f) + sizeof(int64_t) * static_cast<size_t>(d);
}

// Where step 2 takes the columns from, per P (same-box per-round kernel times
// at C3, profiles/r06_bulyan_rounds_ab.txt): up to P = 64 the whole column
// stays in registers at three waves per SIMD; above, the first 44 rows go to
// LDS (4 x 44 x 272 B + the aggregate and partial tiles = 50.9 KiB per
// workgroup: three workgroups per CU, three waves per SIMD; 47 rows no longer
// fit three) and the rest are re-read.  Register copies at two waves per SIMD
// (P = 80 / 96 / 112) lost to the LDS form by 7-10 %.
#ifndef SRA_BULYAN_COPY_MAX_MEDIAN
#define SRA_BULYAN_COPY_MAX_MEDIAN 64
#endif
#ifndef SRA_BULYAN_COPY_MAX_TRIMMED
#define SRA_BULYAN_COPY_MAX_TRIMMED 64
#endif
template <int P, int MODE>
constexpr bool kCopyRows() {
  return P <= 32 || (MODE == 0 ? P <= SRA_BULYAN_COPY_MAX_MEDIAN : P <= SRA_BULYAN_COPY_MAX_TRIMMED);
}
#ifndef SRA_BULYAN_LDS_ROWS
#define SRA_BULYAN_LDS_ROWS 44
#endif
template <int P, int MODE>
constexpr int kLdsRows() { return kCopyRows<P, MODE>() ? 0 : SRA_BULYAN_LDS_ROWS; }
template <int P, int MODE>
constexpr int kRegRows() { return kCopyRows<P, MODE>() ? P : kLdsRows<P, MODE>(); }
template <int P, int MODE>
constexpr int kRoundWaves() { return kCopyRows<P, MODE>() && P > 64 ? 2 : 3; }

#ifndef SRA_BULYAN_BUCKET
#define SRA_BULYAN_BUCKET 8
#endif
constexpr int kRoundBucket = SRA_BULYAN_BUCKET;   // rows per kernel instantiation step
static_assert(kRoundBucket == 8 || kRoundBucket == 16, "bucket width");

template <int MODE>
static int launch_select_dist(const float* X, int64_t ldx, const int* rows, int nrows_x, int n, int64_t d, int lo,
                              int hi, int nan_all, float* out, float* bpart, hipStream_t s) {
  const int64_t tpb = round_tiles_per_block(d);
  const int64_t blocks = round_blocks(d);
  // P: the row count rounded up to the bucket width (>= 16; 8-wide buckets
  // measured 2-3 % faster at C3 than 16-wide, profiles/r06_negative_ab.txt); every kernel
  // constant assumes only n in (P - 16, P], so either width is valid
  const int P = n <= 16 ? 16 : static_cast<int>(cdiv(n, kRoundBucket) * kRoundBucket);
#define SRA_SR(PP)                                                                                             \
  case PP:                                                                                                     \
    hipLaunchKernelGGL((select_dist_rows_kernel<PP, MODE, kLdsRows<PP, MODE>(), kRegRows<PP, MODE>(),             \
                                                kRoundWaves<PP, MODE>()>), dim3(blocks), dim3(256), 0, s, X, ldx,      \
                       rows, nrows_x, n,                                                                       \
                       d, lo,                                                                                  \
                       hi, nan_all, out, bpart, static_cast<int>(blocks), static_cast<int>(tpb));                       \
    return launch_status("select_dist_rows_kernel");
  switch (P) {
    SRA_SR(16) SRA_SR(32) SRA_SR(48) SRA_SR(64) SRA_SR(80) SRA_SR(96) SRA_SR(112) SRA_SR(128)
#if SRA_BULYAN_BUCKET == 8
    SRA_SR(24) SRA_SR(40) SRA_SR(56) SRA_SR(72) SRA_SR(88) SRA_SR(104) SRA_SR(120)
#endif
    default: break;
  }
#undef SRA_SR
  set_error("bulyan median/trimmedmean rounds support N <= 128 (got %d)", n);
  return SRA_ERR_UNSUPPORTED;
}

static int launch_final(const float* S, int64_t lds_, const int* rows, int nrows_s, int theta, int beta, int64_t d,
                        double* out, int* nf_count, int64_t* nf_list, hipStream_t s) {
  const int keep = bulyan_keep(theta, beta);
  // theta rounded up to the round kernels' bucket width (the kernels assume
  // only theta in (P - 16, P])
  const int P = theta <= 16 ? 16 : static_cast<int>(cdiv(theta, kRoundBucket) * kRoundBucket);
  SRA_REQUIRE(theta >= 1 && theta <= kBigMaxClients, SRA_ERR_UNSUPPORTED,
              "bulyan per-coordinate stage supports theta <= %d (got %d)", kBigMaxClients, theta);
  SRA_HIP(hipMemsetAsync(nf_count, 0, sizeof(int), s));
  if (theta > kFinalMaxTheta) {
    const int pn = next_pow2(theta);
    constexpr int kStageLdsFloats = 512 * 64;   // 128 KiB: TW = kStageLdsFloats / pn coordinates per tile
    const size_t lds_bytes = sizeof(float) * static_cast<size_t>(kStageLdsFloats);
    int rc = SRA_OK;
    auto run = [&](auto kern, int tw) -> int {
      SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(lds_bytes)));
      hipLaunchKernelGGL(kern, dim3(cdiv(d, tw)), dim3(256), sizeof(float) * static_cast<size_t>(pn) * tw, s, S, lds_,
                         rows, nrows_s, theta, pn, keep, d, out, nf_count, nf_list);
      return launch_status("bulyan_final_lds_kernel");
    };
    // the widest instantiated tile is 64 coordinates (theta in (128, 256]
    // would allow 128 within the LDS budget)
    switch (kStageLdsFloats / pn < 64 ? kStageLdsFloats / pn : 64) {
      case 64: rc = run(bulyan_final_lds_kernel<64>, 64); break;
      case 32: rc = run(bulyan_final_lds_kernel<32>, 32); break;
      case 16: rc = run(bulyan_final_lds_kernel<16>, 16); break;
      case 8: rc = run(bulyan_final_lds_kernel<8>, 8); break;
      default: rc = run(bulyan_final_lds_kernel<4>, 4); break;
    }
    if (rc) return rc;
    constexpr int kRankSlots = 1024 * 32;   // 128 KiB of rank slots
    const int lanes = kRankSlots / theta < 32 ? kRankSlots / theta : 32;
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(bulyan_listed_big_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(sizeof(int) * kRankSlots)));
    hipLaunchKernelGGL(bulyan_listed_big_kernel, dim3(256), dim3(lanes),
                       sizeof(int) * static_cast<size_t>(theta) * lanes, s, S, lds_, rows, nrows_s, theta, keep,
                       nf_count, nf_list, out);
    return launch_status("bulyan_listed_big_kernel");
  }
  int rc = SRA_ERR_UNSUPPORTED;
#define SRA_FIN(PP)                                                                                              \
  case PP:                                                                                                       \
    hipLaunchKernelGGL((bulyan_final_kernel<PP>), dim3(cdiv(d, 256)), dim3(256), 0, s, S, lds_, rows, nrows_s,   \
                       theta, keep, d, out, nf_count, nf_list);                                                  \
    rc = launch_status("bulyan_final_kernel");                                                                   \
    if (rc) return rc;                                                                                           \
    hipLaunchKernelGGL((bulyan_listed_kernel<PP>), dim3(256), dim3(64), 0, s, S, lds_, rows, nrows_s, theta, keep,  \
                       nf_count,                                                                               \
                       nf_list, out);                                                                            \
    return launch_status("bulyan_listed_kernel");
  switch (P) {
    SRA_FIN(16) SRA_FIN(32) SRA_FIN(48) SRA_FIN(64) SRA_FIN(80) SRA_FIN(96) SRA_FIN(112) SRA_FIN(128)
#if SRA_BULYAN_BUCKET == 8
    SRA_FIN(24) SRA_FIN(40) SRA_FIN(56) SRA_FIN(72) SRA_FIN(88) SRA_FIN(104) SRA_FIN(120)
#endif
    default: break;
  }
#undef SRA_FIN
  return rc;
}

// One selection round of Bulyan's median / trimmed-mean modes
// (robust_estimator.py:297-322) over the listed rows: agg = the coordinate-wise
// aggregate of the remaining clients, dist[r] = squared L2 distance of listed
// row r to it (fp32 within a 256-coordinate block, fp64 across blocks in
// order), both from ONE pass over the rows.  Over a column shard, dist is this
// shard's share: the shards' dist vectors sum (all-reduce) to the distance
// over all columns.  bpart: nr x round_blocks(d) floats.
static int launch_round_big(const float* X, int64_t ldx, const int* rows, int nrows_x, int nr, int64_t d, bool median,
                            int lo, int hi, int nan_all, float* agg, float* bpart, hipStream_t s) {
  SRA_REQUIRE(nr <= kBigMaxClients, SRA_ERR_UNSUPPORTED, "bulyan median/trimmedmean rounds support N <= %d (got %d)",
              kBigMaxClients, nr);
  const int pn = next_pow2(nr);
  const int tile = kBigLdsFloats / pn;
  hipLaunchKernelGGL(select_rows_lds_kernel, dim3(cdiv(d, tile)), dim3(256), sizeof(float) * pn * tile, s, X, ldx,
                     rows, nrows_x, nr, pn, tile, d, median ? 1 : 0, lo, hi, nan_all, agg);
  int rc = launch_status("select_rows_lds_kernel");
  if (rc) return rc;
  const int64_t tpb = round_tiles_per_block(d);
  const int64_t blocks = round_blocks(d);
  if (nr <= 256)
    hipLaunchKernelGGL(dist_rows_kernel<1>, dim3(blocks), dim3(256), 0, s, X, ldx, rows, nrows_x, nr, d, agg, bpart,
                       static_cast<int>(blocks), static_cast<int>(tpb));
  else if (nr <= 512)
    hipLaunchKernelGGL(dist_rows_kernel<2>, dim3(blocks), dim3(256), 0, s, X, ldx, rows, nrows_x, nr, d, agg, bpart,
                       static_cast<int>(blocks), static_cast<int>(tpb));
  else   // groups of up to 1024 listed rows, each with its own slice of the partial table
    for (int g0 = 0; g0 < nr; g0 += kDistRowGroup) {
      const int ng = nr - g0 < kDistRowGroup ? nr - g0 : kDistRowGroup;
      hipLaunchKernelGGL(dist_rows_kernel<4>, dim3(blocks), dim3(256), 0, s, X, ldx, rows + g0, nrows_x, ng, d, agg,
                         bpart + static_cast<int64_t>(g0) * blocks, static_cast<int>(blocks), static_cast<int>(tpb));
      const int rc2 = launch_status("dist_rows_kernel");
      if (rc2) return rc2;
    }
  return launch_status("dist_rows_kernel");
}

static int launch_bulyan_round(const float* X, int nrows_x, int64_t d, int64_t ldx, const int* rows, int nr, int mode,
                               bool dba, float* agg, float* bpart, double* dist, hipStream_t s) {
  int lo, hi, sel_mode, nan_all = 0;
  if (mode == kBulyanMedian && dba) {
    nan_all = 1;         // torch.median propagates NaN (helper.py:1038 -> the assert at :1047)
    lo = (nr - 1) / 2;   // torch.median: s[(n-1)//2]
    hi = lo + 1;
    sel_mode = 1;
  } else if (mode == kBulyanMedian) {
    lo = 0;
    hi = nr;
    sel_mode = 0;
  } else {
    const int b = static_cast<int>(nr * 0.1);  // trimmed_mean(beta=0.1): int(size * beta)
    lo = b;
    hi = nr - b > b ? nr - b : b;
    sel_mode = 1;
  }
  int rc;
  if (nr > 128)
    rc = launch_round_big(X, ldx, rows, nrows_x, nr, d, sel_mode == 0, lo, hi, nan_all, agg, bpart, s);
  else if (sel_mode == 0)
    rc = launch_select_dist<0>(X, ldx, rows, nrows_x, nr, d, lo, hi, nan_all, agg, bpart, s);
  else
    rc = launch_select_dist<1>(X, ldx, rows, nrows_x, nr, d, lo, hi, nan_all, agg, bpart, s);
  if (rc) return rc;
  hipLaunchKernelGGL(bulyan_dist_reduce_kernel, dim3(nr), dim3(256), 0, s, bpart, static_cast<int>(round_blocks(d)),
                     dist);
  return launch_status("bulyan_dist_reduce_kernel");
}

__global__ void iota_kernel(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = i;
}

// dba = true: the DBA harness's Helper.bulyan_* (src/DBA/helper.py:942-1137).  Its Krum rounds keep the
// zero self-distance among the size - i - f - 2 smallest (:979-980), i.e. Krum with f + 1 over the
// other clients (identical while remaining - f - 2 >= 1: f >= 2 or f == 0); its median rounds take
// torch.median's LOWER median (:1025); trimmed-mean rounds and theta / beta are unchanged.
int launch_bulyan(const float* X, int n, int64_t d, int64_t ldx, int f, int mode, double* out, int* sel_out,
                  int* status_out, void* ws, size_t ws_bytes, hipStream_t s, bool dba = false) {
  const int theta = n - 2 * f;
  SRA_REQUIRE(theta > 0, SRA_ERR_THETA, "bulyan needs theta = N - 2f > 0 (N=%d, f=%d)", n, f);
  SRA_REQUIRE(mode >= 0 && mode <= 2, SRA_ERR_ARG, "bad bulyan mode %d", mode);
  SRA_REQUIRE(ws != nullptr && ws_bytes >= bulyan_workspace_bytes(n, d, mode, f), SRA_ERR_WORKSPACE,
              "bulyan workspace too small: need %zu bytes", bulyan_workspace_bytes(n, d, mode, f));
  const int beta = theta - 2 * f;
  char* p = static_cast<char*>(ws);
  int* order = reinterpret_cast<int*>(p + 256);
  int* rows_a = order + n;
  int* rows_b = rows_a + n;
  // status: 1 = a median / trimmed-mean round found no strict minimum (every
  // distance NaN or inf): the reference's `assert min_index != None` (:308, :321)
  int* status = status_out != nullptr ? status_out : rows_b + n;
  SRA_HIP(hipMemsetAsync(status, 0, sizeof(int), s));
  char* rest = p + 4096 + 4 * static_cast<size_t>(n) * 4;
  int* nf_count = reinterpret_cast<int*>(p);
  int64_t* nf_list = reinterpret_cast<int64_t*>(p + bulyan_body_bytes(n, d, mode, f));
  int rc;
  if (mode == kBulyanKrum) {
    rc = launch_krum(X, n, d, ldx, dba ? f + 1 : f, theta, order, nullptr, rest, krum_workspace_bytes(n, d), s);
    if (rc) return rc;
    if (sel_out) SRA_HIP(hipMemcpyAsync(sel_out, order, sizeof(int) * theta, hipMemcpyDeviceToDevice, s));
    return launch_final(X, ldx, order, n, theta, beta, d, out, nf_count, nf_list, s);
  }
  SRA_REQUIRE(n <= kBigMaxClients, SRA_ERR_UNSUPPORTED, "bulyan median/trimmedmean rounds support N <= %d (got %d)",
              kBigMaxClients, n);
  float* S = reinterpret_cast<float*>(rest);
  float* bpart = reinterpret_cast<float*>(
      (reinterpret_cast<uintptr_t>(S + static_cast<size_t>(theta) * static_cast<size_t>(d)) + 255) &
      ~static_cast<uintptr_t>(255));
  hipLaunchKernelGGL(iota_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, rows_a, n);
  hipLaunchKernelGGL(iota_kernel, dim3(cdiv(theta, 256)), dim3(256), 0, s, order, theta);
  rc = launch_status("iota_kernel");
  if (rc) return rc;
  double* dist = reinterpret_cast<double*>(
      (reinterpret_cast<uintptr_t>(bpart) + round_partial_bytes(n, d) + 255) & ~static_cast<uintptr_t>(255));
  int* cur = rows_a;
  int* nxt = rows_b;
  for (int t = 0; t < theta; ++t) {
    const int nr = n - t;
    float* agg = S + static_cast<size_t>(t) * static_cast<size_t>(d);
    rc = launch_bulyan_round(X, n, d, ldx, cur, nr, mode, dba, agg, bpart, dist, s);
    if (rc) return rc;
    hipLaunchKernelGGL(bulyan_pick_kernel, dim3(1), dim3(256), 0, s, dist, cur, nr, nxt, status);
    rc = launch_status("bulyan_pick_kernel");
    if (rc) return rc;
    int* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  return launch_final(S, d, order, theta, theta, beta, d, out, nf_count, nf_list, s);
}

}  // namespace sra

using namespace sra;

extern "C" int sra_bulyan_workspace_bytes(int64_t n, int64_t d, int32_t f, int32_t mode, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && d >= 1, SRA_ERR_SHAPE, "bad shape");
  *bytes = bulyan_workspace_bytes(static_cast<int>(n), d, mode, f);
  return SRA_OK;
}

extern "C" int sra_bulyan_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t mode,
                              double* out, int32_t* selected, int32_t* status, void* ws, size_t ws_bytes,
                              void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= kBigMaxClients && d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad shape (N <= %d)",
              kBigMaxClients);
  return launch_bulyan(X, static_cast<int>(n), d, ldx, f, mode, out, selected, status, ws, ws_bytes,
                       static_cast<hipStream_t>(stream));
}

extern "C" int sra_bulyan_dba_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t mode,
                                  double* out, int32_t* selected, int32_t* status, void* ws, size_t ws_bytes,
                                  void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= kBigMaxClients && d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad shape (N <= %d)",
              kBigMaxClients);
  SRA_REQUIRE(!(mode == kBulyanKrum && f == 1), SRA_ERR_ARG,
              "DBA bulyan_krum with f = 1 (its last round scores an empty neighbour set) is not supported");
  return launch_bulyan(X, static_cast<int>(n), d, ldx, f, mode, out, selected, status, ws, ws_bytes,
                       static_cast<hipStream_t>(stream), true);
}

extern "C" int sra_bulyan_coordinate_f64(const double* A, int64_t theta, int64_t d, int64_t lda, int32_t beta,
                                         double* out, int64_t* median_index, double* median_row, int64_t ldr,
                                         void* stream) {
  SRA_REQUIRE(A != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(theta >= 1 && theta <= kCoordMaxTheta, SRA_ERR_UNSUPPORTED, "1 <= theta <= %d (got %lld)",
              kCoordMaxTheta, static_cast<long long>(theta));
  SRA_REQUIRE(d >= 1 && lda >= d && (median_row == nullptr || ldr >= d), SRA_ERR_SHAPE, "bad d / lda / ldr");
  const int keep = bulyan_keep(static_cast<int>(theta), beta);
  const int lanes = kCoordSlots / theta < 64 ? static_cast<int>(kCoordSlots / theta) : 64;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(bulyan_coord_f64_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     static_cast<int>(sizeof(int) * kCoordSlots));
  SRA_REQUIRE(attr == hipSuccess, SRA_ERR_UNSUPPORTED, "bulyan_coord_f64_kernel: cannot reserve its LDS");
  hipLaunchKernelGGL(bulyan_coord_f64_kernel, dim3(cdiv(d, lanes)), dim3(lanes),
                     sizeof(int) * static_cast<size_t>(theta) * lanes, static_cast<hipStream_t>(stream), A,
                     static_cast<int>(theta), d, lda, keep, out, median_index, median_row, ldr);
  return launch_status("bulyan_coord_f64_kernel");
}

// The per-coordinate stage alone over theta float32 rows (row i = the i-th
// selected vector, in selection order): the final stage of sra_bulyan_f32 for
// selections made elsewhere (a d-sharded Bulyan, a caller's own rounds).
extern "C" int sra_bulyan_stage_workspace_bytes(int64_t theta, int64_t d, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(theta >= 1 && theta <= kBigMaxClients && d >= 1, SRA_ERR_SHAPE, "need 1 <= theta <= %d, d >= 1",
              kBigMaxClients);
  *bytes = 256 + (static_cast<size_t>(theta) * sizeof(int) + 255) / 256 * 256 + sizeof(int64_t) * static_cast<size_t>(d);
  return SRA_OK;
}

extern "C" int sra_bulyan_stage_f32(const float* S, int64_t theta, int64_t d, int64_t lds, int32_t beta, double* out,
                                    void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(S != nullptr && out != nullptr && ws != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(theta >= 1 && theta <= kBigMaxClients, SRA_ERR_UNSUPPORTED, "1 <= theta <= %d (got %lld)",
              kBigMaxClients, static_cast<long long>(theta));
  SRA_REQUIRE(d >= 1 && lds >= d, SRA_ERR_SHAPE, "bad d / lds");
  size_t need = 0;
  sra_bulyan_stage_workspace_bytes(theta, d, &need);
  SRA_REQUIRE(ws_bytes >= need, SRA_ERR_WORKSPACE, "bulyan stage workspace too small: need %zu bytes", need);
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* p = static_cast<char*>(ws);
  int* nf_count = reinterpret_cast<int*>(p);
  int* rows = reinterpret_cast<int*>(p + 256);
  int64_t* nf_list = reinterpret_cast<int64_t*>(p + 256 + (static_cast<size_t>(theta) * sizeof(int) + 255) / 256 * 256);
  hipLaunchKernelGGL(iota_kernel, dim3(cdiv(theta, 256)), dim3(256), 0, s, rows, static_cast<int>(theta));
  const int rc = launch_status("iota_kernel");
  if (rc) return rc;
  return launch_final(S, lds, rows, static_cast<int>(theta), static_cast<int>(theta), beta, d, out, nf_count, nf_list,
                      s);
}

// One Bulyan selection round over a (possibly column-sharded) N x d block, for
// a caller that sums the shards' distances (all-reduce) and picks itself.
extern "C" int sra_bulyan_round_workspace_bytes(int64_t n, int64_t d, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && n <= kBigMaxClients && d >= 1, SRA_ERR_UNSUPPORTED,
              "bulyan rounds support 1 <= N <= %d, d >= 1", kBigMaxClients);
  *bytes = round_partial_bytes(static_cast<int>(n), d) + 256;
  return SRA_OK;
}

extern "C" int sra_bulyan_round_f32(const float* X, int64_t n, int64_t d, int64_t ldx, const int32_t* rows,
                                    int32_t nr, int32_t mode, int32_t dba, float* agg, double* dist, void* ws,
                                    size_t ws_bytes, void* stream) {
  SRA_REQUIRE(X != nullptr && rows != nullptr && agg != nullptr && dist != nullptr && ws != nullptr, SRA_ERR_ARG,
              "null pointer");
  SRA_REQUIRE(n >= 1 && n <= kBigMaxClients && nr >= 1 && nr <= n && d >= 1 && ldx >= d, SRA_ERR_SHAPE,
              "bad shape (N <= %d, 1 <= nr <= N)", kBigMaxClients);
  SRA_REQUIRE(mode == kBulyanMedian || mode == kBulyanTrimmed, SRA_ERR_ARG, "round mode must be median (1) or "
              "trimmedmean (2), got %d", mode);
  size_t need = 0;
  sra_bulyan_round_workspace_bytes(n, d, &need);
  SRA_REQUIRE(ws_bytes >= need, SRA_ERR_WORKSPACE, "bulyan round workspace too small: need %zu bytes", need);
  return launch_bulyan_round(X, static_cast<int>(n), d, ldx, rows, nr, mode, dba != 0, agg, static_cast<float*>(ws),
                             dist, static_cast<hipStream_t>(stream));
}

extern "C" int sra_bulyan_pick(const double* dist, const int32_t* rows, int32_t nr, int32_t* rows_next,
                               int32_t* status, void* stream) {
  SRA_REQUIRE(dist != nullptr && rows != nullptr && rows_next != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(nr >= 1, SRA_ERR_SHAPE, "nr >= 1");
  hipLaunchKernelGGL(bulyan_pick_kernel, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), dist, rows, nr,
                     rows_next, status);
  return launch_status("bulyan_pick_kernel");
}
