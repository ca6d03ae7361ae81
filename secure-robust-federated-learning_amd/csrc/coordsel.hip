// k1 — coordinate-wise aggregators: average, median, trimmed mean.
//
// Replaces src/robust_estimator.py:220-232 (median, trimmed_mean) and the
// inline average of src/simulate.py:235-244.
//
// Layout: X is N x d fp32, client-major (row i = client i), row stride ldx.
// One lane owns one coordinate j; a wave reads 64 consecutive coordinates of a
// row per load (256 contiguous bytes), so every load is coalesced and the whole
// column of N values lands in that lane's VGPRs with N independent loads in
// flight.  The column is then sorted in registers by a Batcher odd-even merge
// network (constexpr table -> immediate register indices, NaN-last compare
// exchange = v_min_f32 + v_maximum3_f32), and the kept order statistics are
// summed sequentially in ascending order in fp32 -- the exact evaluation order
// of numpy's sort + axis-0 mean, so the result is bit-identical to the
// reference.  Padding rows (n..P) are NaN: they sort after every real value
// (and after real NaNs), so positions 0..n-1 of the padded sort are exactly
// numpy's sorted column.
//
// Roofline: HBM-bound, 4*N*d + 4*d bytes per call.  The exact-N trimmed mean
// at N=128 (select_plain_kernel) runs a network pruned to the kept ranks
// (4-blocks + network_plain); its VALU instruction count per tile is reported by
// tools/isa_stats.py and set against the HBM time in DESIGN.md §3.
//
// 128 < N <= 512 (the N=512 MoM / 8-GPU config) uses 2 or 4 lanes per
// coordinate with DPP bitonic merges (select_quad_kernel); larger N, or row
// strides beyond 32-bit lane offsets, fall back to an LDS bitonic tile.
#include "sra_common.hpp"

namespace sra {
#include "net_fused.inc"
}

#include <algorithm>
#include <cstdlib>

namespace sra {

enum SelectMode { kMedian = 0, kTrimmed = 1, kOrder = 2 };  // kOrder: s[lo], any NaN -> NaN

// ---------------------------------------------------------------------------
// average: sequential fp32 sum over clients (numpy axis-0 add.reduce order).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) average_vec4_kernel(const float* __restrict__ X, int n, int64_t d4,
                                                          int64_t ldx, float* __restrict__ out) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= d4) return;
  const f32x4* p = reinterpret_cast<const f32x4*>(X) + q;
  const int64_t ld4 = ldx / 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    f32x4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = __builtin_nontemporal_load(p + (int64_t)(i + u) * ld4);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += r[u];
  }
  for (; i < n; ++i) acc += __builtin_nontemporal_load(p + (int64_t)i * ld4);
  reinterpret_cast<f32x4*>(out)[q] = acc / static_cast<float>(n);
}

__global__ void __launch_bounds__(256) average_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                     float* __restrict__ out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= d) return;
  float acc = 0.f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    float r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = X[(int64_t)(i + u) * ldx + j];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += r[u];
  }
  for (; i < n; ++i) acc += X[(int64_t)i * ldx + j];
  out[j] = acc / static_cast<float>(n);
}

// ---------------------------------------------------------------------------
// register path: P = n rounded up to a multiple of 16 (P <= 128), network size
// P2 = next_pow2(P) with compile-time NaN pads beyond P (the compiler folds
// every compare-exchange that touches them).
//
// Addressing: the row pointer X + i*ldx + blockbase is wave-uniform (SGPRs), the
// lane offset is one 32-bit VGPR shared by every load, so each of the P loads
// is a `global_load_dword v, voff, s[base]` with no per-load address VGPRs.
//
// Median: the runtime pads are split -inf (bottom) / NaN (top) so that the
// middle order statistics of the n real values land on the fixed positions
// P/2-1 and P/2 whatever n is (no runtime register indexing); a NaN anywhere
// in the column is detected by a NaN-propagating max over the raw values.
// Trimmed mean: all runtime pads are NaN (they sort last), and the kept range
// [lo, hi) is summed with wave-uniform predicates.
// ---------------------------------------------------------------------------
// one streaming load from a wave-uniform row base plus a 32-bit lane byte offset
// (readfirstlane pins the row base in SGPRs: without it LLVM reassociates
// (base + i*ld) + lane into one 64-bit VGPR address per load and runs out of
// registers at N=128)
__device__ __forceinline__ float ldrow(const char* row, unsigned off) {
  const uint64_t r = reinterpret_cast<uint64_t>(row);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r >> 32));
  typedef const __attribute__((address_space(1))) float gfloat;
  const uint64_t u = ((static_cast<uint64_t>(hi) << 32) | lo) + off;
  return __builtin_nontemporal_load(reinterpret_cast<gfloat*>(u));
}

__device__ __forceinline__ void opaque_sgpr(uint64_t& p) { asm volatile("" : "+s"(p)); }

template <int P, int MODE, int NX = 0, int BX = -1, int BS = 256>
__global__ void __launch_bounds__(BS) select_reg_kernel(const float* __restrict__ X, int n_rt, int64_t d,
                                                       int64_t ldx, int lo_rt, int hi_rt, float* __restrict__ out) {
  constexpr int P2 = next_pow2(P);
  constexpr bool kExactN = NX > 0;
  constexpr bool kExactB = kExactN && BX >= 0;
  const int n = kExactN ? NX : n_rt;
  const int lo = kExactB ? BX : lo_rt;
  const int hi = kExactB ? NX - BX : hi_rt;
  constexpr int kFirstPad = kExactN ? NX : ((P > 16) ? P - 16 : 0);  // rows below this are always real
  const int64_t base = static_cast<int64_t>(blockIdx.x) * BS;
  const int64_t rem = d - base;                    // > 0
  const unsigned t = threadIdx.x;
  const unsigned last = rem < BS ? static_cast<unsigned>(rem - 1) : static_cast<unsigned>(BS - 1);
  const unsigned off = (t < last ? t : last) * 4u;  // byte offset of this lane (tail lanes clamped)
  const char* xb = reinterpret_cast<const char*>(X + base);
  const int64_t ldb = ldx * 4;
  // exact-N instantiations have no runtime pads: slots [NX, P2) are implicit
  // +inf and the requested order statistics sit on fixed slots
  constexpr int PR = kExactN ? NX : P;
  const int k_bottom = (MODE == kMedian && !kExactN) ? (P - n) / 2 : 0;  // -inf pads (runtime-N median)
  float v[P2];
  // rows through a running SGPR row pointer, opaque to the optimiser: nothing
  // (no per-row 64-bit offset) stays live across the network for the reload
  auto load_column = [&]() {
    const uint64_t a = reinterpret_cast<uint64_t>(xb);
    const uint32_t alo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
    const uint32_t ahi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
    uint64_t rp = (static_cast<uint64_t>(ahi) << 32) | alo;
    typedef const __attribute__((address_space(1))) float gfloat;
#pragma unroll
    for (int i = 0; i < kFirstPad; ++i) {
      v[i] = __builtin_nontemporal_load(reinterpret_cast<gfloat*>(rp + off));
      rp += static_cast<uint64_t>(ldb);
      opaque_sgpr(rp);
      __builtin_amdgcn_sched_barrier(0);
    }
    // runtime-N tail: rows >= n re-read row n-1 (kept in bounds), then padded
    uint64_t rl = rp;
#pragma unroll
    for (int i = kFirstPad; i < PR; ++i) {
      const float x = __builtin_nontemporal_load(reinterpret_cast<gfloat*>(rl + off));
      if (i + 1 < n) {
        rl += static_cast<uint64_t>(ldb);
        opaque_sgpr(rl);
      }
      __builtin_amdgcn_sched_barrier(0);
      const float pad = (i - n < k_bottom) ? -__builtin_inff() : __builtin_inff();
      v[i] = i < n ? x : pad;
    }
  };
  load_column();

  // Median slots: runtime N centres the real values between the -inf/+inf
  // pads (slots P/2-1, P/2); exact N keeps them at the front.
  constexpr int kMedLo = kExactN ? (NX - 1) / 2 : P / 2 - 1;
  constexpr int kMedHi = kExactN ? NX / 2 : P / 2;
  constexpr int kOutLo = MODE == kMedian ? kMedLo : (kExactB ? BX : 0);
  constexpr int kOutHi = MODE == kMedian ? kMedHi + 1 : (kExactB ? NX - BX : PR);

  auto finish = [&](int nan_cnt) -> float {
    float r;
    if constexpr (MODE == kMedian) {
      const float a = kExactN ? v[kMedLo] : v[P / 2 - 1];
      const float b = kExactN ? v[kMedHi] : v[P / 2];
      r = (n & 1) ? a : (a + b) * 0.5f;
    } else {
      // sequential ascending-order sum of s[lo .. hi), numpy's axis-0 reduce;
      // (the empty volatile asm keeps each runtime predicate a wave-uniform
      // scalar branch instead of hoisted SGPR-pair masks that spill)
      float acc = 0.f;
#pragma unroll
      for (int p = 0; p < PR; ++p) {
        if (p >= lo && p < hi) {
          if constexpr (!kExactB) asm volatile("");
          acc += v[p];
        }
      }
      r = acc / static_cast<float>(hi - lo);
      if (nan_cnt > n - hi) r = qnan();   // a NaN sits in the kept range
    }
    return r;
  };

  // NaN handling without a pre-pass: the compare-exchanges are IEEE-754-2019
  // minimum/maximum, which PROPAGATE NaN, and every requested order statistic
  // depends on every input, so a NaN anywhere in the column turns every kept
  // slot into NaN.  Median: that IS numpy's answer (any NaN -> NaN).  Trimmed
  // mean: numpy sorts NaNs last and may trim them, so a NaN result (rare,
  // wave-uniform branch) reloads the column, counts the NaNs, maps them to
  // +inf -- which sorts them last exactly like numpy -- and sorts again.
  network_fast<P2, PR, kOutLo, kOutHi>(v);
  float res = finish(0);
  if constexpr (MODE == kTrimmed) {   // (kOrder keeps the propagated NaN: torch.median's answer)
    if (__builtin_amdgcn_ballot_w64(__builtin_isnan(res)) != 0) {
      load_column();
      int nan_cnt = 0;
#pragma unroll
      for (int i = 0; i < PR; ++i) {
        const bool isn = __builtin_isnan(v[i]);
        nan_cnt += isn ? 1 : 0;
        v[i] = isn ? __builtin_inff() : v[i];
      }
      network_fast<P2, PR, kOutLo, kOutHi>(v);
      res = finish(nan_cnt);
    }
  }
  if (t < rem) out[base + t] = res;
}

// Exact-N trimmed mean (N = 128 / 100: the default and config C1's client
// count) and median: 4-blocks sorted with 3-input min / med3 / max whose
// NaN-propagating maxima double as the NaN check (a column with a NaN --
// wave-uniform, rare -- reloads, counts the NaNs and maps them to +inf, which
// sorts them last like numpy), then the pruned odd-even merges as a fused
// three-input program (tools/fuse_net.py -> net_fused.inc): a compare-exchange
// pair whose output feeds one later compare-exchange is folded into it as
// min3 / max3 / med3, 2,554 -> 1,888 VALU ops for the north-star network
// (trimmed mean N = 128), 26 % fewer; the kernel was VALU-issue bound.
template <int MODE, int NX, int BX>
struct FusedFor;
template <> struct FusedFor<kTrimmed, 128, 12> { using T = FusedTm128; };
template <> struct FusedFor<kTrimmed, 100, 10> { using T = FusedTm100; };
template <> struct FusedFor<kMedian, 128, 0> { using T = FusedMed128; };
template <> struct FusedFor<kMedian, 100, 0> { using T = FusedMed100; };

template <int MODE, int NX, int BX>
__global__ void __launch_bounds__(256) select_plain_kernel(const float* __restrict__ X, int64_t d, int64_t ldx,
                                                          float* __restrict__ out) {
  using Prog = typename FusedFor<MODE, NX, BX>::T;
  constexpr int kSlots = Prog::kSlots > NX ? Prog::kSlots : NX;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256;
  const int64_t rem = d - base;
  const unsigned t = threadIdx.x;
  const unsigned last = rem < 256 ? static_cast<unsigned>(rem - 1) : 255u;
  const unsigned off = (t < last ? t : last) * 4u;
  const uint64_t a = reinterpret_cast<uint64_t>(X + base);
  const uint32_t alo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t ahi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  const uint64_t ldb = static_cast<uint64_t>(ldx) * 4;
  typedef const __attribute__((address_space(1))) float gfloat;
  float v[kSlots];
  auto load_column = [&]() {
    uint64_t rp = (static_cast<uint64_t>(ahi) << 32) | alo;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      v[i] = __builtin_nontemporal_load(reinterpret_cast<gfloat*>(rp + off));
      rp += ldb;
      opaque_sgpr(rp);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  load_column();
  // rare slow path: count NaNs, map them to +inf (sorted last, like numpy)
  auto nan_map = [&]() -> int {
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const bool isn = __builtin_isnan(v[i]);
      cnt += isn ? 1 : 0;
      v[i] = isn ? __builtin_inff() : v[i];
    }
    return cnt;
  };
  // sorted 4-blocks whose NaN-propagating maxima double as the NaN check
  const float m = sort4_blocks_nancheck<NX>(v);
  int cnt = 0;
  if (__builtin_amdgcn_ballot_w64(__builtin_isnan(m)) != 0) {   // rare: redo the blocks NaN-free
    load_column();
    cnt = nan_map();
    sort4_blocks<NX>(v);
  }
  fused_network<Prog>(v);
  float res;
  if constexpr (MODE == kMedian) {
    res = (NX & 1) ? v[Prog::kOut[0]] : (v[Prog::kOut[0]] + v[Prog::kOut[1]]) * 0.5f;
    if (cnt > 0) res = qnan();
  } else {
    // sequential ascending-order fp32 sum of the kept ranks (numpy's axis-0
    // reduce, which starts from the identity +0), then the division
    float acc = 0.f;
#pragma unroll
    for (int p = 0; p < Prog::kOuts; ++p) acc += v[Prog::kOut[p]];
    res = acc / static_cast<float>(NX - 2 * BX);
    if (cnt > BX) res = qnan();   // a NaN sits in the kept window
  }
  if (t < rem) out[base + t] = res;
}

// ---------------------------------------------------------------------------
// Multi-lane path for 128 < N <= 512 (the N = 512 MoM / 8-GPU config): L = 2 or
// 4 lanes share one coordinate, 128 values each, all in registers.
//   lane (c, h) = lane L*c + h holds rows {L*i + h} of coordinate c (per load
//   instruction the L rows are consecutive: row base in SGPRs + a 32-bit lane
//   offset).  Rows >= n are padding (+inf; split -inf/+inf for the median).
//   1. NaN pre-pass (max3; NaNs counted, mapped to +inf), then each lane
//      flips its values into its sign domain sigma_h (+,-,-,+): every later
//      step sorts ASCENDING in the stored domain, a descending run is an
//      ascending run of negated values;
//   2. each lane sorts its 128 values (3-input sorted 4-blocks + odd-even
//      merges, VOP2 min/max);
//   3. bitonic merges across lanes, one DPP instruction per element:
//      new = min(own, -partner) is the lower half in one lane and the negated
//      upper half in the partner, because their domains are opposite
//      (v_min_f32_dpp with a negated quad_perm source); lanes then flip back
//      where needed and finish with an in-lane half-cleaner cascade.
//      L=2: one level (pairs); L=4: pairs, then the 4-lane merge (a stride-256
//      step between lanes h, h^2 and a stride-128 step between h, h^1).
//   4. sorted order: L=2: lane0[0..127], lane1[0..127];
//      L=4: lane0[0..127], lane1[0..127], -lane3[127..0], -lane2[127..0];
//      the trimmed mean walks it in ascending order with one fp32 accumulator
//      handed from lane to lane (numpy's sequential sum, bit for bit).
// Validated in numpy (tools/quad_model.py) before it was written here.
// ---------------------------------------------------------------------------
template <int PERM>
__device__ __forceinline__ float min_neg_partner(float own) {
  float r;
  if constexpr (PERM == 1)
    asm volatile("v_min_f32_dpp %0, -%1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(own));
  else
    asm volatile("v_min_f32_dpp %0, -%1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(own));
  return r;
}

template <int PERM>
__device__ __forceinline__ void cross_step(float (&v)[128]) {
  // DPP reads VGPRs written by VALU: 2 wait states; nothing may move across
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
#pragma unroll
  for (int i = 0; i < 128; ++i) v[i] = min_neg_partner<PERM>(v[i]);
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void flip(float (&v)[128], uint32_t mask) {
#pragma unroll
  for (int i = 0; i < 128; ++i) v[i] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v[i]) ^ mask);
}

// value of `x` in lane h = H of this lane's group of L (quad_perm [H,H,H,H] for
// L = 4, [H,H,2+H,2+H] for the two pairs of a quad when L = 2)
template <int L, int H>
__device__ __forceinline__ float from_lane(float x) {
  constexpr int ctrl = L == 4 ? (H | (H << 2) | (H << 4) | (H << 6)) : (H | (H << 2) | ((2 + H) << 4) | ((2 + H) << 6));
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), ctrl, 0xF, 0xF, false));
}

// NT: streaming (non-temporal) row loads.  A wave's load instruction covers
// 16 coordinates = half a 128-byte line per row, the other half belongs to
// the neighbouring wave of the block, so the N = 512 launches use plain loads
// (the NT template parameter picks the load kind per instantiation).
template <int L, int MODE, int NX = 0, int BX = -1, bool NT = true>
__global__ void __launch_bounds__(256) select_quad_kernel(const float* __restrict__ X, int n_rt, int64_t d,
                                                         int64_t ldx, int lo_rt, int hi_rt, float* __restrict__ out) {
  static_assert(L == 2 || L == 4, "2 or 4 lanes per coordinate");
  constexpr bool kExactN = NX > 0;
  constexpr bool kExactB = kExactN && BX >= 0;
  const int n = kExactN ? NX : n_rt;
  const int lo = kExactB ? BX : lo_rt;
  const int hi = kExactB ? NX - BX : hi_rt;
  constexpr int P = 128 * L;
  constexpr int CPW = kWave / L;                 // coordinates per wave
  constexpr int CPB = 4 * CPW;                   // per 256-thread block
  const unsigned lane = threadIdx.x & 63u;
  const int h = static_cast<int>(lane % L);
  const int c = static_cast<int>(threadIdx.x / L);   // coordinate within the block
  const int64_t base = static_cast<int64_t>(blockIdx.x) * CPB;
  const int64_t rem = d - base;
  const int cc = c < rem ? c : static_cast<int>(rem - 1);
  const uint64_t ldb = static_cast<uint64_t>(ldx) * 4;
  const unsigned off = static_cast<unsigned>(h * ldb) + static_cast<unsigned>(cc) * 4u;
  const uint64_t a = reinterpret_cast<uint64_t>(X + base);
  const uint32_t alo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t ahi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  uint64_t rp = (static_cast<uint64_t>(ahi) << 32) | alo;
  const uint64_t rstep = ldb * L;
  typedef const __attribute__((address_space(1))) float gfloat;
  const int k_bottom = (MODE == kMedian && !kExactN) ? (P - n) / 2 : 0;
  float v[128];
#pragma unroll
  for (int i = 0; i < 128; ++i) {
    if (kExactN ? (L * i + L - 1 < NX) : (L * i + L - 1 < n)) {     // wave-uniform: all L rows real
      if constexpr (NT) v[i] = __builtin_nontemporal_load(reinterpret_cast<gfloat*>(rp + off));
      else v[i] = *reinterpret_cast<gfloat*>(rp + off);
    } else {                                                          // tail: clamp the row, then pad
      const int row = L * i + h;
      const int rr = row < n ? row : n - 1;
      const uint64_t ad = a + static_cast<uint64_t>(rr) * ldb + static_cast<unsigned>(cc) * 4u;
      const float x = __builtin_nontemporal_load(reinterpret_cast<gfloat*>(ad));
      const float pad = (row - n < k_bottom) ? -__builtin_inff() : __builtin_inff();
      v[i] = row < n ? x : pad;
    }
    rp += rstep;
    opaque_sgpr(rp);
    __builtin_amdgcn_sched_barrier(0);
  }
  // NaN pre-pass
  float m = v[0];
#pragma unroll
  for (int i = 1; i < 128; ++i) m = __builtin_elementwise_maximum(m, v[i]);
  int nan_cnt = 0;
  if (__builtin_amdgcn_ballot_w64(__builtin_isnan(m)) != 0) {
#pragma unroll
    for (int i = 0; i < 128; ++i) {
      const bool isn = __builtin_isnan(v[i]);
      nan_cnt += isn ? 1 : 0;
      v[i] = isn ? __builtin_inff() : v[i];
    }
  }
  // sign domains: L=2 (+,-); L=4 (+,-,-,+)
  const uint32_t sgn0 = (L == 2 ? (h == 1) : (h == 1 || h == 2)) ? 0x80000000u : 0u;
  const uint32_t odd = (h & 1) ? 0x80000000u : 0u;
  flip(v, sgn0);
  // in-lane sort and half-cleaner cascades as fused three-input programs
  // (tools/fuse_net.py: 2,622 -> 1,940 and 896 -> 704 VALU ops)
  sort4_blocks<128>(v);
  fused_sort128<FusedSort128>(v);
  // level 1: pairs (h, h^1)
  cross_step<1>(v);
  flip(v, odd);
  fused_sort128<FusedBitonic128>(v);
  if constexpr (L == 4) {
    // level 2: stride-256 step with h^2, stride-128 step with h^1 (odd lanes flipped around it)
    cross_step<2>(v);
    flip(v, odd);
    cross_step<1>(v);
    flip(v, odd);
    fused_sort128<FusedBitonic128>(v);
  }
  // total NaN count of the coordinate
  if constexpr (L == 2) {
    nan_cnt += __builtin_bit_cast(int, swap_adjacent(__builtin_bit_cast(float, nan_cnt)));
  } else {
    nan_cnt = __builtin_bit_cast(int, from_lane<L, 0>(__builtin_bit_cast(float, nan_cnt))) +
              __builtin_bit_cast(int, from_lane<L, 1>(__builtin_bit_cast(float, nan_cnt))) +
              __builtin_bit_cast(int, from_lane<L, 2>(__builtin_bit_cast(float, nan_cnt))) +
              __builtin_bit_cast(int, from_lane<L, 3>(__builtin_bit_cast(float, nan_cnt)));
  }
  float res;
  if constexpr (MODE == kMedian) {
    // sorted slots P/2-1 and P/2
    float zl, zh;
    if constexpr (L == 2) {
      zl = from_lane<L, 0>(v[127]);
      zh = from_lane<L, 1>(v[0]);
    } else {
      zl = from_lane<L, 1>(v[127]);
      zh = -from_lane<L, 3>(v[127]);
    }
    res = (n & 1) ? zl : (zl + zh) * 0.5f;
    if (nan_cnt > 0) res = qnan();
  } else {
    // ascending walk over [lo, hi) with one accumulator handed lane to lane
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < 128; ++r)
      if (r >= lo && r < hi) { if constexpr (!kExactB) asm volatile(""); acc += v[r]; }   // lane 0: slots 0..127
    acc = from_lane<L, 0>(acc);
#pragma unroll
    for (int r = 0; r < 128; ++r)
      if (128 + r >= lo && 128 + r < hi) { if constexpr (!kExactB) asm volatile(""); acc += v[r]; }   // lane 1
    acc = from_lane<L, 1>(acc);
    if constexpr (L == 4) {
#pragma unroll
      for (int r = 127; r >= 0; --r)
        if (383 - r >= lo && 383 - r < hi) { if constexpr (!kExactB) asm volatile(""); acc -= v[r]; }   // lane 3
      acc = from_lane<L, 3>(acc);
#pragma unroll
      for (int r = 127; r >= 0; --r)
        if (511 - r >= lo && 511 - r < hi) { if constexpr (!kExactB) asm volatile(""); acc -= v[r]; }   // lane 2
      acc = from_lane<L, 2>(acc);
    }
    res = acc / static_cast<float>(hi - lo);
    if (nan_cnt > n - hi) res = qnan();
  }
  if (h == 0 && c < rem) out[base + c] = res;
}

// ---------------------------------------------------------------------------
// LDS path for n > 128: a tile of T coordinates x Pn (next_pow2(n)) values,
// stored [position][coordinate] so that a wave's CE accesses hit 64 distinct
// banks; bitonic network by the whole workgroup; one lane per coordinate then
// reduces its sorted column in ascending order.
// ---------------------------------------------------------------------------
constexpr int kLdsFloats = 16384;  // 64 KiB tile

__global__ void __launch_bounds__(256) select_lds_kernel(const float* __restrict__ X, int n, int pn, int tile,
                                                        int64_t d, int64_t ldx, int mode, int lo, int hi,
                                                        float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * tile;
  const int tid = threadIdx.x;
  const int lt = __builtin_ctz(static_cast<unsigned>(tile));   // tile: a power of two
  // load: row-major sweep, consecutive lanes -> consecutive coordinates
  for (int e = tid; e < pn * tile; e += blockDim.x) {
    const int r = e >> lt, c = e & (tile - 1);
    const int64_t j = j0 + c;
    float x = qnan();
    if (r < n && j < d) x = X[(int64_t)r * ldx + j];
    lds[e] = x;
  }
  __syncthreads();
  const int pairs = (pn / 2) * tile;
  for (int k = 2; k <= pn; k <<= 1) {
    for (int s = k >> 1; s > 0; s >>= 1) {
      for (int q = tid; q < pairs; q += blockDim.x) {
        const int c = q & (tile - 1);
        const int h = q >> lt;                             // pair index within the column
        const int i = h + (h & ~(s - 1));   // lower element of the pair: (h / s) * 2s + h % s
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
      if (mode == kMedian) {
        if (n & 1) res = lds[((n - 1) / 2) * tile + tid];
        else res = (lds[(n / 2 - 1) * tile + tid] + lds[(n / 2) * tile + tid]) * 0.5f;
        if (__builtin_isnan(lds[(n - 1) * tile + tid])) res = qnan();
      } else {
        float acc = 0.f;
        for (int p = lo; p < hi; ++p) acc += lds[p * tile + tid];
        res = acc / static_cast<float>(hi - lo);
      }
      out[j] = res;
    }
  }
}

static int64_t num_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 256;
  return cus;
}

// Variant selection (the measured-fastest per shape).
template <int MODE>
static int launch_select(const float* X, int n, int64_t d, int64_t ldx, int lo, int hi, float* out,
                         hipStream_t s) {
  const int P = static_cast<int>(cdiv(n, 16) * 16);
  const bool trim128 = MODE == kTrimmed && n == 128 && lo == 12 && hi == 116;
  const bool trim100 = MODE == kTrimmed && n == 100 && lo == 10 && hi == 90;

  // Exact N = 128 / 100 (trimmed mean at beta = 0.1, median): the fused
  // three-input networks behind a NaN check (select_plain_kernel).
  if constexpr (MODE == kTrimmed || MODE == kMedian) {
    const int64_t blocks = cdiv(d, 256);
    if (trim128) {
      hipLaunchKernelGGL((select_plain_kernel<kTrimmed, 128, 12>), dim3(blocks), dim3(256), 0, s, X, d, ldx, out);
      return launch_status("select_plain_kernel");
    }
    if (trim100) {
      hipLaunchKernelGGL((select_plain_kernel<kTrimmed, 100, 10>), dim3(blocks), dim3(256), 0, s, X, d, ldx, out);
      return launch_status("select_plain_kernel");
    }
    if (MODE == kMedian && n == 128) {
      hipLaunchKernelGGL((select_plain_kernel<kMedian, 128, 0>), dim3(blocks), dim3(256), 0, s, X, d, ldx, out);
      return launch_status("select_plain_kernel");
    }
    if (MODE == kMedian && n == 100) {
      hipLaunchKernelGGL((select_plain_kernel<kMedian, 100, 0>), dim3(blocks), dim3(256), 0, s, X, d, ldx, out);
      return launch_status("select_plain_kernel");
    }
  }
  if (n <= 128) {
#define SRA_SEL1(PP, NXX, BXX)                                                                                   \
  do {                                                                                                           \
    hipLaunchKernelGGL((select_reg_kernel<PP, MODE, NXX, BXX, 256>), dim3(cdiv(d, 256)), dim3(256), 0, s, X, n,   \
                       d, ldx, lo, hi, out);                                                                     \
    return launch_status("select_reg_kernel");                                                                   \
  } while (0)
    switch (P) {
      case 16: SRA_SEL1(16, 0, -1);
      case 32: SRA_SEL1(32, 0, -1);
      case 48: SRA_SEL1(48, 0, -1);
      case 64: SRA_SEL1(64, 0, -1);
      case 80: SRA_SEL1(80, 0, -1);
      case 96: SRA_SEL1(96, 0, -1);
      case 112: SRA_SEL1(112, 0, -1);
      case 128: SRA_SEL1(128, 0, -1);
      default: break;
    }
#undef SRA_SEL1
  }
  // 128 < N <= 512: 2 or 4 lanes per coordinate, register-resident, DPP merges
  const bool quad_ok = ldx * 4 * 3 + 256 < (int64_t(1) << 32);   // 32-bit lane offsets
  if (quad_ok && n > 128 && n <= 256) {
    hipLaunchKernelGGL((select_quad_kernel<2, MODE>), dim3(cdiv(d, 128)), dim3(256), 0, s, X, n, d, ldx, lo, hi, out);
    return launch_status("select_quad_kernel");
  }
  if (quad_ok && n > 256 && n <= 512) {
    if (n == 512 && (MODE == kMedian || (lo == 51 && hi == 461))) {
      // plain loads: with streaming loads the half line a wave leaves for its
      // neighbour was refetched (median 1.12x the algorithmic bytes, 7.03 ms;
      // plain 1.00x, 6.83 ms at d = 1.25e7)
      hipLaunchKernelGGL((select_quad_kernel<4, MODE, 512, MODE == kMedian ? -1 : 51, false>), dim3(cdiv(d, 64)),
                         dim3(256), 0, s, X, n, d, ldx, lo, hi, out);
    } else {
      hipLaunchKernelGGL((select_quad_kernel<4, MODE>), dim3(cdiv(d, 64)), dim3(256), 0, s, X, n, d, ldx, lo, hi,
                         out);
    }
    return launch_status("select_quad_kernel");
  }
  const int pn = next_pow2(n);
  SRA_REQUIRE(pn <= kLdsFloats, SRA_ERR_UNSUPPORTED, "k-select supports N <= %d (got %d)", kLdsFloats, n);
  const int tile = kLdsFloats / pn;
  const int64_t lblocks = cdiv(d, tile);
  hipLaunchKernelGGL(select_lds_kernel, dim3(lblocks), dim3(256), sizeof(float) * pn * tile, s, X, n, pn, tile, d,
                     ldx, MODE, lo, hi, out);
  return launch_status("select_lds_kernel");
}

static int check_matrix(const float* X, int64_t n, int64_t d, int64_t ldx, const float* out) {
  SRA_REQUIRE(X != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= (1 << 20), SRA_ERR_SHAPE, "need 1 <= N <= 2^20 (got %lld)", (long long)n);
  SRA_REQUIRE(d >= 1, SRA_ERR_SHAPE, "need d >= 1 (got %lld)", (long long)d);
  SRA_REQUIRE(ldx >= d, SRA_ERR_SHAPE, "ldx (%lld) < d (%lld)", (long long)ldx, (long long)d);
  return SRA_OK;
}

}  // namespace sra

using namespace sra;

extern "C" int sra_average_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* out, void* stream) {
  int rc = check_matrix(X, n, d, ldx, out);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = (d % 4 == 0) && (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  if (vec) {
    const int64_t d4 = d / 4;
    hipLaunchKernelGGL(average_vec4_kernel, dim3(cdiv(d4, 256)), dim3(256), 0, s, X, (int)n, d4, ldx, out);
    return launch_status("average_vec4_kernel");
  }
  hipLaunchKernelGGL(average_kernel, dim3(cdiv(d, 256)), dim3(256), 0, s, X, (int)n, d, ldx, out);
  return launch_status("average_kernel");
}

extern "C" int sra_median_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* out, void* stream) {
  int rc = check_matrix(X, n, d, ldx, out);
  if (rc) return rc;
  return launch_select<kMedian>(X, (int)n, d, ldx, 0, (int)n, out, static_cast<hipStream_t>(stream));
}

extern "C" int sra_trimmed_mean_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t b, float* out,
                                    void* stream) {
  int rc = check_matrix(X, n, d, ldx, out);
  if (rc) return rc;
  SRA_REQUIRE(b >= 0, SRA_ERR_ARG, "trim count b must be >= 0 (got %d)", b);
  // numpy slices s[b : n-b]; an empty slice gives mean = NaN (0/0)
  const int lo = b, hi = (int)n - b;
  return launch_select<kTrimmed>(X, (int)n, d, ldx, lo, hi > lo ? hi : lo, out, static_cast<hipStream_t>(stream));
}

// The k-th order statistic of every column (sorted ascending, NaN anywhere in
// the column -> NaN).  k = (n-1)/2 is torch.median's lower median, which the
// DBA harness aggregates with (src/DBA/helper.py:561, :1025).  Runtime-N
// register network (n <= 128); the kept slot s[k] is summed alone and divided
// by 1, i.e. returned exactly.
// Order statistic for 128 < N <= 16384 (the DBA harness's torch.median lower
// median, src/DBA/helper.py:561, with more clients): a tile of `tile`
// coordinates x pn = next_pow2(N) slots in LDS ([slot][coordinate], so a
// wave's compare-exchanges hit distinct banks), bitonic-sorted by the whole
// workgroup in the NaN-last order of ce(); s[k], or NaN when the column holds
// one (then slot N - 1 is NaN): torch.median's answer.
constexpr int kOrderLdsFloats = 16384;   // 64 KiB tile
__global__ void __launch_bounds__(256) order_stat_lds_kernel(const float* __restrict__ X, int n, int64_t d,
                                                             int64_t ldx, int pn, int tile, int k,
                                                             float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];   // [pn][tile]
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * tile;
  const int tid = threadIdx.x;
  const int lt = __builtin_ctz(static_cast<unsigned>(tile));   // tile: a power of two
  for (int e = tid; e < pn * tile; e += blockDim.x) {
    const int r = e >> lt, c = e & (tile - 1);
    const int64_t j = j0 + c;
    lds[e] = (r < n && j < d) ? X[static_cast<int64_t>(r) * ldx + j] : qnan();
  }
  __syncthreads();
  const int pairs = (pn / 2) * tile;
  for (int kk = 2; kk <= pn; kk <<= 1) {
    for (int st = kk >> 1; st > 0; st >>= 1) {
      for (int q = tid; q < pairs; q += blockDim.x) {
        const int c = q & (tile - 1);
        const int h = q >> lt;
        const int i = h + (h & ~(st - 1));   // (h / st) * 2st + h % st, st a power of two
        const int l = i + st;
        float a = lds[i * tile + c], b = lds[l * tile + c];
        if ((i & kk) == 0) ce(a, b); else ce(b, a);
        lds[i * tile + c] = a;
        lds[l * tile + c] = b;
      }
      __syncthreads();
    }
  }
  if (tid < tile) {
    const int64_t j = j0 + tid;
    if (j < d) out[j] = __builtin_isnan(lds[(n - 1) * tile + tid]) ? qnan() : lds[k * tile + tid];
  }
}

extern "C" int sra_order_stat_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t k, float* out,
                                  void* stream) {
  int rc = check_matrix(X, n, d, ldx, out);
  if (rc) return rc;
  SRA_REQUIRE(n <= kOrderLdsFloats, SRA_ERR_UNSUPPORTED, "order statistic supports N <= %d (got %lld)",
              kOrderLdsFloats, (long long)n);
  SRA_REQUIRE(k >= 0 && k < n, SRA_ERR_ARG, "order statistic k=%d out of [0, %lld)", k, (long long)n);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n > 128) {
    const int pn = next_pow2(static_cast<int>(n));
    const int tile = kOrderLdsFloats / pn;
    const size_t lds = sizeof(float) * static_cast<size_t>(pn) * tile;
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&order_stat_lds_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    hipLaunchKernelGGL(order_stat_lds_kernel, dim3(cdiv(d, tile)), dim3(256), lds, s, X, static_cast<int>(n), d, ldx,
                       pn, tile, static_cast<int>(k), out);
    return launch_status("order_stat_lds_kernel");
  }
  const int P = static_cast<int>(cdiv(n, 16) * 16);
  const int64_t blocks = cdiv(d, 256);
#define SRA_ORD(PP)                                                                                                  \
  case PP:                                                                                                           \
    hipLaunchKernelGGL((select_reg_kernel<PP, kOrder, 0, -1, 256>), dim3(blocks), dim3(256), 0, s, X, (int)n, d, ldx, \
                       (int)k, (int)k + 1, out);                                                                     \
    return launch_status("select_reg_kernel");
  switch (P) {
    SRA_ORD(16) SRA_ORD(32) SRA_ORD(48) SRA_ORD(64) SRA_ORD(80) SRA_ORD(96) SRA_ORD(112) SRA_ORD(128)
    default: break;
  }
#undef SRA_ORD
  set_error("order statistic: unsupported N %lld", (long long)n);
  return SRA_ERR_UNSUPPORTED;
}
