// Shared helpers for the SRA (secure robust aggregation) HIP library.
// gfx950 (MI355X / CDNA4) only: wave64, 256 CUs in 8 XCDs.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>
#include <cmath>
#include <limits>
#include <utility>

#include "../../include/sra.h"

namespace sra {

// thread-local last-error text (sra_last_error)
void set_error(const char* fmt, ...);
const char* last_error();

#define SRA_REQUIRE(cond, code, ...)        \
  do {                                      \
    if (!(cond)) {                          \
      ::sra::set_error(__VA_ARGS__);        \
      return (code);                        \
    }                                       \
  } while (0)

#define SRA_HIP(call)                                                              \
  do {                                                                             \
    hipError_t _e = (call);                                                        \
    if (_e != hipSuccess) {                                                        \
      ::sra::set_error("%s failed: %s", #call, hipGetErrorString(_e));             \
      return SRA_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

// check the launch that was just queued
inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch of %s failed: %s", what, hipGetErrorString(e));
    return SRA_ERR_HIP;
  }
  return SRA_OK;
}

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// Row indices read from device row lists (Krum / Bulyan selections, gathers)
// go through checked_row: an index outside the matrix is clamped so it cannot
// address outside it, AND counted in this translation unit's fault counter
// (a vector atomic), which sra_row_fault_count() reports -- the GPU tests
// assert it stays 0.  Built with -DSRA_DEVICE_ASSERT (make DEVICE_ASSERT=1)
// the kernel traps on it instead.
// ---------------------------------------------------------------------------
static __device__ unsigned int g_row_faults;

__device__ __forceinline__ int checked_row(int row, int nrows) {
  if (static_cast<unsigned>(row) >= static_cast<unsigned>(nrows)) {
#ifdef SRA_DEVICE_ASSERT
    __builtin_trap();
#else
    atomicAdd(&g_row_faults, 1u);
#endif
  }
  return static_cast<int>(min(static_cast<unsigned>(row), static_cast<unsigned>(nrows - 1)));
}

// this translation unit's fault count (and reset); synchronous
static inline unsigned int tu_row_faults(bool reset) {
  unsigned int v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_row_faults), sizeof(v), 0, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  if (reset) {
    const unsigned int z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_row_faults), &z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return v;
}
unsigned int krum_row_faults(bool reset);
unsigned int bulyan_row_faults(bool reset);

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ constexpr int next_pow2(int x) { int p = 1; while (p < x) p <<= 1; return p; }

// ---------------------------------------------------------------------------
// Compare-exchange with NaN-last ordering.  lo = minNum (drops a NaN operand),
// hi = IEEE-754-2019 maximum (propagates it): every CE is a permutation of its
// inputs under the order "reals ascending, then NaN", which is numpy's sort
// order.  On gfx950 this is v_min_f32 + v_maximum3_f32, both full rate.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ce(float& a, float& b) {
  const float lo = __builtin_fminf(a, b);
  const float hi = __builtin_elementwise_maximum(a, b);
  a = lo;
  b = hi;
}

// ---------------------------------------------------------------------------
// Sorting-network planner (all constexpr).
//
// Two base networks on P2 = 2^k slots:
//   kNetSort  — Batcher's odd-even merge sort (sorts anything);
//   kNetMerge — bitonic half-cleaner cascade (sorts a bitonic sequence).
// Slots [PR, P2) hold a compile-time "top" value (sorts after everything), so
// the forward pass folds every CE that touches them: (x, top) is a no-op,
// (top, x) is a register move.  A backward pass then keeps only the cone of
// the requested output slots [OLO, OHI): a CE with one live output becomes a
// single min or max, one with none is dropped.  The resulting op list is
// expanded with immediate register indices.
// ---------------------------------------------------------------------------
enum NetOpKind : int { kOpCE = 0, kOpMin = 1, kOpMax = 2, kOpMove = 3 };
// kNetFrom4: odd-even merges only, for inputs whose aligned blocks of 4 are
// already sorted (sort4_blocks below does that with 3-input min/med/max).
enum NetKind : int { kNetSort = 0, kNetMerge = 1, kNetFrom4 = 2 };

template <int P2, int KIND>
struct BaseNet {
  template <typename F>
  static constexpr void each(F&& f) {
    if constexpr (KIND == kNetFrom4) {
      from4(f, 0, P2);
    } else if constexpr (KIND == kNetSort) {
      // depth-first Batcher odd-even merge sort: sort(lo half), sort(hi half),
      // merge.  Same comparators as the stage-major form, but the first rows'
      // sub-sort only reads the first loads, so a wave starts sorting while
      // the rest of its column is still in flight.
      sort_hybrid(f, 0, P2);
    } else {
      for (int s = P2 / 2; s >= 1; s >>= 1)
        for (int i = 0; i < P2; ++i)
          if ((i & s) == 0) f(i, i + s);
    }
  }
  template <typename F>
  static constexpr void merge_rec(F& f, int lo, int n, int r) {
    const int step = r * 2;
    if (step < n) {
      merge_rec(f, lo, n, step);
      merge_rec(f, lo + r, n, step);
      for (int i = lo + r; i + r < lo + n; i += step) f(i, i + r);
    } else {
      f(lo, lo + r);
    }
  }
  // stage-major odd-even merge of the two sorted halves of [lo, lo+n)
  template <typename F>
  static constexpr void merge_stages(F& f, int lo, int n) {
    const int p = n / 2;
    for (int k = p; k >= 1; k >>= 1)
      for (int j = k % p; j + k < n; j += 2 * k)
        for (int i = 0; i < k && i + j + k < n; ++i) f(lo + i + j, lo + i + j + k);
  }
  // stage-major odd-even merge sort of [lo, lo+n)
  template <typename F>
  static constexpr void sort_stages(F& f, int lo, int n) {
    for (int p = 1; p < n; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < n; j += 2 * k)
          for (int i = 0; i < k && i + j + k < n; ++i)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) f(lo + i + j, lo + i + j + k);
  }
  // depth-first over blocks of kBlock rows (a wave starts sorting its first
  // rows while later loads are in flight), stage-major inside a block and in
  // each merge (consecutive comparators independent -> wide asm groups and
  // few dependent asm boundaries)
  static constexpr int kBlock = 32;
  // 16-input sorting network with 60 comparators (Green; the best known size,
  // 3 fewer than Batcher's 63), 10 layers.  Checked exhaustively with the 0-1
  // principle in tests/test_networks.py.
  static constexpr short kGreen16[60][2] = {
      {0, 13}, {1, 12}, {2, 15}, {3, 14}, {4, 8}, {5, 6}, {7, 11}, {9, 10},
      {0, 5}, {1, 7}, {2, 9}, {3, 4}, {6, 13}, {8, 14}, {10, 15}, {11, 12},
      {0, 1}, {2, 3}, {4, 5}, {6, 8}, {7, 9}, {10, 11}, {12, 13}, {14, 15},
      {0, 2}, {1, 3}, {4, 10}, {5, 11}, {6, 7}, {8, 9}, {12, 14}, {13, 15},
      {1, 2}, {3, 12}, {4, 6}, {5, 7}, {8, 10}, {9, 11}, {13, 14},
      {1, 4}, {2, 6}, {5, 8}, {7, 10}, {9, 13}, {11, 14},
      {2, 4}, {3, 6}, {9, 12}, {11, 13},
      {3, 5}, {6, 8}, {7, 9}, {10, 12},
      {3, 4}, {5, 6}, {7, 8}, {9, 10}, {11, 12},
      {6, 7}, {8, 9}};
  template <typename F>
  static constexpr void sort_hybrid(F& f, int lo, int n) {
    if (n == 16) {
      for (int q = 0; q < 60; ++q) f(lo + kGreen16[q][0], lo + kGreen16[q][1]);
      return;
    }
    if (n == 32) {   // 2 x 60 + 65 = 185 comparators (Batcher: 191)
      sort_hybrid(f, lo, 16);
      sort_hybrid(f, lo + 16, 16);
      merge_stages(f, lo, 32);
      return;
    }
    if (n <= kBlock) {
      sort_stages(f, lo, n);
      return;
    }
    sort_hybrid(f, lo, n / 2);
    sort_hybrid(f, lo + n / 2, n / 2);
    merge_stages(f, lo, n);
  }
  template <typename F>
  static constexpr void from4(F& f, int lo, int n) {
    if (n <= 4) return;
    from4(f, lo, n / 2);
    from4(f, lo + n / 2, n / 2);
    merge_stages(f, lo, n);
  }
  template <typename F>
  static constexpr void sort_rec(F& f, int lo, int n) {
    if (n > 1) {
      const int m = n / 2;
      sort_rec(f, lo, m);
      sort_rec(f, lo + m, m);
      merge_rec(f, lo, n, 1);
    }
  }
  static constexpr int count() {
    int c = 0;
    each([&](int, int) { ++c; });
    return c > 0 ? c : 1;
  }
  static constexpr int N = count();
};

template <int P2, int PR, int OLO, int OHI, int KIND>
struct NetPlanData {
  static constexpr int NF = BaseNet<P2, KIND>::N;
  int n = 0;
  short kind[NF] = {};
  short a[NF] = {};
  short b[NF] = {};
  constexpr NetPlanData() {
    short fk[NF] = {}, fa[NF] = {}, fb[NF] = {};
    bool cst[P2] = {};
    for (int i = 0; i < P2; ++i) cst[i] = i >= PR;
    int m = 0;
    BaseNet<P2, KIND>::each([&](int x, int y) {
      if (cst[y]) return;                           // (v, top): already ordered
      if (cst[x]) {                                 // (top, v): move v down
        fk[m] = kOpMove; fa[m] = x; fb[m] = y; ++m;
        cst[x] = false; cst[y] = true;
        return;
      }
      fk[m] = kOpCE; fa[m] = x; fb[m] = y; ++m;
    });
    bool need[P2] = {};
    for (int i = OLO; i < OHI; ++i) need[i] = true;
    bool keep[NF] = {};
    for (int q = m - 1; q >= 0; --q) {
      const int x = fa[q], y = fb[q];
      if (fk[q] == kOpMove) {
        keep[q] = need[x];
        need[y] = need[x];
        need[x] = false;
        continue;
      }
      const bool nx = need[x], ny = need[y];
      if (!nx && !ny) { keep[q] = false; continue; }
      keep[q] = true;
      fk[q] = (nx && ny) ? kOpCE : (nx ? kOpMin : kOpMax);
      need[x] = need[y] = true;
    }
    for (int q = 0; q < m; ++q)
      if (keep[q]) { kind[n] = fk[q]; a[n] = fa[q]; b[n] = fb[q]; ++n; }
    // greedy groups of up to kGroup consecutive, mutually independent CEs
    // (one inline-asm statement each; other ops are groups of one)
    int q = 0;
    while (q < n) {
      gstart[ngroups] = q;
      int len = 1;
      if (kind[q] == kOpCE) {
        while (q + len < n && len < kGroup && kind[q + len] == kOpCE) {
          bool clash = false;
          for (int t = q; t < q + len; ++t)
            if (a[t] == a[q + len] || a[t] == b[q + len] || b[t] == a[q + len] || b[t] == b[q + len]) clash = true;
          if (clash) break;
          ++len;
        }
      }
      glen[ngroups] = len;
      ++ngroups;
      q += len;
    }
  }
  static constexpr int kGroup = 4;
  int ngroups = 0;
  short gstart[NF] = {};
  short glen[NF] = {};
};

// evaluated once per instantiation
template <int P2, int PR, int OLO, int OHI, int KIND = kNetSort>
struct NetPlan {
  static constexpr NetPlanData<P2, PR, OLO, OHI, KIND> value{};
};

// One compare-exchange as an indivisible pair (lo into a fresh register, hi in
// place of b): keeps the live set at P+1 values however the scheduler orders
// the independent CEs of a stage.  NaN-last semantics as ce().
__device__ __forceinline__ void ce_pair(float& a, float& b) {
  float lo;
  asm("v_min_f32 %0, %2, %1\n\tv_maximum3_f32 %1, %2, %1, %1" : "=&v"(lo), "+v"(b) : "v"(a));
  a = lo;
}

// Up to four independent NaN-free compare-exchanges in ONE asm statement:
// lo into a fresh register, hi in place.  The asm keeps the CE order (and
// therefore the live set at ~P values); grouping keeps the compiler's
// conservative post-asm hazard padding (one s_nop per dependent asm boundary)
// to one per group.  IEEE-754-2019 minimum/maximum need no canonicalised
// operands; callers map NaN to +inf beforehand.
__device__ __forceinline__ void ce_asm1(float& a0, float& b0) {
  float l0;
  asm("v_minimum3_f32 %0, %2, %1, %1\n\tv_maximum3_f32 %1, %2, %1, %1" : "=&v"(l0), "+v"(b0) : "v"(a0));
  a0 = l0;
}
__device__ __forceinline__ void ce_asm2(float& a0, float& b0, float& a1, float& b1) {
  float l0, l1;
  asm("v_minimum3_f32 %0, %4, %2, %2\n\tv_maximum3_f32 %2, %4, %2, %2\n\t"
      "v_minimum3_f32 %1, %5, %3, %3\n\tv_maximum3_f32 %3, %5, %3, %3"
      : "=&v"(l0), "=&v"(l1), "+v"(b0), "+v"(b1) : "v"(a0), "v"(a1));
  a0 = l0; a1 = l1;
}
__device__ __forceinline__ void ce_asm3(float& a0, float& b0, float& a1, float& b1, float& a2, float& b2) {
  float l0, l1, l2;
  asm("v_minimum3_f32 %0, %6, %3, %3\n\tv_maximum3_f32 %3, %6, %3, %3\n\t"
      "v_minimum3_f32 %1, %7, %4, %4\n\tv_maximum3_f32 %4, %7, %4, %4\n\t"
      "v_minimum3_f32 %2, %8, %5, %5\n\tv_maximum3_f32 %5, %8, %5, %5"
      : "=&v"(l0), "=&v"(l1), "=&v"(l2), "+v"(b0), "+v"(b1), "+v"(b2) : "v"(a0), "v"(a1), "v"(a2));
  a0 = l0; a1 = l1; a2 = l2;
}
__device__ __forceinline__ void ce_asm4(float& a0, float& b0, float& a1, float& b1, float& a2, float& b2,
                                        float& a3, float& b3) {
  float l0, l1, l2, l3;
  asm("v_minimum3_f32 %0, %8, %4, %4\n\tv_maximum3_f32 %4, %8, %4, %4\n\t"
      "v_minimum3_f32 %1, %9, %5, %5\n\tv_maximum3_f32 %5, %9, %5, %5\n\t"
      "v_minimum3_f32 %2, %10, %6, %6\n\tv_maximum3_f32 %6, %10, %6, %6\n\t"
      "v_minimum3_f32 %3, %11, %7, %7\n\tv_maximum3_f32 %7, %11, %7, %7"
      : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
  a0 = l0; a1 = l1; a2 = l2; a3 = l3;
}

template <typename Plan, int G, int P2>
__device__ __forceinline__ void net_group(float (&v)[P2]) {
  // every index is forced through a constexpr so it becomes an immediate
  // register number (a plain use of the table would be a runtime load)
  constexpr int q = Plan::value.gstart[G], len = Plan::value.glen[G];
  constexpr int kd = Plan::value.kind[q];
  constexpr int a0 = Plan::value.a[q], b0 = Plan::value.b[q];
  constexpr int a1 = len > 1 ? Plan::value.a[q + 1] : 0, b1 = len > 1 ? Plan::value.b[q + 1] : 0;
  constexpr int a2 = len > 2 ? Plan::value.a[q + 2] : 0, b2 = len > 2 ? Plan::value.b[q + 2] : 0;
  constexpr int a3 = len > 3 ? Plan::value.a[q + 3] : 0, b3 = len > 3 ? Plan::value.b[q + 3] : 0;
  if constexpr (kd == kOpCE) {
    if constexpr (len == 1) ce_asm1(v[a0], v[b0]);
    else if constexpr (len == 2) ce_asm2(v[a0], v[b0], v[a1], v[b1]);
    else if constexpr (len == 3) ce_asm3(v[a0], v[b0], v[a1], v[b1], v[a2], v[b2]);
    else ce_asm4(v[a0], v[b0], v[a1], v[b1], v[a2], v[b2], v[a3], v[b3]);
  } else if constexpr (kd == kOpMin) {
    v[a0] = __builtin_elementwise_minimum(v[a0], v[b0]);
  } else if constexpr (kd == kOpMax) {
    v[b0] = __builtin_elementwise_maximum(v[a0], v[b0]);
  } else {
    v[a0] = v[b0];
  }
}

template <typename Plan, int P2, size_t... G>
__device__ __forceinline__ void net_run_groups(float (&v)[P2], std::index_sequence<G...>) {
  (net_group<Plan, G>(v), ...);
}

// NaN-free sort of (the requested slots of) v[0..P2): slots [PR, P2) are
// implicit +inf; on return slots [OLO, OHI) hold ascending order statistics.
template <int P2, int PR, int OLO, int OHI, int KIND = kNetSort>
__device__ __forceinline__ void network_fast(float (&v)[P2]) {
  using Plan = NetPlan<P2, PR, OLO, OHI, KIND>;
  if constexpr (P2 > 1) net_run_groups<Plan>(v, std::make_index_sequence<Plan::value.ngroups>{});
}

template <typename Plan, int Q, int P2>
__device__ __forceinline__ void net_op(float (&v)[P2]) {
  constexpr int kd = Plan::value.kind[Q], x = Plan::value.a[Q], y = Plan::value.b[Q];
  if constexpr (kd == kOpCE) ce_pair(v[x], v[y]);
  else if constexpr (kd == kOpMin) v[x] = __builtin_fminf(v[x], v[y]);
  else if constexpr (kd == kOpMax) v[y] = __builtin_elementwise_maximum(v[x], v[y]);
  else v[x] = v[y];
}

template <typename Plan, int P2, size_t... Q>
__device__ __forceinline__ void net_run(float (&v)[P2], std::index_sequence<Q...>) {
  (net_op<Plan, Q>(v), ...);
}

// Sort (the requested slots of) v[0..P2): slots [0, PR) are live values,
// [PR, P2) are implicit "top" values; on return slots [OLO, OHI) hold the
// ascending order statistics (NaN last).  P2 must be a power of two >= PR.
template <int P2, int PR, int OLO, int OHI>
__device__ __forceinline__ void sort_network(float (&v)[P2]) {
  using Plan = NetPlan<P2, PR, OLO, OHI, kNetSort>;
  if constexpr (P2 > 1) net_run<Plan>(v, std::make_index_sequence<Plan::value.n>{});
}

// Sort a bitonic sequence v[0..P2) ascending (bitonic half-cleaner cascade).
template <int P2>
__device__ __forceinline__ void bitonic_merge(float (&v)[P2]) {
  using Plan = NetPlan<P2, P2, 0, P2, kNetMerge>;
  if constexpr (P2 > 1) net_run<Plan>(v, std::make_index_sequence<Plan::value.n>{});
}

// Plain (NaN-free) variants, used after NaNs have been mapped to +inf (their
// count is tracked separately).  CE form CEF:
//   0: lo = v_min_f32, hi = v_max_f32 (4-byte VOP2 each);
//   1: hi recovered as a ^ b ^ lo with one v_bitop3_b32 (truth table 0x96 =
//      xor3): v_min_f32 of two non-NaN values returns one of its operands bit
//      for bit (fp32 denormals are preserved in these kernels, +-0 are both
//      operands), so the xor of all three is exactly the other one;
// Form 1 is 1.5-3.5 % faster than form 0 on register-resident columns
// (tools/ubench/net_rate.hip) but 3 % SLOWER in select_plain_kernel, whose
// clock is power-limited by the HBM stream beside the VALU (three register
// reads per xor3 against two per max): the product uses form 0.
template <int CEF>
__device__ __forceinline__ void ce_pair_plain(float& a, float& b) {
  float lo;
  if constexpr (CEF == 0)
    asm("v_min_f32 %0, %2, %1\n\tv_max_f32 %1, %2, %1" : "=&v"(lo), "+v"(b) : "v"(a));
  else
    asm("v_min_f32 %0, %2, %1\n\tv_bitop3_b32 %1, %2, %1, %0 bitop3:0x96" : "=&v"(lo), "+v"(b) : "v"(a));
  a = lo;
}

template <typename Plan, int Q, int P2, int CEF>
__device__ __forceinline__ void net_op_plain(float (&v)[P2]) {
  constexpr int kd = Plan::value.kind[Q], x = Plan::value.a[Q], y = Plan::value.b[Q];
  if constexpr (kd == kOpCE) ce_pair_plain<CEF>(v[x], v[y]);
  else if constexpr (kd == kOpMin) v[x] = __builtin_fminf(v[x], v[y]);
  else if constexpr (kd == kOpMax) v[y] = __builtin_fmaxf(v[x], v[y]);
  else v[x] = v[y];
}

template <typename Plan, int P2, int CEF, size_t... Q>
__device__ __forceinline__ void net_run_plain(float (&v)[P2], std::index_sequence<Q...>) {
  (net_op_plain<Plan, Q, P2, CEF>(v), ...);
}

template <int P2, int PR, int OLO, int OHI, int KIND, int CEF = 0>
__device__ __forceinline__ void network_plain(float (&v)[P2]) {
  using Plan = NetPlan<P2, PR, OLO, OHI, KIND>;
  if constexpr (P2 > 1) net_run_plain<Plan, P2, CEF>(v, std::make_index_sequence<Plan::value.n>{});
}

// ---------------------------------------------------------------------------
// Straight-line three-input networks (tools/fuse_net.py -> csrc/net_fused_*.inc).
// A merge network's compare-exchange pair whose one output feeds a single
// later compare-exchange is folded into that consumer as min3 / max3 / med3 of
// the pair's inputs (valid where the 0-1 principle says so), e.g. for the
// north-star network 2,554 -> 1,888 VALU ops.  Prog::k* are the constexpr
// tables (kind, dst, a, b, c) over register slots v[0 .. Prog::kSlots) (the
// CPU tests re-run them), Prog::run the same program as code; NaN-free inputs
// (callers map NaN to +inf first).
// ---------------------------------------------------------------------------
// Prog::run is the program as inline asm, a few ops per statement: with
// builtins the compiler re-splits min3 / max3 into shared two-input mins,
// canonicalises med3 operands and hoists for ILP (259 registers at N = 128:
// one wave per SIMD); asm keeps the generator's order and its bounded live
// set (221), and grouping cuts the hazard s_nops the compiler puts after
// dependent asm boundaries.
template <class Prog, int S>
__device__ __forceinline__ void fused_network(float (&v)[S]) {
  Prog::run(v);
}

// In-place form for a full sort of v[0 .. 128): the program runs on a
// kSlots-wide copy and the ranks are read back in order (register renaming,
// no moves unless the allocator needs them).
template <class Prog>
__device__ __forceinline__ void fused_sort128(float (&v)[128]) {
  static_assert(Prog::kOuts == 128, "a full 128-value program");
  float w[Prog::kSlots > 128 ? Prog::kSlots : 128];
#pragma unroll
  for (int i = 0; i < 128; ++i) w[i] = v[i];
  fused_network<Prog>(w);
#pragma unroll
  for (int i = 0; i < 128; ++i) v[i] = w[Prog::kOut[i]];
}

// Sort the aligned blocks of 4 of v[0..PR) (NaN-free) with 7 VALU ops each
// instead of 5 compare-exchanges (10 ops): a 3-sorter (min3, med3, max3) and
// an insertion of the 4th value, whose sorted position is
//   [min(s0,d), med3(s0,s1,d), med3(s1,s2,d), max(s2,d)]  (s0 <= s1 <= s2).
// Blocks at or beyond PR are compile-time padding and skipped.
template <int PR, int P2>
__device__ __forceinline__ void sort4_blocks(float (&v)[P2]) {
#pragma unroll
  for (int b = 0; b + 4 <= PR; b += 4) {
    const float a0 = v[b], a1 = v[b + 1], a2 = v[b + 2], d = v[b + 3];
    const float s0 = __builtin_fminf(__builtin_fminf(a0, a1), a2);
    const float s1 = __builtin_amdgcn_fmed3f(a0, a1, a2);
    const float s2 = __builtin_fmaxf(__builtin_fmaxf(a0, a1), a2);
    v[b] = __builtin_fminf(s0, d);
    v[b + 1] = __builtin_amdgcn_fmed3f(s0, s1, d);
    v[b + 2] = __builtin_amdgcn_fmed3f(s1, s2, d);
    v[b + 3] = __builtin_fmaxf(s2, d);
  }
  static_assert(PR % 4 == 0, "sort4_blocks needs whole blocks");
}

// As sort4_blocks, but the block maximum (slot 3) is computed with the
// NaN-PROPAGATING IEEE-754-2019 maximum: a NaN anywhere in a block makes its
// slot 3 NaN, so a max3 over the slots 3 (PR/8 ops) detects NaNs in the whole
// column.  The other slots are unspecified when a block holds a NaN (the
// caller then reloads, maps NaN -> +inf and uses sort4_blocks).
template <int PR, int P2>
__device__ __forceinline__ float sort4_blocks_nancheck(float (&v)[P2]) {
  static_assert(PR % 4 == 0, "sort4_blocks needs whole blocks");
#pragma unroll
  for (int b = 0; b + 4 <= PR; b += 4) {
    const float a0 = v[b], a1 = v[b + 1], a2 = v[b + 2], d = v[b + 3];
    const float s0 = __builtin_fminf(__builtin_fminf(a0, a1), a2);
    const float s1 = __builtin_amdgcn_fmed3f(a0, a1, a2);
    const float s2 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a0, a1), a2);
    // IEEE-754-2019 minimum: no operand canonicalisation (fminf of a loaded
    // value costs an extra v_max_f32 x, x, x per block in IEEE mode)
    v[b] = __builtin_elementwise_minimum(s0, d);
    v[b + 1] = __builtin_amdgcn_fmed3f(s0, s1, d);
    v[b + 2] = __builtin_amdgcn_fmed3f(s1, s2, d);
    v[b + 3] = __builtin_elementwise_maximum(s2, d);
  }
  float m = v[3];
#pragma unroll
  for (int b = 4; b + 4 <= PR; b += 8) {
    const float hi = b + 4 < PR ? v[b + 7] : v[b + 3];
    m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m, v[b + 3]), hi);
  }
  return m;
}

// DPP lane exchange with the neighbour lane (quad_perm [1,0,3,2]: 2c <-> 2c+1)
__device__ __forceinline__ float swap_adjacent(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

__device__ __forceinline__ float qnan() { return __builtin_nanf(""); }

// numpy pairwise fp64 sum of f(0..n) for n <= 128 (eight accumulators)
template <typename F>
__device__ __forceinline__ double np_pw_block64(int n, F&& f) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += f(i);
    return res;
  }
  double r0 = f(0), r1 = f(1), r2 = f(2), r3 = f(3), r4 = f(4), r5 = f(5), r6 = f(6), r7 = f(7);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += f(i); r1 += f(i + 1); r2 += f(i + 2); r3 += f(i + 3);
    r4 += f(i + 4); r5 += f(i + 5); r6 += f(i + 6); r7 += f(i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += f(i);
  return res;
}

// numpy's pairwise fp64 sum of f(lo .. lo + n), n <= 512: numpy splits while
// a piece holds more than 128 elements; from n <= 512 the largest piece after
// three splits is <= 76, so three levels are exact
template <typename F>
__device__ __forceinline__ double np_pw64(int lo, int n, F&& f) {
  if (n <= 128) return np_pw_block64(n, [&](int i) { return f(lo + i); });
  auto quarter = [&](int l2, int m2) -> double {
    if (m2 <= 128) return np_pw_block64(m2, [&](int i) { return f(l2 + i); });
    int q = m2 / 2;
    q -= q % 8;
    return np_pw_block64(q, [&](int i) { return f(l2 + i); }) +
           np_pw_block64(m2 - q, [&](int i) { return f(l2 + q + i); });
  };
  auto half = [&](int l2, int m2) -> double {
    if (m2 <= 128) return np_pw_block64(m2, [&](int i) { return f(l2 + i); });
    int q = m2 / 2;
    q -= q % 8;
    return quarter(l2, q) + quarter(l2 + q, m2 - q);
  };
  int n2 = n / 2;
  n2 -= n2 % 8;
  return half(lo, n2) + half(lo + n2, n - n2);
}

// numpy's pairwise sum at any split depth (fp64 / fp32): DEPTH levels of the
// split at n/2 rounded down to a multiple of 8 cover n <= 128 * 2^DEPTH - 16.
// Used by the N > 512 paths; np_pw64 above stays the <= 512 form.
template <int DEPTH, typename F>
__device__ __forceinline__ double np_pw64_rec(int lo, int n, F&& f) {
  if constexpr (DEPTH == 0) {
    return np_pw_block64(n, [&](int i) { return f(lo + i); });
  } else {
    if (n <= 128) return np_pw_block64(n, [&](int i) { return f(lo + i); });
    int q = n / 2;
    q -= q % 8;
    const double a = np_pw64_rec<DEPTH - 1>(lo, q, f);
    return a + np_pw64_rec<DEPTH - 1>(lo + q, n - q, f);
  }
}

template <typename F>
__device__ __forceinline__ float np_pw_block32(int n, F&& f) {
  if (n < 8) {
    float res = 0.f;
    for (int i = 0; i < n; ++i) res += f(i);
    return res;
  }
  float r0 = f(0), r1 = f(1), r2 = f(2), r3 = f(3), r4 = f(4), r5 = f(5), r6 = f(6), r7 = f(7);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += f(i); r1 += f(i + 1); r2 += f(i + 2); r3 += f(i + 3);
    r4 += f(i + 4); r5 += f(i + 5); r6 += f(i + 6); r7 += f(i + 7);
  }
  float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += f(i);
  return res;
}

template <int DEPTH, typename F>
__device__ __forceinline__ float np_pw32_rec(int lo, int n, F&& f) {
  if constexpr (DEPTH == 0) {
    return np_pw_block32(n, [&](int i) { return f(lo + i); });
  } else {
    if (n <= 128) return np_pw_block32(n, [&](int i) { return f(lo + i); });
    int q = n / 2;
    q -= q % 8;
    const float a = np_pw32_rec<DEPTH - 1>(lo, q, f);
    return a + np_pw32_rec<DEPTH - 1>(lo + q, n - q, f);
  }
}

}  // namespace sra
