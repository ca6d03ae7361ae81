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
// Batcher's odd-even merge sort on P2 = 2^k slots.  Slots [PR, P2) hold a
// compile-time NaN (they sort last), so the forward pass folds every CE that
// touches them: (x, NaN) is a no-op, (NaN, x) is a register move.  A backward
// pass then keeps only the cone of the requested output slots [OLO, OHI): a CE
// with one live output becomes a single min or max, one with none is dropped.
// The result is an op list whose indices are immediates after expansion.
// ---------------------------------------------------------------------------
enum NetOpKind : int { kOpCE = 0, kOpMin = 1, kOpMax = 2, kOpMove = 3 };

template <int P2>
struct OddEvenFull {
  static constexpr int count() {
    int c = 0;
    for (int p = 1; p < P2; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < P2; j += 2 * k)
          for (int i = 0; i < k && i + j + k < P2; ++i)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) ++c;
    return c;
  }
  static constexpr int N = count() > 0 ? count() : 1;
};

template <int P2, int PR, int OLO, int OHI>
struct NetPlanData {
  static constexpr int NF = OddEvenFull<P2>::N;
  int n = 0;
  short kind[NF] = {};
  short a[NF] = {};
  short b[NF] = {};
  constexpr NetPlanData() {
    // forward: full network with constant-NaN folding
    short fk[NF] = {}, fa[NF] = {}, fb[NF] = {};
    bool cst[P2] = {};
    for (int i = 0; i < P2; ++i) cst[i] = i >= PR;
    int m = 0;
    for (int p = 1; p < P2; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < P2; j += 2 * k)
          for (int i = 0; i < k && i + j + k < P2; ++i)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) {
              const int x = i + j, y = i + j + k;
              if (cst[y]) continue;                       // (v, NaN): already ordered
              if (cst[x]) {                               // (NaN, v): move v down
                fk[m] = kOpMove; fa[m] = x; fb[m] = y; ++m;
                cst[x] = false; cst[y] = true;
                continue;
              }
              fk[m] = kOpCE; fa[m] = x; fb[m] = y; ++m;
            }
    // backward: keep the cone of the requested outputs
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
  }
};

// evaluated once per (P2, PR, OLO, OHI)
template <int P2, int PR, int OLO, int OHI>
struct NetPlan {
  static constexpr NetPlanData<P2, PR, OLO, OHI> value{};
};

// One compare-exchange as an indivisible pair (lo into a fresh register, hi in
// place of b): keeps the live set at P+1 values however the scheduler orders
// the independent CEs of a stage.  NaN-last semantics as ce().
__device__ __forceinline__ void ce_pair(float& a, float& b) {
  float lo;
  asm("v_min_f32 %0, %2, %1\n\tv_maximum3_f32 %1, %2, %1, %1" : "=&v"(lo), "+v"(b) : "v"(a));
  a = lo;
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
// [PR, P2) are implicit NaN; on return slots [OLO, OHI) hold the ascending
// order statistics (NaN last).  P2 must be a power of two >= PR.
template <int P2, int PR, int OLO, int OHI>
__device__ __forceinline__ void sort_network(float (&v)[P2]) {
  using Plan = NetPlan<P2, PR, OLO, OHI>;
  if constexpr (P2 > 1) net_run<Plan>(v, std::make_index_sequence<Plan::value.n>{});
}

__device__ __forceinline__ float qnan() { return __builtin_nanf(""); }

}  // namespace sra
