// Shared by gram.hip and gram_pipe.hip (k2, the bf16x3 Gram): fragment types,
// the tile configuration, the packed three-way split, compile-time loops.
#pragma once
#include "sra_common.hpp"

namespace sra {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int NB, int WAVES = 4, int STG = 0>
struct GramCfg {
  static constexpr int NP = 32 * NB;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int STAGE = STG ? STG : (NB <= 4 ? 128 : 64);  // coordinates per stage
  static constexpr int ROWPAD = STAGE + 4;                       // LDS row stride (floats)
  static constexpr int T = NB * (NB + 1) / 2;                    // upper-triangle tiles
  // tile groups: 4 waves -> keep <= 176 accumulators per wave; 8 waves (two
  // per SIMD) -> <= 128 so that a wave fits in 256 registers
  static constexpr int WT = WAVES == 4 ? (NB <= 4 ? 1 : (NB <= 6 ? 2 : 4))
                                       : (NB <= 3 ? 1 : (NB <= 5 ? 2 : (NB <= 7 ? 4 : 8)));
  static constexpr int WK = WAVES / WT;                          // k groups
  static constexpr int TPW = (T + WT - 1) / WT;                  // tiles per wave (max)
  static constexpr int KSTEPS = STAGE / 16;                      // 16-coordinate k-steps per stage
  static constexpr int KPW = KSTEPS / WK;                        // k-steps per wave per stage
  static constexpr int C4 = STAGE / 4;                           // float4 columns per row
  static constexpr int RSTEP = THREADS / C4;                     // rows covered per load sweep
  static constexpr int LOADS = NP / RSTEP > 0 ? NP / RSTEP : 1;  // float4 per thread per stage
  static constexpr int kTileI(int t) {
    int c = 0;
    for (int i = 0; i < NB; ++i)
      for (int j = i; j < NB; ++j) {
        if (c == t) return i;
        ++c;
      }
    return 0;
  }
  static constexpr int kTileJ(int t) {
    int c = 0;
    for (int i = 0; i < NB; ++i)
      for (int j = i; j < NB; ++j) {
        if (c == t) return j;
        ++c;
      }
    return 0;
  }
  static constexpr int BUF = NP * ROWPAD;                        // floats per stage buffer
  static constexpr int PART = WAVES * STAGE;                     // per-wave column partials
  static constexpr int lds_floats = 2 * BUF + PART + 2 * STAGE;  // stage buffers, partials, means
};

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// the exact three-way split of two values, packed: one v_cvt_pk_bf16_f32 per
// level, the bf16 -> fp32 widening by shift / mask (the same bits as split3)
__device__ __forceinline__ void split3_pair(float x0, float x1, uint32_t& hb, uint32_t& mb, uint32_t& lb) {
  hb = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x0, x1}, bf16x2));
  const float r0 = x0 - __builtin_bit_cast(float, hb << 16);
  const float r1 = x1 - __builtin_bit_cast(float, hb & 0xffff0000u);
  mb = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){r0, r1}, bf16x2));
  const float q0 = r0 - __builtin_bit_cast(float, mb << 16);
  const float q1 = r1 - __builtin_bit_cast(float, mb & 0xffff0000u);
  lb = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){q0, q1}, bf16x2));
}

__device__ __forceinline__ void set_pair(bf16x8& v, int e2, uint32_t bits) {
  u32x4 u = __builtin_bit_cast(u32x4, v);
  u[e2] = bits;
  v = __builtin_bit_cast(bf16x8, u);
}

template <int V>
struct IC {
  static constexpr int value = V;
};

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<I + 1, N>(f);
  }
}

// gram_pipe.hip: the software-pipelined N = 128 Gram.  Every row is addressed
// by a 32-bit byte offset from one SGPR base (rows 0..7 of a load group, plus a
// 128-coordinate stage), so the pipe kernel is taken only when those offsets fit.
__host__ __device__ constexpr bool gram_pipe_offsets_fit(int64_t ldx) {
  return ldx >= 0 && 7 * ldx * 4 + 4 * 128 < (int64_t(1) << 31);
}
int launch_gram_pipe(const float* X, int n, int64_t d, int64_t ldx, float* slab, int nwg, hipStream_t s);

// gram_bucket.hip: the Gram of the means of consecutive client buckets of size
// bs (mom_krum), the bucket matrix never written; nb = ceil(n / bs) buckets.
constexpr int kBucketGramMaxNB = 6;   // at most 192 buckets
int launch_gram_bucket_partial(const float* X, int n, int nb, int bs, int64_t d, int64_t ldx, float* slab, int nwg,
                               hipStream_t s);

}  // namespace sra
