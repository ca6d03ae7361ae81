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
// Roofline: HBM-bound, 4*N*d + 4*d bytes per call.  At N=128 the network is
// ~1.5k compare-exchanges per coordinate (~3k VALU lane-ops), below the
// ~6.7k lane-ops per coordinate the VALU affords at 6 TB/s.
//
// N > 128 (e.g. the N=512 MoM/8-GPU config) uses an LDS bitonic path.
#include "sra_common.hpp"

namespace sra {

enum SelectMode { kMedian = 0, kTrimmed = 1 };

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

template <int P, int MODE>
__global__ void __launch_bounds__(256) select_reg_kernel(const float* __restrict__ X, int n, int64_t d,
                                                        int64_t ldx, int lo, int hi, float* __restrict__ out) {
  constexpr int P2 = next_pow2(P);
  constexpr int kFirstPad = (P > 16) ? P - 16 : 0;  // rows below this are always real
  const int64_t base = static_cast<int64_t>(blockIdx.x) * blockDim.x;
  const int64_t rem = d - base;                    // > 0
  const unsigned t = threadIdx.x;
  const unsigned last = rem < 256 ? static_cast<unsigned>(rem - 1) : 255u;
  const unsigned off = (t < last ? t : last) * 4u;  // byte offset of this lane (tail lanes clamped)
  const char* xb = reinterpret_cast<const char*>(X + base);
  const int64_t ldb = ldx * 4;
  const int k_bottom = (MODE == kMedian) ? (P - n) / 2 : 0;  // -inf pads for the median
  float v[P2];
#pragma unroll
  for (int i = 0; i < kFirstPad; ++i) v[i] = ldrow(xb + i * ldb, off);
#pragma unroll
  for (int i = kFirstPad; i < P; ++i) {
    const int r = i < n ? i : n - 1;
    const float x = ldrow(xb + r * ldb, off);
    const float pad = (i - n < k_bottom) ? -__builtin_inff() : qnan();
    v[i] = i < n ? x : pad;
  }

  float res;
  if constexpr (MODE == kMedian) {
    float m = v[0];
#pragma unroll
    for (int i = 1; i < P; ++i) m = __builtin_elementwise_maximum(m, v[i]);  // NaN-propagating
    sort_network<P2, P, P / 2 - 1, P / 2 + 1>(v);
    res = (n & 1) ? v[P / 2 - 1] : (v[P / 2 - 1] + v[P / 2]) * 0.5f;
    if (__builtin_isnan(m)) res = qnan();
  } else {
    sort_network<P2, P, 0, P>(v);
    // sequential ascending-order sum of s[lo .. hi), numpy's axis-0 reduce;
    // out-of-range positions contribute +0 (acc + 0 == acc), so the order of
    // the kept terms is exactly numpy's
    // (the empty volatile asm keeps each predicate a wave-uniform scalar
    // branch instead of 128 hoisted SGPR-pair masks that spill)
    float acc = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if (p >= lo && p < hi) {
        asm volatile("");
        acc += v[p];
      }
    }
    res = acc / static_cast<float>(hi - lo);
  }
  if (t < rem) out[base + t] = res;
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
  // load: row-major sweep, consecutive lanes -> consecutive coordinates
  for (int e = tid; e < pn * tile; e += blockDim.x) {
    const int r = e / tile, c = e - r * tile;
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
        const int c = q % tile;
        const int h = q / tile;                            // pair index within the column
        const int i = ((h / s) * (2 * s)) + (h % s);       // lower element of the pair
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

template <int MODE>
static int launch_select(const float* X, int n, int64_t d, int64_t ldx, int lo, int hi, float* out,
                         hipStream_t s) {
  const int64_t blocks = cdiv(d, 256);
  const int P = static_cast<int>(cdiv(n, 16) * 16);
#define SRA_SEL_CASE(PP)                                                                              \
  case PP:                                                                                            \
    hipLaunchKernelGGL((select_reg_kernel<PP, MODE>), dim3(blocks), dim3(256), 0, s, X, n, d, ldx, lo, \
                       hi, out);                                                                      \
    return launch_status("select_reg_kernel");
  if (n <= 128) {
    switch (P) {
      SRA_SEL_CASE(16)
      SRA_SEL_CASE(32)
      SRA_SEL_CASE(48)
      SRA_SEL_CASE(64)
      SRA_SEL_CASE(80)
      SRA_SEL_CASE(96)
      SRA_SEL_CASE(112)
      SRA_SEL_CASE(128)
      default: break;
    }
  }
#undef SRA_SEL_CASE
  const int pn = next_pow2(n);
  SRA_REQUIRE(pn <= kLdsFloats / 4, SRA_ERR_UNSUPPORTED, "k-select supports N <= %d (got %d)", kLdsFloats / 4, n);
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
