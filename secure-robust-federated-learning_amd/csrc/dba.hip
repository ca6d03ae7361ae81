// k10 -- streaming row reductions with the DBA harness's exact fp32 rounding
// (src/DBA/helper.py).
//
// Both kernels are HBM-bound column sweeps over an n x d row-major matrix: one
// lane owns 4 consecutive coordinates (16-byte loads, a wave reads 1 KiB of a
// row per instruction) and walks down the rows in order, so the fp32 rounding
// sequence is exactly torch's in-place accumulation:
//
//   sra_rows_sum_div_f32  out = (((0 + x_r0) + x_r0+1) + ...) / divisor
//       Helper.mom_krum's bucket (zero_, +=, /= (count + 1), :859-863) and
//       Helper.sharding's shard average (copy, +=, /= count, :1157-1163).
//   sra_weighted_sum_f32  out = ((0 + w_0*x_0) + w_1*x_1) + ...   (w on device)
//       Helper.weighted_average_oracle (:1199-1221): temp = w * p, data.add_(temp),
//       two roundings per row -- never contracted into an FMA.
//
// Algorithmic bytes: 4 * rows * d read + 4d written.
#include "sra_common.hpp"

namespace sra {

constexpr int kDbaBS = 256;

// w * x rounded on its own: the empty asm makes the product opaque, so the
// backend cannot fuse it with the following add into an FMA (torch rounds twice)
__device__ __forceinline__ float mul_rn(float a, float b) {
  float p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}

__device__ __forceinline__ f32x4 ld4(const float* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
}

template <bool WEIGHTED>
__global__ void __launch_bounds__(kDbaBS) rows_vec4_kernel(const float* __restrict__ X, int64_t ldx, int rows,
                                                           int64_t d4, const float* __restrict__ w, float divisor,
                                                           float* __restrict__ out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kDbaBS + threadIdx.x;
  if (j >= d4) return;
  const float* p = X + 4 * j;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < rows; ++r) {
    const f32x4 x = ld4(p);
    if constexpr (WEIGHTED) {
      const float c = w[r];
      a.x = __fadd_rn(a.x, mul_rn(c, x.x));
      a.y = __fadd_rn(a.y, mul_rn(c, x.y));
      a.z = __fadd_rn(a.z, mul_rn(c, x.z));
      a.w = __fadd_rn(a.w, mul_rn(c, x.w));
    } else {
      a.x = __fadd_rn(a.x, x.x);
      a.y = __fadd_rn(a.y, x.y);
      a.z = __fadd_rn(a.z, x.z);
      a.w = __fadd_rn(a.w, x.w);
    }
    p += ldx;
  }
  if constexpr (!WEIGHTED) {
    a.x = __fdiv_rn(a.x, divisor);
    a.y = __fdiv_rn(a.y, divisor);
    a.z = __fdiv_rn(a.z, divisor);
    a.w = __fdiv_rn(a.w, divisor);
  }
  reinterpret_cast<f32x4*>(out)[j] = a;
}

template <bool WEIGHTED>
__global__ void __launch_bounds__(kDbaBS) rows_kernel(const float* __restrict__ X, int64_t ldx, int rows, int64_t d,
                                                      const float* __restrict__ w, float divisor,
                                                      float* __restrict__ out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kDbaBS + threadIdx.x;
  if (j >= d) return;
  const float* p = X + j;
  float a = 0.f;
  for (int r = 0; r < rows; ++r) {
    const float x = __builtin_nontemporal_load(p);
    a = WEIGHTED ? __fadd_rn(a, mul_rn(w[r], x)) : __fadd_rn(a, x);
    p += ldx;
  }
  out[j] = WEIGHTED ? a : __fdiv_rn(a, divisor);
}

template <bool WEIGHTED>
static int launch_rows(const float* X, int64_t rows, int64_t d, int64_t ldx, const float* w, float divisor, float* out,
                       void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr && (!WEIGHTED || w != nullptr), SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(rows >= 0 && rows <= (int64_t(1) << 30) && d >= 1 && ldx >= d, SRA_ERR_SHAPE,
              "bad shape (rows=%lld d=%lld ldx=%lld)", (long long)rows, (long long)d, (long long)ldx);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = (reinterpret_cast<uintptr_t>(X) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                   ldx % 4 == 0 && d % 4 == 0;
  if (vec) {
    const int64_t d4 = d / 4;
    hipLaunchKernelGGL(rows_vec4_kernel<WEIGHTED>, dim3(cdiv(d4, kDbaBS)), dim3(kDbaBS), 0, s, X, ldx, (int)rows, d4,
                       w, divisor, out);
    return launch_status("rows_vec4_kernel");
  }
  hipLaunchKernelGGL(rows_kernel<WEIGHTED>, dim3(cdiv(d, kDbaBS)), dim3(kDbaBS), 0, s, X, ldx, (int)rows, d, w, divisor,
                     out);
  return launch_status("rows_kernel");
}

}  // namespace sra

using namespace sra;

extern "C" int sra_rows_sum_div_f32(const float* X, int64_t rows, int64_t d, int64_t ldx, float divisor, float* out,
                                    void* stream) {
  return launch_rows<false>(X, rows, d, ldx, nullptr, divisor, out, stream);
}

extern "C" int sra_weighted_sum_f32(const float* X, int64_t rows, int64_t d, int64_t ldx, const float* w, float* out,
                                    void* stream) {
  return launch_rows<true>(X, rows, d, ldx, w, 1.0f, out, stream);
}
