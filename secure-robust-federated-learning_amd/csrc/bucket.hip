// k5 — bucket means for the median-of-means wrappers.
//
// Replaces the bucketing of mom_krum (src/robust_estimator.py:251-256),
// mom_filterL2 (:210-216) and mom_ex_noregret (:135-140): bucket b is the
// np.mean over clients [b*size, min((b+1)*size, N)) in list order -- a
// sequential fp32 sum over the bucket's rows divided by its row count, bit
// for bit.  An empty bucket (the reference's NaN scalar that np.array then
// rejects) is reported as SRA_ERR_EMPTY_BUCKET before anything is launched.
//
// HBM-bound: 4*N*d read + 4*B*d written; one float4 column per lane.
#include "sra_common.hpp"

namespace sra {

__global__ void __launch_bounds__(256) bucket_mean_vec4_kernel(const float* __restrict__ X, int n, int64_t d4,
                                                              int64_t ldx, int bsize, float* __restrict__ out,
                                                              int64_t ldo) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (q >= d4) return;
  const int lo = b * bsize;
  const int hi = lo + bsize < n ? lo + bsize : n;
  const f32x4* p = reinterpret_cast<const f32x4*>(X) + q;
  const int64_t ld4 = ldx / 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = lo; i < hi; ++i) acc += __builtin_nontemporal_load(p + static_cast<int64_t>(i) * ld4);
  reinterpret_cast<f32x4*>(out + b * ldo)[q] = acc / static_cast<float>(hi - lo);
}

__global__ void __launch_bounds__(256) bucket_mean_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                         int bsize, float* __restrict__ out, int64_t ldo) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (j >= d) return;
  const int lo = b * bsize;
  const int hi = lo + bsize < n ? lo + bsize : n;
  float acc = 0.f;
  for (int i = lo; i < hi; ++i) acc += X[static_cast<int64_t>(i) * ldx + j];
  out[b * ldo + j] = acc / static_cast<float>(hi - lo);
}

}  // namespace sra

using namespace sra;

extern "C" int sra_bucket_mean_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t bucket_size,
                                   int32_t nbuckets, float* out, int64_t ldo, void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && d >= 1 && ldx >= d && ldo >= d, SRA_ERR_SHAPE, "bad shape");
  SRA_REQUIRE(bucket_size >= 1 && nbuckets >= 1 && nbuckets <= 65535, SRA_ERR_ARG, "bad bucket parameters");
  SRA_REQUIRE(static_cast<int64_t>(nbuckets - 1) * bucket_size < n, SRA_ERR_EMPTY_BUCKET,
              "bucket %d of size %d is empty for N=%lld (the reference's np.mean of an empty slice)",
              (int)((n + bucket_size - 1) / bucket_size), bucket_size, (long long)n);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = d % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  if (vec) {
    hipLaunchKernelGGL(bucket_mean_vec4_kernel, dim3(cdiv(d / 4, 256), nbuckets), dim3(256), 0, s, X, (int)n, d / 4,
                       ldx, bucket_size, out, ldo);
    return launch_status("bucket_mean_vec4_kernel");
  }
  hipLaunchKernelGGL(bucket_mean_kernel, dim3(cdiv(d, 256), nbuckets), dim3(256), 0, s, X, (int)n, d, ldx,
                     bucket_size, out, ldo);
  return launch_status("bucket_mean_kernel");
}
