// k9 — the device-resident client-update store: the step either side of the
// aggregation path.
//
// In the reference every chosen client trains on the device, then its update
// crosses PCIe one layer at a time (simulate.py:190-194:
// `params_copy[idx].data.cpu().numpy() - p.data.cpu().numpy()`), lives in a
// host list `local_grads[c][idx]`, is stacked again per layer for the
// aggregator, and the aggregate crosses back (simulate.py:400-404:
// `p.data.sub_(torch.from_numpy(avg).to(device))`).  Here the updates never
// leave HBM: a parameter table (one device pointer per parameter tensor plus
// the flat segment offsets) lets ONE launch walk the whole network:
//
//   params_flatten   flat = concat(params)                 (params_copy, :146-148)
//   record_delta     row = snapshot - params  (fp32, exactly numpy's f32 minus)
//                    and params = snapshot                  (:190-199, fused restore)
//   record_momentum  row = (f64) fl32(omb * fl32(snapshot - params)) + beta * row
//                    (:187-189, numpy's promotion of float32 * python float,
//                    then float32 + float64), params = snapshot
//   apply_update     params -= agg; an fp64 aggregate is subtracted in fp64 and
//                    rounded once to fp32 (torch's in-place sub_ of a float32
//                    tensor by a float64 one computes in the promoted type)
//
// All four are HBM-bound streams: 4-byte coalesced accesses, grid-stride over
// the flat index space, segment found by a short binary search over the
// (L1/scalar-cached) offset table.  Algorithmic bytes per element: flatten 8,
// record 16 (f32 row) / 24 (f64 row, read+write), apply 12 (f32 agg) / 16 (f64).
#include "sra_common.hpp"

namespace sra {

constexpr int kStoreBS = 256;
constexpr int kStorePerThread = 4;

__device__ __forceinline__ int seg_of(const int64_t* __restrict__ seg, int nseg, int64_t j) {
  int lo = 0, hi = nseg - 1;           // largest k with seg[k] <= j
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (seg[mid] <= j) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Visit every flat index j in [0, D) as (param tensor k, offset j - seg[k]).
template <typename F>
__device__ __forceinline__ void for_each_flat(const int64_t* __restrict__ seg, int nseg, int64_t D, F&& f) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kStoreBS;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kStoreBS * kStorePerThread + threadIdx.x; base < D;
       base += stride * kStorePerThread) {
#pragma unroll
    for (int u = 0; u < kStorePerThread; ++u) {
      const int64_t j = base + static_cast<int64_t>(u) * kStoreBS;
      if (j < D) {
        const int k = seg_of(seg, nseg, j);
        f(k, j, j - seg[k]);
      }
    }
  }
}

__global__ void __launch_bounds__(kStoreBS) flatten_kernel(const uint64_t* __restrict__ ptrs,
                                                           const int64_t* __restrict__ seg, int nseg, int64_t D,
                                                           float* __restrict__ flat) {
  for_each_flat(seg, nseg, D, [&](int k, int64_t j, int64_t o) {
    flat[j] = reinterpret_cast<const float*>(ptrs[k])[o];
  });
}

__global__ void __launch_bounds__(kStoreBS) record_delta_kernel(const uint64_t* __restrict__ ptrs,
                                                                const int64_t* __restrict__ seg, int nseg, int64_t D,
                                                                const float* __restrict__ snap,
                                                                float* __restrict__ row) {
  for_each_flat(seg, nseg, D, [&](int k, int64_t j, int64_t o) {
    float* p = reinterpret_cast<float*>(ptrs[k]) + o;
    const float s = snap[j];
    row[j] = s - *p;
    *p = s;
  });
}

__global__ void __launch_bounds__(kStoreBS) record_momentum_kernel(const uint64_t* __restrict__ ptrs,
                                                                   const int64_t* __restrict__ seg, int nseg,
                                                                   int64_t D, const float* __restrict__ snap,
                                                                   float omb, double beta,
                                                                   double* __restrict__ row) {
  for_each_flat(seg, nseg, D, [&](int k, int64_t j, int64_t o) {
#pragma clang fp contract(off)   // numpy rounds every product and sum separately
    float* p = reinterpret_cast<float*>(ptrs[k]) + o;
    const float s = snap[j];
    const float delta = omb * (s - *p);                 // float32 * float32
    const double keep = beta * row[j];
    row[j] = static_cast<double>(delta) + keep;
    *p = s;
  });
}

template <typename T>
__global__ void __launch_bounds__(kStoreBS) apply_update_kernel(const uint64_t* __restrict__ ptrs,
                                                                const int64_t* __restrict__ seg, int nseg, int64_t D,
                                                                const T* __restrict__ agg) {
  for_each_flat(seg, nseg, D, [&](int k, int64_t j, int64_t o) {
#pragma clang fp contract(off)
    float* p = reinterpret_cast<float*>(ptrs[k]) + o;
    if constexpr (sizeof(T) == 8) {
      *p = static_cast<float>(static_cast<double>(*p) - agg[j]);
    } else {
      *p = *p - agg[j];
    }
  });
}

static int grid_for(int64_t D) {
  const int64_t per_block = static_cast<int64_t>(kStoreBS) * kStorePerThread;
  const int64_t want = cdiv(D, per_block);
  return static_cast<int>(want < 256 * 32 ? want : 256 * 32);   // >= 1; grid-stride beyond 32 blocks/CU
}

static int check_table(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D) {
  SRA_REQUIRE(ptrs != nullptr && seg != nullptr, SRA_ERR_ARG, "parameter table pointers must be non-null");
  SRA_REQUIRE(nseg >= 1 && nseg <= 65536, SRA_ERR_ARG, "nseg must be in [1, 65536], got %d", nseg);
  SRA_REQUIRE(D >= 1, SRA_ERR_SHAPE, "D must be >= 1, got %lld", static_cast<long long>(D));
  return SRA_OK;
}

}  // namespace sra

using namespace sra;

extern "C" int sra_params_flatten_f32(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D,
                                      float* flat, void* stream) {
  if (int rc = check_table(ptrs, seg, nseg, D)) return rc;
  SRA_REQUIRE(flat != nullptr, SRA_ERR_ARG, "flat must be non-null");
  hipLaunchKernelGGL(flatten_kernel, dim3(grid_for(D)), dim3(kStoreBS), 0, static_cast<hipStream_t>(stream), ptrs,
                     seg, nseg, D, flat);
  return launch_status("flatten_kernel");
}

extern "C" int sra_record_delta_f32(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D,
                                    const float* snapshot, float* row, void* stream) {
  if (int rc = check_table(ptrs, seg, nseg, D)) return rc;
  SRA_REQUIRE(snapshot != nullptr && row != nullptr, SRA_ERR_ARG, "snapshot and row must be non-null");
  hipLaunchKernelGGL(record_delta_kernel, dim3(grid_for(D)), dim3(kStoreBS), 0, static_cast<hipStream_t>(stream),
                     ptrs, seg, nseg, D, snapshot, row);
  return launch_status("record_delta_kernel");
}

extern "C" int sra_record_momentum_f64(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D,
                                       const float* snapshot, float one_minus_beta, double beta, double* row,
                                       void* stream) {
  if (int rc = check_table(ptrs, seg, nseg, D)) return rc;
  SRA_REQUIRE(snapshot != nullptr && row != nullptr, SRA_ERR_ARG, "snapshot and row must be non-null");
  hipLaunchKernelGGL(record_momentum_kernel, dim3(grid_for(D)), dim3(kStoreBS), 0, static_cast<hipStream_t>(stream),
                     ptrs, seg, nseg, D, snapshot, one_minus_beta, beta, row);
  return launch_status("record_momentum_kernel");
}

extern "C" int sra_apply_update_f32(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D,
                                    const float* agg, void* stream) {
  if (int rc = check_table(ptrs, seg, nseg, D)) return rc;
  SRA_REQUIRE(agg != nullptr, SRA_ERR_ARG, "agg must be non-null");
  hipLaunchKernelGGL(apply_update_kernel<float>, dim3(grid_for(D)), dim3(kStoreBS), 0,
                     static_cast<hipStream_t>(stream), ptrs, seg, nseg, D, agg);
  return launch_status("apply_update_kernel<float>");
}

extern "C" int sra_apply_update_f64(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D,
                                    const double* agg, void* stream) {
  if (int rc = check_table(ptrs, seg, nseg, D)) return rc;
  SRA_REQUIRE(agg != nullptr, SRA_ERR_ARG, "agg must be non-null");
  hipLaunchKernelGGL(apply_update_kernel<double>, dim3(grid_for(D)), dim3(kStoreBS), 0,
                     static_cast<hipStream_t>(stream), ptrs, seg, nseg, D, agg);
  return launch_status("apply_update_kernel<double>");
}
