// k7 — cross-layer-norm clipping aggregators (the stateful inline aggregators
// of src/simulate.py):
//
//   iclr2022_bucketing (simulate.py:335-366): overlapping windows
//     choices[b : b + perround//buckets] -> per-window mean (np.average, i.e. a
//     sequential sum over the window's rows / count), then every window mean is
//     clipped against the previous aggregate by its norm ACROSS ALL LAYERS,
//     then the mean over windows;
//   icml2021_history (simulate.py:367-388): every client row is clipped against
//     the previous aggregate the same way (and written back: the reference
//     mutates local_grads), then the mean over clients.
//
// Kernels (all HBM-bound streaming passes, one coordinate per lane):
//   window_mean   rows [w*stride, min(w*stride+width, n)) -> sequential sum / count
//                 in the input precision (numpy's axis-0 add.reduce + true_divide);
//   sqdist_*      per row, per layer segment: sum_j (m_j - prev_j)^2 in fp64 with a
//                 fixed-order two-level reduction (deterministic), then
//                 sq_r = sum_l sqrt(s_rl)^2 in layer order and
//                 scale_r = min(1, tau / sqrt(sq_r)) with Python's min semantics
//                 (tau/0 = inf -> 1, NaN -> 1);
//   clipped_mean  out_j = (sum_r fl((m_rj - prev_j) * scale_r)) / k, sequential over
//                 r starting from row 0 (numpy's reduce), optional write-back of the
//                 clipped rows (fp64, the arrays the reference stores into
//                 local_grads).
// The norms use a different summation order than BLAS ddot (np.linalg.norm), so
// scale_r agrees with the reference to ~1e-15 relative; everything else is the
// reference's evaluation order.
#include "sra_common.hpp"

namespace sra {

constexpr int kClipBS = 256;
constexpr int kClipTile = kClipBS * 16;   // columns per norm tile

typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename T> struct Vec16;
template <> struct Vec16<float> { typedef f32x4 type; static constexpr int w = 4; };
template <> struct Vec16<double> { typedef f64x2 type; static constexpr int w = 2; };

// ---------------------------------------------------------------------------
// window means
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(kClipBS) window_mean_vec_kernel(const T* __restrict__ X, int n, int64_t dv,
                                                                 int64_t ldx, int stride, int width,
                                                                 T* __restrict__ out, int64_t ldo) {
  typedef typename Vec16<T>::type VT;
  constexpr int W = Vec16<T>::w;
  const int64_t q = static_cast<int64_t>(blockIdx.x) * kClipBS + threadIdx.x;
  if (q >= dv) return;
  const int w = blockIdx.y;
  const int lo = w * stride;
  const int hi = lo + width < n ? lo + width : n;
  const VT* p = reinterpret_cast<const VT*>(X) + q;
  const int64_t ldv = ldx / W;
  VT acc = {};
  if (hi > lo) {
    acc = __builtin_nontemporal_load(p + static_cast<int64_t>(lo) * ldv);
    for (int i = lo + 1; i < hi; ++i) acc += __builtin_nontemporal_load(p + static_cast<int64_t>(i) * ldv);
  }
  reinterpret_cast<VT*>(out + static_cast<int64_t>(w) * ldo)[q] = acc / static_cast<T>(hi - lo);
}

template <typename T>
__global__ void __launch_bounds__(kClipBS) window_mean_kernel(const T* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                             int stride, int width, T* __restrict__ out,
                                                             int64_t ldo) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kClipBS + threadIdx.x;
  if (j >= d) return;
  const int w = blockIdx.y;
  const int lo = w * stride;
  const int hi = lo + width < n ? lo + width : n;
  T acc = 0;
  if (hi > lo) {
    acc = X[static_cast<int64_t>(lo) * ldx + j];
    for (int i = lo + 1; i < hi; ++i) acc += X[static_cast<int64_t>(i) * ldx + j];
  }
  out[static_cast<int64_t>(w) * ldo + j] = acc / static_cast<T>(hi - lo);
}

template <typename T>
static int launch_window_mean(const T* X, int64_t n, int64_t d, int64_t ldx, int32_t stride, int32_t width,
                              int32_t nwin, T* out, int64_t ldo, void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n < (1 << 30) && d >= 1 && ldx >= d && ldo >= d, SRA_ERR_SHAPE, "bad shape");
  SRA_REQUIRE(stride >= 0 && width >= 0 && nwin >= 1 && nwin <= 65535, SRA_ERR_ARG,
              "bad window parameters (stride %d, width %d, windows %d)", stride, width, nwin);
  hipStream_t s = static_cast<hipStream_t>(stream);
  constexpr int W = Vec16<T>::w;
  const bool vec = d % W == 0 && ldx % W == 0 && ldo % W == 0 && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  if (vec) {
    hipLaunchKernelGGL(window_mean_vec_kernel<T>, dim3(cdiv(d / W, kClipBS), nwin), dim3(kClipBS), 0, s, X, (int)n,
                       d / W, ldx, stride, width, out, ldo);
    return launch_status("window_mean_vec_kernel");
  }
  hipLaunchKernelGGL(window_mean_kernel<T>, dim3(cdiv(d, kClipBS), nwin), dim3(kClipBS), 0, s, X, (int)n, d, ldx,
                     stride, width, out, ldo);
  return launch_status("window_mean_kernel");
}

// ---------------------------------------------------------------------------
// clipping scales
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum_f64(double v) {
  // fixed butterfly order: the same bits on every run
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// part[r * ldp + tile0 + t] = sum over tile t of segment [c0, c0+len) of (M[r,j]-prev[j])^2
template <typename T>
__global__ void __launch_bounds__(kClipBS) sqdist_partial_kernel(const T* __restrict__ M, int64_t ldm,
                                                                const double* __restrict__ prev, int64_t c0,
                                                                int64_t len, double* __restrict__ part, int64_t ldp,
                                                                int64_t tile0) {
  __shared__ double red[kClipBS / kWave];
  const int r = blockIdx.y;
  const int64_t t = blockIdx.x;
  const int64_t lo = c0 + t * kClipTile;
  const int64_t hi = lo + kClipTile < c0 + len ? lo + kClipTile : c0 + len;
  const T* row = M + static_cast<int64_t>(r) * ldm;
  double acc = 0.0;
  for (int64_t j = lo + threadIdx.x; j < hi; j += kClipBS) {
    const double dl = static_cast<double>(row[j]) - prev[j];
    acc = __builtin_fma(dl, dl, acc);
  }
  acc = wave_sum_f64(acc);
  const int wv = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) red[wv] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = red[0];
#pragma unroll
    for (int i = 1; i < kClipBS / kWave; ++i) s += red[i];
    part[static_cast<int64_t>(r) * ldp + tile0 + t] = s;
  }
}

// segsq[r * nseg + l] = sqrt(s)^2 with s the ordered sum of segment l's tiles
// (np.linalg.norm(diff) ** 2 of simulate.py:355 / 377)
__global__ void __launch_bounds__(kWave) sqdist_segment_kernel(const double* __restrict__ part, int64_t ldp,
                                                              int64_t tile0, int64_t ntiles,
                                                              double* __restrict__ segsq, int nseg, int l) {
  const int r = blockIdx.x;
  const double* p = part + static_cast<int64_t>(r) * ldp + tile0;
  double acc = 0.0;
  for (int64_t t = threadIdx.x; t < ntiles; t += kWave) acc += p[t];
  acc = wave_sum_f64(acc);
  if (threadIdx.x == 0) {
    const double nrm = __builtin_sqrt(acc);
    segsq[static_cast<int64_t>(r) * nseg + l] = nrm * nrm;
  }
}

// scale[r] = min(1, tau / sqrt(sum_l segsq[r, l]))   (Python min(1, x): x only if x < 1)
__global__ void __launch_bounds__(kClipBS) clip_scale_kernel(const double* __restrict__ segsq, int k, int nseg,
                                                            double tau, double* __restrict__ scale,
                                                            double* __restrict__ norm_out) {
  const int r = blockIdx.x * kClipBS + threadIdx.x;
  if (r >= k) return;
  double sq = 0.0;
  for (int l = 0; l < nseg; ++l) sq += segsq[static_cast<int64_t>(r) * nseg + l];
  const double nrm = __builtin_sqrt(sq);
  const double x = tau / nrm;
  scale[r] = x < 1.0 ? x : 1.0;
  if (norm_out != nullptr) norm_out[r] = nrm;
}

// DBA Helper.history / bucketing (src/DBA/helper.py:753-759, 803-809): the
// running value is re-rooted after every layer, norm_l = sqrt(norm_{l-1} +
// ||layer_l||^2) -- not the L2 norm across layers; scale = min(1, tau / norm_L).
__global__ void __launch_bounds__(kClipBS) clip_scale_running_kernel(const double* __restrict__ segsq, int k,
                                                                    int nseg, double tau,
                                                                    double* __restrict__ scale,
                                                                    double* __restrict__ norm_out) {
  const int r = blockIdx.x * kClipBS + threadIdx.x;
  if (r >= k) return;
  double nrm = 0.0;
  for (int l = 0; l < nseg; ++l) nrm = __builtin_sqrt(nrm + segsq[static_cast<int64_t>(r) * nseg + l]);
  const double x = tau / nrm;
  scale[r] = x < 1.0 ? x : 1.0;
  if (norm_out != nullptr) norm_out[r] = nrm;
}

// ---------------------------------------------------------------------------
// clipped mean
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(kClipBS) clipped_mean_kernel(const T* __restrict__ M, int k, int64_t d,
                                                              int64_t ldm, const double* __restrict__ prev,
                                                              const double* __restrict__ scale,
                                                              double* __restrict__ clipped, int64_t ldc,
                                                              double* __restrict__ out) {
  // two coordinates per lane (16-byte fp64 stores / prev loads)
  const int64_t j0 = (static_cast<int64_t>(blockIdx.x) * kClipBS + threadIdx.x) * 2;
  if (j0 >= d) return;
  const bool two = j0 + 1 < d;
  const double p0 = prev[j0];
  const double p1 = two ? prev[j0 + 1] : 0.0;
  double a0 = 0.0, a1 = 0.0;
  for (int r = 0; r < k; ++r) {
    const double s = scale[r];
    const T* row = M + static_cast<int64_t>(r) * ldm + j0;
    const double v0 = (static_cast<double>(__builtin_nontemporal_load(row)) - p0) * s;
    const double v1 = two ? (static_cast<double>(__builtin_nontemporal_load(row + 1)) - p1) * s : 0.0;
    if (clipped != nullptr) {
      double* c = clipped + static_cast<int64_t>(r) * ldc + j0;
      c[0] = v0;
      if (two) c[1] = v1;
    }
    if (r == 0) { a0 = v0; a1 = v1; } else { a0 += v0; a1 += v1; }
  }
  out[j0] = a0 / static_cast<double>(k);
  if (two) out[j0 + 1] = a1 / static_cast<double>(k);
}

static int64_t seg_tiles(const int64_t* seg, int32_t nseg) {
  int64_t t = 0;
  for (int l = 0; l < nseg; ++l) t += cdiv(seg[l + 1] - seg[l], kClipTile);
  return t;
}

template <typename T, bool RUNNING = false>
static int launch_clip_scale(const T* M, int64_t k, int64_t d, int64_t ldm, const double* prev, const int64_t* seg,
                             int32_t nseg, double tau, double* scale, double* norm_out, void* ws, size_t ws_bytes,
                             void* stream) {
  SRA_REQUIRE(M != nullptr && prev != nullptr && seg != nullptr && scale != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(k >= 1 && k <= 65535 && d >= 1 && ldm >= d, SRA_ERR_SHAPE, "bad shape (k=%lld d=%lld)", (long long)k,
              (long long)d);
  SRA_REQUIRE(nseg >= 1 && seg[0] == 0 && seg[nseg] == d, SRA_ERR_SHAPE,
              "segment table must run from 0 to d (%lld) in %d segments", (long long)d, nseg);
  for (int l = 0; l < nseg; ++l)
    SRA_REQUIRE(seg[l + 1] >= seg[l], SRA_ERR_SHAPE, "segment %d has negative length", l);
  const int64_t ntiles = seg_tiles(seg, nseg);
  const size_t need = sizeof(double) * (static_cast<size_t>(k) * (ntiles + nseg));
  SRA_REQUIRE(ws != nullptr && ws_bytes >= need, SRA_ERR_WORKSPACE, "workspace %zu < %zu bytes", ws_bytes, need);
  double* part = static_cast<double*>(ws);
  double* segsq = part + static_cast<size_t>(k) * ntiles;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int64_t tile0 = 0;
  for (int l = 0; l < nseg; ++l) {
    const int64_t len = seg[l + 1] - seg[l];
    const int64_t nt = cdiv(len, kClipTile);
    if (nt > 0) {
      SRA_REQUIRE(nt <= (int64_t(1) << 31) - 1, SRA_ERR_SHAPE, "segment %d too long", l);
      hipLaunchKernelGGL(sqdist_partial_kernel<T>, dim3(nt, k), dim3(kClipBS), 0, s, M, ldm, prev, seg[l], len,
                         part, ntiles, tile0);
      int rc = launch_status("sqdist_partial_kernel");
      if (rc) return rc;
    }
    hipLaunchKernelGGL(sqdist_segment_kernel, dim3(k), dim3(kWave), 0, s, part, ntiles, tile0, nt, segsq, nseg, l);
    int rc = launch_status("sqdist_segment_kernel");
    if (rc) return rc;
    tile0 += nt;
  }
  if constexpr (RUNNING) {
    hipLaunchKernelGGL(clip_scale_running_kernel, dim3(cdiv(k, kClipBS)), dim3(kClipBS), 0, s, segsq, (int)k, nseg,
                       tau, scale, norm_out);
    return launch_status("clip_scale_running_kernel");
  }
  hipLaunchKernelGGL(clip_scale_kernel, dim3(cdiv(k, kClipBS)), dim3(kClipBS), 0, s, segsq, (int)k, nseg, tau, scale,
                     norm_out);
  return launch_status("clip_scale_kernel");
}

template <typename T>
static int launch_clipped_mean(const T* M, int64_t k, int64_t d, int64_t ldm, const double* prev, const double* scale,
                               double* clipped, int64_t ldc, double* out, void* stream) {
  SRA_REQUIRE(M != nullptr && prev != nullptr && scale != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(k >= 1 && d >= 1 && ldm >= d && (clipped == nullptr || ldc >= d), SRA_ERR_SHAPE, "bad shape");
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(clipped_mean_kernel<T>, dim3(cdiv(cdiv(d, 2), kClipBS)), dim3(kClipBS), 0, s, M, (int)k, d, ldm,
                     prev, scale, clipped, ldc, out);
  return launch_status("clipped_mean_kernel");
}

}  // namespace sra

using namespace sra;

extern "C" int sra_window_mean_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t stride, int32_t width,
                                   int32_t nwin, float* out, int64_t ldo, void* stream) {
  return launch_window_mean<float>(X, n, d, ldx, stride, width, nwin, out, ldo, stream);
}

extern "C" int sra_window_mean_f64(const double* X, int64_t n, int64_t d, int64_t ldx, int32_t stride, int32_t width,
                                   int32_t nwin, double* out, int64_t ldo, void* stream) {
  return launch_window_mean<double>(X, n, d, ldx, stride, width, nwin, out, ldo, stream);
}

extern "C" int sra_clip_workspace_bytes(int64_t k, const int64_t* seg, int32_t nseg, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr && seg != nullptr && k >= 1 && nseg >= 1, SRA_ERR_ARG, "bad arguments");
  *bytes = sizeof(double) * static_cast<size_t>(k) * (seg_tiles(seg, nseg) + nseg);
  return SRA_OK;
}

extern "C" int sra_clip_scale_f32(const float* M, int64_t k, int64_t d, int64_t ldm, const double* prev,
                                  const int64_t* seg, int32_t nseg, double tau, double* scale, double* norm,
                                  void* ws, size_t ws_bytes, void* stream) {
  return launch_clip_scale<float>(M, k, d, ldm, prev, seg, nseg, tau, scale, norm, ws, ws_bytes, stream);
}

extern "C" int sra_clip_scale_f64(const double* M, int64_t k, int64_t d, int64_t ldm, const double* prev,
                                  const int64_t* seg, int32_t nseg, double tau, double* scale, double* norm,
                                  void* ws, size_t ws_bytes, void* stream) {
  return launch_clip_scale<double>(M, k, d, ldm, prev, seg, nseg, tau, scale, norm, ws, ws_bytes, stream);
}

extern "C" int sra_clipped_mean_f32(const float* M, int64_t k, int64_t d, int64_t ldm, const double* prev,
                                    const double* scale, double* clipped, int64_t ldc, double* out, void* stream) {
  return launch_clipped_mean<float>(M, k, d, ldm, prev, scale, clipped, ldc, out, stream);
}

extern "C" int sra_clipped_mean_f64(const double* M, int64_t k, int64_t d, int64_t ldm, const double* prev,
                                    const double* scale, double* clipped, int64_t ldc, double* out, void* stream) {
  return launch_clipped_mean<double>(M, k, d, ldm, prev, scale, clipped, ldc, out, stream);
}

extern "C" int sra_clip_scale_running_f32(const float* M, int64_t k, int64_t d, int64_t ldm, const double* prev,
                                          const int64_t* seg, int32_t nseg, double tau, double* scale, double* norm,
                                          void* ws, size_t ws_bytes, void* stream) {
  return launch_clip_scale<float, true>(M, k, d, ldm, prev, seg, nseg, tau, scale, norm, ws, ws_bytes, stream);
}
