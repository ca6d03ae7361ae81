// k2 — centred pairwise Gram matrix G = Xc Xc^T (N x N, fp64 result) on the
// fp32 MFMA (v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulate).
//
// Feeds every pairwise-L2 consumer of the reference:
//   krum_ / krum / mom_krum  (src/robust_estimator.py:234-257)
//   bulyan(aggsubfunc='krum') (src/robust_estimator.py:286-296)
// through ||x_i - x_j||^2 = G_ii + G_jj - 2 G_ij.
//
// Centring: before the MFMA every 64-coordinate stage is shifted by its
// per-coordinate client mean (distances are translation invariant), which
// removes the cancellation of the expanded form when clients share a large
// common component.  All (i, j) entries accumulate their products in the same
// k order, so two identical clients get G_ii == G_jj == G_ij bit for bit and
// distance exactly 0, as in the reference (identical rows of the `xie`
// attack, src/attack.py:362-372).
//
// Layout / schedule (one 256-thread workgroup per CU, persistent over a
// contiguous coordinate range so every row is streamed contiguously):
//   stage = NP rows x 64 coordinates, register-staged float4 loads (one stage
//   ahead) -> LDS [row][64 + 4 pad] (conflict-free ds_read_b128), double
//   buffered; per-stage column means from the staging registers.
//   wave w owns a set of upper-triangle 32x32 output tiles (I <= J) and a
//   subset of the 8-coordinate groups (K split across waves when the tile
//   count is small).  One ds_read_b128 per row block gives the A/B fragments
//   of 4 MFMA k-steps (k order permuted identically for A and B).
//   Partial tiles go to a slab [wg][kgroup][tile][32x32]; gram_reduce sums the
//   slab in a fixed order in fp64 (deterministic) and mirrors to N x N.
//
// Roofline at N=128 (10 tiles): 2*8256*d flops on MFMA vs 4*N*d bytes: MFMA
// bound (~1.05 ms per 1e7 coordinates at the 157 TF fp32 MFMA peak).
#include "sra_common.hpp"

namespace sra {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kStage = 64;            // coordinates per stage
constexpr int kRowPad = kStage + 4;   // LDS row stride in floats

template <int NB>
struct GramCfg {
  static constexpr int NP = 32 * NB;
  static constexpr int T = NB * (NB + 1) / 2;                  // upper-triangle tiles
  static constexpr int WT = NB <= 4 ? 1 : (NB <= 6 ? 2 : 4);   // tile groups
  static constexpr int WK = 4 / WT;                            // k groups
  static constexpr int TPW = (T + WT - 1) / WT;                // tiles per wave (max)
  static constexpr int LOADS = NP * (kStage / 4) / 256;        // float4 per thread per stage
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
  static constexpr int lds_floats = 2 * NP * kRowPad + 2 * kStage + 16 * kStage;
};

int gram_slab_floats(int nb, int64_t num_wg) {
  const int T = nb * (nb + 1) / 2;
  const int WT = nb <= 4 ? 1 : (nb <= 6 ? 2 : 4);
  return static_cast<int>(num_wg * (4 / WT) * T * 1024);
}

template <int NB, bool VEC, int TG>
__device__ __forceinline__ void gram_body(const float* __restrict__ X, int n, int64_t d, int64_t ldx, int64_t chunk,
                                          float* __restrict__ slab, float* lds) {
  using C = GramCfg<NB>;
  constexpr int NP = C::NP;
  constexpr int tg = TG;
  float* buf[2] = {lds, lds + NP * kRowPad};
  float* meanb[2] = {lds + 2 * NP * kRowPad, lds + 2 * NP * kRowPad + kStage};
  float* part = lds + 2 * NP * kRowPad + 2 * kStage;  // [16][64]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int kg = wave / C::WT;
  const int64_t k_begin = static_cast<int64_t>(blockIdx.x) * chunk;
  const int64_t k_end = k_begin + chunk < d ? k_begin + chunk : d;
  const int nstage = k_begin < k_end ? static_cast<int>(cdiv(k_end - k_begin, kStage)) : 0;
  const float inv_n = 1.0f / static_cast<float>(n);

  f32x16 acc[C::TPW];
#pragma unroll
  for (int t = 0; t < C::TPW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // staging registers: thread t owns float4 column c4 = t & 15 of rows (t >> 4) + 16 q
  f32x4 stg[C::LOADS];
  const int c4 = tid & 15;
  const int row0 = tid >> 4;

  auto load_stage = [&](int s) {
    const int64_t k0 = k_begin + static_cast<int64_t>(s) * kStage + 4 * c4;
#pragma unroll
    for (int q = 0; q < C::LOADS; ++q) {
      const int row = row0 + 16 * q;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (row < n) {
        const float* p = X + static_cast<int64_t>(row) * ldx + k0;
        if (VEC && k0 + 3 < k_end) {
          v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (k0 + e < k_end) ? p[e] : 0.f;
        }
      }
      stg[q] = v;
    }
  };
  auto store_stage = [&](float* b) {
    f32x4 colsum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < C::LOADS; ++q) {
      const int row = row0 + 16 * q;
      *reinterpret_cast<f32x4*>(b + row * kRowPad + 4 * c4) = stg[q];
      colsum += stg[q];
    }
    *reinterpret_cast<f32x4*>(part + row0 * kStage + 4 * c4) = colsum;
  };
  // after a barrier: column means of the stage (real rows only) and mean-filled pad rows
  auto finish_means = [&](float* b, float* mb) {
    if (tid < kStage) {
      float s = 0.f;
#pragma unroll
      for (int p = 0; p < 16; ++p) s += part[p * kStage + tid];
      const float mu = s * inv_n;
      mb[tid] = mu;
      for (int r = n; r < NP; ++r) b[r * kRowPad + tid] = mu;  // centred pad rows are exactly 0
    }
  };

  if (nstage > 0) {
    load_stage(0);
    store_stage(buf[0]);
    __syncthreads();
    finish_means(buf[0], meanb[0]);
    if (nstage > 1) load_stage(1);
    __syncthreads();
  }

  const int r = lane & 31;
  const int h = lane >> 5;
  for (int s = 0; s < nstage; ++s) {
    const float* b = buf[s & 1];
    const float* mb = meanb[s & 1];
    // ---- MFMA over this wave's 8-coordinate groups of the stage ----
#pragma unroll 1
    for (int g = kg; g < kStage / 8; g += C::WK) {
      const int col = 8 * g + 4 * h;
      const f32x4 mu = *reinterpret_cast<const f32x4*>(mb + col);
      f32x4 fr[NB];
#pragma unroll
      for (int blk = 0; blk < NB; ++blk)
        fr[blk] = *reinterpret_cast<const f32x4*>(b + (32 * blk + r) * kRowPad + col) - mu;
#pragma unroll
      for (int t = 0; t < C::TPW; ++t) {
        const int tile = tg + C::WT * t;     // compile-time: tg is a template parameter
        if (tile < C::T) {
          const int ti = C::kTileI(tile), tj = C::kTileJ(tile);
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(fr[ti][ks], fr[tj][ks], acc[t], 0, 0, 0);
        }
      }
    }
    // ---- stage s+1 -> LDS (registers were loaded one stage ahead) ----
    if (s + 1 < nstage) {
      store_stage(buf[(s + 1) & 1]);
      if (s + 2 < nstage) load_stage(s + 2);
    }
    __syncthreads();
    if (s + 1 < nstage) finish_means(buf[(s + 1) & 1], meanb[(s + 1) & 1]);
    __syncthreads();
  }

  // ---- partial tiles -> slab[wg][kg][tile][32 x 32] (row-major) ----
  float* my = slab + (static_cast<int64_t>(blockIdx.x) * C::WK + kg) * C::T * 1024;
#pragma unroll
  for (int t = 0; t < C::TPW; ++t) {
    const int tile = tg + C::WT * t;
    if (tile < C::T) {
      float* o = my + tile * 1024;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        o[row * 32 + r] = acc[t][reg];
      }
    }
  }
}

template <int NB, bool VEC>
__global__ void __launch_bounds__(256) gram_partial_kernel(const float* __restrict__ X, int n, int64_t d,
                                                           int64_t ldx, int64_t chunk, float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tg = (threadIdx.x >> 6) % GramCfg<NB>::WT;  // wave-uniform
  if (tg == 0) gram_body<NB, VEC, 0>(X, n, d, ldx, chunk, slab, lds);
  else if (tg == 1) gram_body<NB, VEC, 1>(X, n, d, ldx, chunk, slab, lds);
  else if (tg == 2) gram_body<NB, VEC, 2>(X, n, d, ldx, chunk, slab, lds);
  else gram_body<NB, VEC, 3>(X, n, d, ldx, chunk, slab, lds);
}

// Sum the slab in a fixed order (fp64) and write the symmetric N x N Gram.
template <int NB>
__global__ void __launch_bounds__(256) gram_reduce_kernel(const float* __restrict__ slab, int n, int64_t nslab,
                                                          double* __restrict__ G) {
  using C = GramCfg<NB>;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // (tile, element)
  if (e >= C::T * 1024) return;
  const int tile = e >> 10;
  const int el = e & 1023;
  const int i = 32 * C::kTileI(tile) + (el >> 5);
  const int j = 32 * C::kTileJ(tile) + (el & 31);
  if (i >= n || j >= n) return;
  double s = 0.0;
  for (int64_t w = 0; w < nslab; ++w) s += static_cast<double>(slab[w * C::T * 1024 + e]);
  G[static_cast<int64_t>(i) * n + j] = s;
  G[static_cast<int64_t>(j) * n + i] = s;
}

int gram_num_wg(int64_t d) {
  const int64_t stages = cdiv(d, kStage);
  return static_cast<int>(stages < 256 ? (stages > 0 ? stages : 1) : 256);
}

template <int NB>
static int launch_gram_nb(const float* X, int n, int64_t d, int64_t ldx, double* G, float* slab, hipStream_t s) {
  using C = GramCfg<NB>;
  const int nwg = gram_num_wg(d);
  const int64_t chunk = cdiv(cdiv(d, nwg), kStage) * kStage;
  const size_t lds = sizeof(float) * C::lds_floats;
  const bool vec = (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  if (vec) {
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gram_partial_kernel<NB, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    hipLaunchKernelGGL((gram_partial_kernel<NB, true>), dim3(nwg), dim3(256), lds, s, X, n, d, ldx, chunk, slab);
  } else {
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gram_partial_kernel<NB, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    hipLaunchKernelGGL((gram_partial_kernel<NB, false>), dim3(nwg), dim3(256), lds, s, X, n, d, ldx, chunk, slab);
  }
  int rc = launch_status("gram_partial_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL((gram_reduce_kernel<NB>), dim3(cdiv(C::T * 1024, 256)), dim3(256), 0, s, slab, n,
                     static_cast<int64_t>(nwg) * C::WK, G);
  return launch_status("gram_reduce_kernel");
}

size_t gram_workspace_bytes(int n, int64_t d) {
  const int nb = static_cast<int>(cdiv(n, 32));
  return sizeof(float) * static_cast<size_t>(gram_slab_floats(nb, gram_num_wg(d)));
}

int launch_gram(const float* X, int n, int64_t d, int64_t ldx, double* G, void* ws, size_t ws_bytes,
                hipStream_t s) {
  SRA_REQUIRE(n >= 1 && n <= 256, SRA_ERR_UNSUPPORTED, "Gram supports 1 <= N <= 256 (got %d)", n);
  SRA_REQUIRE(ws != nullptr && ws_bytes >= gram_workspace_bytes(n, d), SRA_ERR_WORKSPACE,
              "Gram workspace too small: need %zu bytes", gram_workspace_bytes(n, d));
  float* slab = static_cast<float*>(ws);
  switch (cdiv(n, 32)) {
    case 1: return launch_gram_nb<1>(X, n, d, ldx, G, slab, s);
    case 2: return launch_gram_nb<2>(X, n, d, ldx, G, slab, s);
    case 3: return launch_gram_nb<3>(X, n, d, ldx, G, slab, s);
    case 4: return launch_gram_nb<4>(X, n, d, ldx, G, slab, s);
    case 5: return launch_gram_nb<5>(X, n, d, ldx, G, slab, s);
    case 6: return launch_gram_nb<6>(X, n, d, ldx, G, slab, s);
    case 7: return launch_gram_nb<7>(X, n, d, ldx, G, slab, s);
    default: return launch_gram_nb<8>(X, n, d, ldx, G, slab, s);
  }
}

}  // namespace sra

extern "C" int sra_gram_workspace_bytes(int64_t n, int64_t d, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && n <= 256 && d >= 1, SRA_ERR_UNSUPPORTED, "Gram supports 1 <= N <= 256, d >= 1");
  *bytes = sra::gram_workspace_bytes(static_cast<int>(n), d);
  return SRA_OK;
}

extern "C" int sra_gram_f32(const float* X, int64_t n, int64_t d, int64_t ldx, double* G, void* ws, size_t ws_bytes,
                            void* stream) {
  SRA_REQUIRE(X != nullptr && G != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx (%lld/%lld)", (long long)d, (long long)ldx);
  return sra::launch_gram(X, static_cast<int>(n), d, ldx, G, ws, ws_bytes, static_cast<hipStream_t>(stream));
}
