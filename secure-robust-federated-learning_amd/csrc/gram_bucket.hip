// k2 + k5 fused -- the centred bf16x3 Gram of mom_krum's bucket means without
// the bucket matrix ("fused into k2's loads for mom_*").
//
// The reference buckets the clients (src/robust_estimator.py:250-256: bucket b
// = np.mean of clients [b*BS, min((b+1)*BS, N)), a sequential fp32 sum over
// axis 0 divided by the count) and runs krum on the bucket means (:234-249).
// The unfused route wrote the B = ceil(N/BS) means to HBM (bucket.hip) and the
// Gram read them back; here every stage of client rows is loaded once, the
// means are formed in registers with the bucket kernel's exact expression
// (so they are the bits np.mean gives), centred by the stage's column means,
// split three ways (x = h + m + l in bf16, exact) and the split fragments are
// written to LDS once, in the MFMA operand layout; the waves then run the six
// bf16 MFMAs per tile and 16-coordinate k-step (hh + hm + mh + hl + lh + mm,
// as gram.hip) reading those fragments.  Only the clients are read from HBM:
// 4*N*d bytes, where the unfused route moved 4*N*d + 8*B*d.
//
// Layout (one 512-thread workgroup per CU, persistent; stage s of workgroup w
// = coordinate tile s * #WG + w, 64 coordinates):
//   loads: 8 lanes per bucket row, lane c8 holds coordinates 4*c8 .. 4*c8+3 and
//     32+4*c8 .. 32+4*c8+3 of every client row of its bucket (each load
//     instruction of a wave covers whole 128-byte lines of 8 rows); 64 bucket
//     rows per sweep; the next stage's loads are issued as soon as this
//     stage's means are formed, so one stage (N*256 bytes) is in flight per CU.
//   fragments: k-step g of the stage = the coordinates of lanes c8 = 2g, 2g+1
//     (a fixed permutation of the stage's columns, the same for every row, so
//     every Gram entry sums the same products); region (g, part, block) holds
//     the 32 x 16 bf16 operand of one 32-row block, lane slot r + 32*hh at
//     16*r + 544*hh bytes; regions 1088 bytes apart and k-steps GS = 64 mod 256
//     bytes apart, so the 16 lanes of a ds_write_b128 / ds_read_b128 phase hit
//     16 distinct 16-byte bank groups.
//   tiles: the T = NB(NB+1)/2 upper-triangle 32x32 tiles, tile t on wave t % 8,
//     all four k-steps of the stage (no k split: one fp32 accumulator set per
//     tile per workgroup); partial tiles -> slab[wg][tile][32x32] reduced by
//     gram.hip's fixed-order fp64 kernels.
// Two barriers per stage: partial column sums visible (also: the previous
// stage's fragment reads are done), fragments written.
#include "gram_common.hpp"

namespace sra {

template <int NB>
struct BucketGramCfg {
  static constexpr int NP = 32 * NB;              // padded bucket rows
  static constexpr int WAVES = 8;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int STAGE = 64;                // coordinates per stage
  static constexpr int SWEEPS = (NP + 63) / 64;   // 64 bucket rows per sweep
  static constexpr int T = NB * (NB + 1) / 2;     // upper-triangle tiles
  static constexpr int TPW = (T + WAVES - 1) / WAVES;
  static constexpr int REG = 1088;                // bytes per (k-step, part, block) operand region
  static constexpr int GS = (3 * NB * REG + 255) / 256 * 256 + 64;   // bytes per k-step
  static constexpr int FRAG = 4 * GS;
  static constexpr int LDS = FRAG + WAVES * STAGE * 4;   // + per-wave column partials
};

template <int NB, int BS, bool VEC>
__global__ void __launch_bounds__(512) gram_bucket_kernel(const float* __restrict__ X, int n, int nb, int64_t d,
                                                          int64_t ldx, float* __restrict__ slab) {
  using C = BucketGramCfg<NB>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* frag = lds;
  float* part = reinterpret_cast<float*>(lds + C::FRAG);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int c8 = tid & 7;
  const int rs = tid >> 3;   // bucket row within a sweep
  const int64_t ntiles = cdiv(d, C::STAGE);
  const int nstage = blockIdx.x < ntiles ? static_cast<int>(cdiv(ntiles - blockIdx.x, gridDim.x)) : 0;
  const float inv_nb = 1.0f / static_cast<float>(nb);

  // this wave's tiles (wave-uniform; they only select LDS regions)
  int ti[C::TPW], tj[C::TPW];
#pragma unroll
  for (int q = 0; q < C::TPW; ++q) {
    int t = wave + C::WAVES * q, i = 0;
    if (t >= C::T) t = 0;
    while (t >= NB - i) {
      t -= NB - i;
      ++i;
    }
    ti[q] = i;
    tj[q] = i + t;
  }

  f32x16 acc[C::TPW];
#pragma unroll
  for (int q = 0; q < C::TPW; ++q)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;

  f32x4 raw[C::SWEEPS][BS][2];
  auto load = [&](int s) {
    const int64_t kb = (static_cast<int64_t>(s) * gridDim.x + blockIdx.x) * C::STAGE;
    const bool full = VEC && kb + C::STAGE <= d;
#pragma unroll
    for (int sw = 0; sw < C::SWEEPS; ++sw)
#pragma unroll
      for (int i = 0; i < BS; ++i) {
        const int row = (64 * sw + rs) * BS + i;
        f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
        if (row < n) {
          const float* p = X + static_cast<int64_t>(row) * ldx + kb + 4 * c8;
          if (full) {
            v0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
            v1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 32));
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v0[e] = kb + 4 * c8 + e < d ? p[e] : 0.f;
              v1[e] = kb + 32 + 4 * c8 + e < d ? p[32 + e] : 0.f;
            }
          }
        }
        raw[sw][i][0] = v0;
        raw[sw][i][1] = v1;
      }
  };

  const int r = lane & 31;
  const int hh = lane >> 5;
  const int rd_off = 16 * r + 544 * hh;   // this lane's operand slot in a region

  if (nstage > 0) load(0);
  for (int s = 0; s < nstage; ++s) {
    // ---- bucket means (bucket.hip's expression: sequential fp32 sum / count)
    f32x4 m[C::SWEEPS][2];
    f32x4 cs0 = {0.f, 0.f, 0.f, 0.f}, cs1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sw = 0; sw < C::SWEEPS; ++sw) {
      const int b = 64 * sw + rs;
      const int left = n - b * BS;
      const float cnt = static_cast<float>(left < BS ? left : BS);
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < BS; ++i) {   // rows past N were loaded as 0: adding them changes nothing
        a0 += raw[sw][i][0];
        a1 += raw[sw][i][1];
      }
      const bool live = b < nb;
      m[sw][0] = live ? a0 / cnt : f32x4{0.f, 0.f, 0.f, 0.f};
      m[sw][1] = live ? a1 / cnt : f32x4{0.f, 0.f, 0.f, 0.f};
      cs0 += m[sw][0];
      cs1 += m[sw][1];
    }
    if (s + 1 < nstage) load(s + 1);
    // ---- column sums: the wave's 8 rows (xor butterfly, same bits in every
    // lane), then the 8 waves in a fixed order after the barrier
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int off = 8; off <= 32; off <<= 1) {
        cs0[e] += __shfl_xor(cs0[e], off);
        cs1[e] += __shfl_xor(cs1[e], off);
      }
    }
    if (lane < 8) {
      *reinterpret_cast<f32x4*>(part + wave * C::STAGE + 4 * c8) = cs0;
      *reinterpret_cast<f32x4*>(part + wave * C::STAGE + 32 + 4 * c8) = cs1;
    }
    __syncthreads();   // partials visible; every wave is past the previous stage's fragment reads
    f32x4 mu0 = *reinterpret_cast<const f32x4*>(part + 4 * c8);
    f32x4 mu1 = *reinterpret_cast<const f32x4*>(part + 32 + 4 * c8);
#pragma unroll
    for (int w = 1; w < C::WAVES; ++w) {
      mu0 += *reinterpret_cast<const f32x4*>(part + w * C::STAGE + 4 * c8);
      mu1 += *reinterpret_cast<const f32x4*>(part + w * C::STAGE + 32 + 4 * c8);
    }
    mu0 *= inv_nb;
    mu1 *= inv_nb;
    // ---- centre, split, fragments -> LDS
    {
      const int g = c8 >> 1, h2 = c8 & 1;
#pragma unroll
      for (int sw = 0; sw < C::SWEEPS; ++sw) {
        const int b = 64 * sw + rs;
        if (64 * sw + 64 > C::NP && b >= C::NP) continue;
        const bool live = b < nb;
        const f32x4 a0 = live ? m[sw][0] - mu0 : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 a1 = live ? m[sw][1] - mu1 : f32x4{0.f, 0.f, 0.f, 0.f};
        uint32_t h4[4], m4[4], l4[4];
        split3_pair(a0[0], a0[1], h4[0], m4[0], l4[0]);
        split3_pair(a0[2], a0[3], h4[1], m4[1], l4[1]);
        split3_pair(a1[0], a1[1], h4[2], m4[2], l4[2]);
        split3_pair(a1[2], a1[3], h4[3], m4[3], l4[3]);
        const u32x4 ph = {h4[0], h4[1], h4[2], h4[3]};
        const u32x4 pm = {m4[0], m4[1], m4[2], m4[3]};
        const u32x4 pl = {l4[0], l4[1], l4[2], l4[3]};
        char* base = frag + g * C::GS + (b >> 5) * C::REG + 16 * (b & 31) + 544 * h2;
        *reinterpret_cast<u32x4*>(base) = ph;
        *reinterpret_cast<u32x4*>(base + NB * C::REG) = pm;
        *reinterpret_cast<u32x4*>(base + 2 * NB * C::REG) = pl;
      }
    }
    __syncthreads();   // fragments written
    // ---- six bf16 MFMAs per tile and k-step
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const char* fg = frag + g * C::GS + rd_off;
#pragma unroll
      for (int q = 0; q < C::TPW; ++q) {
        if (wave + C::WAVES * q < C::T) {
          const char* fa = fg + ti[q] * C::REG;
          const char* fb = fg + tj[q] * C::REG;
          const bf16x8 ah = *reinterpret_cast<const bf16x8*>(fa);
          const bf16x8 am = *reinterpret_cast<const bf16x8*>(fa + NB * C::REG);
          const bf16x8 al = *reinterpret_cast<const bf16x8*>(fa + 2 * NB * C::REG);
          const bf16x8 bh = *reinterpret_cast<const bf16x8*>(fb);
          const bf16x8 bm = *reinterpret_cast<const bf16x8*>(fb + NB * C::REG);
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(fb + 2 * NB * C::REG);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc[q], 0, 0, 0);
        }
      }
    }
  }

  // ---- partial tiles -> slab[wg][tile][32 x 32] (gram.hip's layout)
  float* my = slab + static_cast<int64_t>(blockIdx.x) * C::T * 1024;
#pragma unroll
  for (int q = 0; q < C::TPW; ++q) {
    const int t = wave + C::WAVES * q;
    if (t < C::T) {
      float* o = my + t * 1024;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * hh;
        o[row * 32 + r] = acc[q][reg];
      }
    }
  }
}

template <int NB, int BS>
static int launch_bucket_nb(const float* X, int n, int nb, int64_t d, int64_t ldx, float* slab, int nwg,
                            hipStream_t s) {
  using C = BucketGramCfg<NB>;
  const bool vec = ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  const void* fn = vec ? reinterpret_cast<const void*>(&gram_bucket_kernel<NB, BS, true>)
                       : reinterpret_cast<const void*>(&gram_bucket_kernel<NB, BS, false>);
  SRA_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS));
  if (vec)
    hipLaunchKernelGGL((gram_bucket_kernel<NB, BS, true>), dim3(nwg), dim3(C::THREADS), C::LDS, s, X, n, nb, d, ldx,
                       slab);
  else
    hipLaunchKernelGGL((gram_bucket_kernel<NB, BS, false>), dim3(nwg), dim3(C::THREADS), C::LDS, s, X, n, nb, d, ldx,
                       slab);
  return launch_status("gram_bucket_kernel");
}

template <int NB>
static int launch_bucket_bs(const float* X, int n, int nb, int bs, int64_t d, int64_t ldx, float* slab, int nwg,
                            hipStream_t s) {
  switch (bs) {
    case 1: return launch_bucket_nb<NB, 1>(X, n, nb, d, ldx, slab, nwg, s);
    case 2: return launch_bucket_nb<NB, 2>(X, n, nb, d, ldx, slab, nwg, s);
    case 3: return launch_bucket_nb<NB, 3>(X, n, nb, d, ldx, slab, nwg, s);
    default: return launch_bucket_nb<NB, 4>(X, n, nb, d, ldx, slab, nwg, s);
  }
}

// slab: nwg x T(NB) x 1024 floats, NB = ceil(nb / 32) <= kBucketGramMaxNB, 1 <= bs <= 4
int launch_gram_bucket_partial(const float* X, int n, int nb, int bs, int64_t d, int64_t ldx, float* slab, int nwg,
                               hipStream_t s) {
  SRA_REQUIRE(bs >= 1 && bs <= 4 && nb == static_cast<int>(cdiv(n, bs)) && nb <= 32 * kBucketGramMaxNB,
              SRA_ERR_UNSUPPORTED, "bucket Gram: 1 <= bucket size <= 4 and at most %d buckets",
              32 * kBucketGramMaxNB);
  switch (cdiv(nb, 32)) {
    case 1: return launch_bucket_bs<1>(X, n, nb, bs, d, ldx, slab, nwg, s);
    case 2: return launch_bucket_bs<2>(X, n, nb, bs, d, ldx, slab, nwg, s);
    case 3: return launch_bucket_bs<3>(X, n, nb, bs, d, ldx, slab, nwg, s);
    case 4: return launch_bucket_bs<4>(X, n, nb, bs, d, ldx, slab, nwg, s);
    case 5: return launch_bucket_bs<5>(X, n, nb, bs, d, ldx, slab, nwg, s);
    default: return launch_bucket_bs<6>(X, n, nb, bs, d, ldx, slab, nwg, s);
  }
}

}  // namespace sra
