// k2 — centred pairwise Gram matrix G = Xc Xc^T (N x N, fp64 result) on the
// bf16 MFMA with a three-way split of every fp32 value (v_mfma_f32_32x32x16_bf16).
//
// Feeds every pairwise-L2 consumer of the reference:
//   krum_ / krum / mom_krum  (src/robust_estimator.py:234-257)
//   bulyan(aggsubfunc='krum') (src/robust_estimator.py:286-296)
// through ||x_i - x_j||^2 = G_ii + G_jj - 2 G_ij.
//
// Centring: before the MFMA every stage is shifted by its per-coordinate
// client mean (distances are translation invariant), which removes the
// cancellation of the expanded form when clients share a large common
// component.  All (i, j) entries accumulate their products in the same k
// order, so two identical clients get G_ii == G_jj == G_ij bit for bit and
// distance exactly 0, as in the reference (identical rows of the `xie`
// attack, src/attack.py:362-372).
//
// Precision: each centred fp32 value x is split exactly into three bf16
// parts x = h + m + l (round-to-nearest h, then m of the remainder, then l of
// what is left: 8 + 8 + 8 significant bits); the product x y is formed from
// the six terms hh + hm + mh + hl + lh + mm on the bf16 MFMA (exact products,
// fp32 accumulation), dropping ml + lm + ll (< 3 * 2^-24 of |x y|) -- the
// accuracy of an fp32 product -- at 16x the fp32 MFMA's rate: six bf16
// MFMAs cost 3/8 of one fp32 32x32x2 pass over the same k, so the kernel is
// bound by HBM instead of the fp32 MFMA (round 1: 2.15 ms at N=128, d=1e7).
//
// Layout / schedule (one workgroup of 4 or 8 waves per CU, persistent;
// workgroup w takes coordinate tiles w, w + #WG, ... so the chip streams
// neighbouring tiles of every row at once):
//   stage = NP rows x STAGE coordinates, register-staged float4 loads (one
//   stage ahead) -> LDS [row][STAGE + 4 pad], double buffered; per-wave column
//   partial sums from the staging registers, reduced to the stage's column
//   means in a fixed order after the stage barrier.
//   wave w owns a set of upper-triangle 32x32 output tiles (I <= J) and a
//   subset of the 16-coordinate k-steps (K split across waves).  Two
//   ds_read_b128 per row block give a lane its 8 values of a k-step; centre
//   by the stage means, split, six MFMAs per tile.
//   Partial tiles go to a slab [wg][kgroup][tile][32x32]; gram_reduce sums the
//   slab in a fixed order in fp64 (deterministic) and mirrors to N x N.
//
// Roofline at N=128: 4*N*d bytes streamed once; the MFMA work (6 bf16
// 32x32x16 per tile and k-step, 10 tiles) is ~0.5 ms per 1e7 coordinates at
// the 2.5 PF bf16 peak, below the ~0.8 ms of HBM time.
#include "sra_common.hpp"
#include "gram_common.hpp"

#include <cstdlib>

namespace sra {

// exact three-way bf16 split of 8 fp32 values: x = h + m + l
__device__ __forceinline__ void split3(const f32x4& a, const f32x4& b, bf16x8& h, bf16x8& m, bf16x8& l) {
  float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 hh = static_cast<__bf16>(x[e]);
    const float r1 = x[e] - static_cast<float>(hh);
    const __bf16 mm = static_cast<__bf16>(r1);
    const float r2 = r1 - static_cast<float>(mm);
    h[e] = hh;
    m[e] = mm;
    l[e] = static_cast<__bf16>(r2);
  }
}

template <int NB, int WAVES, int STG = 0>
int gram_slab_floats_t(int64_t num_wg) {
  using C = GramCfg<NB, WAVES, STG>;
  return static_cast<int>(num_wg * C::WK * C::T * 1024);
}

// sum of x over the 4 lanes {l, l^16, l^32, l^48} of a wave
__device__ __forceinline__ float sum_lanes_16_32(float x) {
  // xor 16 inside each 32-lane half (ds_swizzle bit mode: and 0x1f, xor 0x10)
  x += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, x), 0x401f));
  // xor 32 across the halves
  x += __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(((threadIdx.x & 63) ^ 32) << 2,
                                                              __builtin_bit_cast(int, x)));
  return x;
}

// Row r of the (virtual) input is X + r ldx for r < split, else X2 + (r - split)
// ldx: two 128-row blocks of a larger matrix side by side (N > 256, the pair
// path below).  shift != nullptr replaces the per-stage client mean by a
// fixed per-coordinate shift (the mean over ALL N clients), so the pairs'
// Grams are centred alike and assemble into one matrix.
// sum of x over the 32 lanes of each wave half (xor butterfly: every lane of a
// half ends with the same bits, since a + b == b + a exactly)
__device__ __forceinline__ float sum_lanes_32(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, x), 0x101f));
  x += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, x), 0x201f));
  x += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, x), 0x401f));
  return x;
}

// PF: register stage sets in flight (2: the loads of stage s + 3 are issued
// while stage s computes, two stages of MFMA work to cover HBM latency).
// WM: every wave derives the column means of its own k-steps from the values
// it reads for the MFMA (sum_lanes_32 over the 32 rows of a block, blocks in
// a fixed order; waves sharing k-steps compute the same bits), so a stage
// needs one barrier and no partial-sum pass.  WM requires shift == nullptr.
template <int NB, int WAVES, bool VEC, int TG, int STG, int PF = 1, bool WM = false>
__device__ __forceinline__ void gram_body(const float* __restrict__ X, const float* __restrict__ X2, int split, int n,
                                          int64_t d, int64_t ldx, const float* __restrict__ shift, int64_t chunk,
                                          float* __restrict__ slab, float* lds) {
  using C = GramCfg<NB, WAVES, STG>;
  constexpr int STAGE = C::STAGE;
  constexpr int tg = TG;
  // LDS carve-up (pointers derived arithmetically from the __shared__ base so
  // the compiler keeps them in the LDS address space: ds_read/ds_write)
  auto bufp = [&](int which) { return lds + which * C::BUF; };
  float* part = lds + 2 * C::BUF;
  auto mup = [&](int which) { return lds + 2 * C::BUF + C::PART + which * STAGE; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int kg = wave / C::WT;
  // stage s of this workgroup = coordinate tile s * gridDim.x + blockIdx.x: all
  // workgroups stream neighbouring tiles of the N rows at any moment (a
  // contiguous chunk per workgroup kept N x #WG pages open at once)
  (void)chunk;
  const int64_t ntiles = cdiv(d, STAGE);
  const int nstage = blockIdx.x < ntiles ? static_cast<int>(cdiv(ntiles - blockIdx.x, gridDim.x)) : 0;
  const int64_t k_end = d;
  const float inv_n = 1.0f / static_cast<float>(n);

  f32x16 acc[C::TPW];
#pragma unroll
  for (int t = 0; t < C::TPW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // staging: thread t owns float4 column c4 = t % C4 of rows t / C4 + RSTEP * q
  f32x4 stg[PF][C::LOADS];
  const int c4 = tid % C::C4;
  const int row0 = tid / C::C4;

  // fast path (all NP rows present in X, the stage inside [0, d), 16-byte
  // aligned rows): a wave-uniform row base per load plus one 32-bit lane
  // offset (global_load with an SGPR base), no per-load guards
  const bool rows_full = VEC && n >= C::NP && split >= C::NP &&
                         static_cast<int64_t>(C::RSTEP - 1) * ldx * 4 + 4 * STAGE < (int64_t(1) << 31);
  const uint32_t lane_off = static_cast<uint32_t>((static_cast<int64_t>(row0) * ldx + 4 * c4) * 4);
  auto load_stage = [&](int s, auto setc) {
    constexpr int P = decltype(setc)::value;
    const int64_t kb = (static_cast<int64_t>(s) * gridDim.x + blockIdx.x) * STAGE;
    // (the WM kernels only: in the eight-wave N > 128 kernels the extra path
    // cost 17 % -- 4.07 vs 4.75 ms at N = 171 buckets, same box)
    if (WM && rows_full && kb + STAGE <= k_end) {
#pragma unroll
      for (int q = 0; q < C::LOADS; ++q) {
        const char* bq = reinterpret_cast<const char*>(X + static_cast<int64_t>(C::RSTEP * q) * ldx + kb);
        stg[P][q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(bq + lane_off));
      }
      return;
    }
    const int64_t k0 = kb + 4 * c4;
#pragma unroll
    for (int q = 0; q < C::LOADS; ++q) {
      const int row = row0 + C::RSTEP * q;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (row < n && row < C::NP) {
        const float* p = (row < split ? X + static_cast<int64_t>(row) * ldx
                                      : X2 + static_cast<int64_t>(row - split) * ldx) + k0;
        if (VEC && k0 + 3 < k_end) {
          v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (k0 + e < k_end) ? p[e] : 0.f;
        }
      }
      stg[P][q] = v;
    }
  };
  // registers -> LDS stage buffer, plus this wave's column partial sums
  // (the 64 lanes of a wave cover C4/…: lanes with equal c4 are reduced by
  // swizzles, then lanes with lane < C4 own the wave's partial of 4 columns)
  auto store_stage = [&](float* b, float* part, auto setc) {
    constexpr int P = decltype(setc)::value;
    f32x4 colsum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < C::LOADS; ++q) {
      const int row = row0 + C::RSTEP * q;
      if (row < C::NP) *reinterpret_cast<f32x4*>(b + row * C::ROWPAD + 4 * c4) = stg[P][q];
      if constexpr (!WM) colsum += stg[P][q];
    }
    if constexpr (WM) return;
    if constexpr (C::C4 == 16) {
#pragma unroll
      for (int e = 0; e < 4; ++e) colsum[e] = sum_lanes_16_32(colsum[e]);
      if (lane < 16) *reinterpret_cast<f32x4*>(part + wave * STAGE + 4 * c4) = colsum;
    } else {  // C4 == 32: lanes l and l^32 share columns
#pragma unroll
      for (int e = 0; e < 4; ++e)
        colsum[e] += __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute((lane ^ 32) << 2,
                                                                            __builtin_bit_cast(int, colsum[e])));
      if (lane < 32) *reinterpret_cast<f32x4*>(part + wave * STAGE + 4 * c4) = colsum;
    }
  };

  // column means of a stored stage: fixed order over the waves' partials
  auto stage_means = [&](float* mu, int s) {
    if (shift != nullptr) {
      const int64_t c0 = (static_cast<int64_t>(s) * gridDim.x + blockIdx.x) * STAGE;
      for (int c = tid; c < STAGE; c += C::THREADS) mu[c] = c0 + c < k_end ? shift[c0 + c] : 0.f;
      return;
    }
    for (int c = tid; c < STAGE; c += C::THREADS) {
      float m = part[c];
#pragma unroll
      for (int w = 1; w < WAVES; ++w) m += part[w * STAGE + c];
      mu[c] = m * inv_n;
    }
  };

  if (nstage > 0) {
    load_stage(0, IC<0>{});
    if constexpr (PF == 2) {
      if (nstage > 1) load_stage(1, IC<1>{});
    }
    store_stage(bufp(0), part, IC<0>{});
    if (nstage > PF) load_stage(PF, IC<0>{});
    __syncthreads();
    if constexpr (!WM) {
      stage_means(mup(0), 0);
      __syncthreads();
    }
  }

  const int r = lane & 31;
  const int h = lane >> 5;
  // rows >= n of the last block are zeroed after centring (their staged value is 0)
  const float last_mask = (32 * (NB - 1) + r) < n ? 1.f : 0.f;
  auto step = [&](int s, auto parc) {
    constexpr int SN = PF == 2 ? 1 - decltype(parc)::value : 0;   // register set of stage s + 1
    const float* b = bufp(s & 1);
    const float* mu = mup(s & 1);
    // ---- MFMA over this wave's 16-coordinate k-steps of the stage ----
#pragma unroll
    for (int gi = 0; gi < C::KPW; ++gi) {
      const int g = kg + C::WK * gi;
      const int col = 16 * g + 8 * h;
      f32x4 mu0, mu1;
      f32x4 raw0[NB], raw1[NB];
      if constexpr (WM) {
#pragma unroll
        for (int blk = 0; blk < NB; ++blk) {
          const float* rp = b + (32 * blk + r) * C::ROWPAD + col;
          raw0[blk] = *reinterpret_cast<const f32x4*>(rp);
          raw1[blk] = *reinterpret_cast<const f32x4*>(rp + 4);
        }
        mu0 = raw0[0];
        mu1 = raw1[0];
#pragma unroll
        for (int blk = 1; blk < NB; ++blk) {
          mu0 += raw0[blk];
          mu1 += raw1[blk];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          mu0[e] = sum_lanes_32(mu0[e]) * inv_n;
          mu1[e] = sum_lanes_32(mu1[e]) * inv_n;
        }
      } else {
        mu0 = *reinterpret_cast<const f32x4*>(mu + col);
        mu1 = *reinterpret_cast<const f32x4*>(mu + col + 4);
      }
      bf16x8 fh[NB], fm[NB], fl[NB];
#pragma unroll
      for (int blk = 0; blk < NB; ++blk) {
        const float* rp = b + (32 * blk + r) * C::ROWPAD + col;
        f32x4 a0, a1;
        if constexpr (WM) {
          a0 = raw0[blk] - mu0;
          a1 = raw1[blk] - mu1;
        } else {
          a0 = *reinterpret_cast<const f32x4*>(rp) - mu0;
          a1 = *reinterpret_cast<const f32x4*>(rp + 4) - mu1;
        }
        if (blk == NB - 1) {
          a0 *= last_mask;
          a1 *= last_mask;
        }
        split3(a0, a1, fh[blk], fm[blk], fl[blk]);
      }
#pragma unroll
      for (int t = 0; t < C::TPW; ++t) {
        const int tile = tg + C::WT * t;     // compile-time: tg is a template parameter
        if (tile < C::T) {
          const int ti = C::kTileI(tile), tj = C::kTileJ(tile);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh[ti], fh[tj], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh[ti], fm[tj], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fm[ti], fh[tj], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh[ti], fl[tj], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fl[ti], fh[tj], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fm[ti], fm[tj], acc[t], 0, 0, 0);
        }
      }
    }
    // ---- stage s+1 -> LDS (its registers were loaded one stage ahead) ----
    if (s + 1 < nstage) {
      store_stage(bufp((s + 1) & 1), part, IC<SN>{});
      if (s + 1 + PF < nstage) load_stage(s + 1 + PF, IC<SN>{});
    }
    __syncthreads();
    if constexpr (!WM) {
      if (s + 1 < nstage) {
        stage_means(mup((s + 1) & 1), s + 1);
        __syncthreads();
      }
    }
  };
  if constexpr (PF == 1) {
    for (int s = 0; s < nstage; ++s) step(s, IC<0>{});   // one body: the I-cache holds it
  } else {
    for (int s = 0; s < nstage; s += 2) {
      step(s, IC<0>{});
      if (s + 1 < nstage) step(s + 1, IC<1>{});
    }
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

template <int NB, int WAVES, bool VEC, int STG = 0, int PF = 1, bool WM = false>
__global__ void __launch_bounds__(64 * WAVES) gram_partial_kernel(const float* __restrict__ X,
                                                                  const float* __restrict__ X2, int split, int n,
                                                                  int64_t d, int64_t ldx,
                                                                  const float* __restrict__ shift, int64_t chunk,
                                                                  float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int WT = GramCfg<NB, WAVES, STG>::WT;
  const int tg = (threadIdx.x >> 6) % WT;  // wave-uniform
#define SRA_GB(TGV) gram_body<NB, WAVES, VEC, TGV, STG, PF, WM>(X, X2, split, n, d, ldx, shift, chunk, slab, lds)
  if (tg == 0) SRA_GB(0);
  if constexpr (WT > 1) if (tg == 1) SRA_GB(1);
  if constexpr (WT > 2) {
    if (tg == 2) SRA_GB(2);
    if (tg == 3) SRA_GB(3);
  }
  if constexpr (WT > 4) {
    if (tg == 4) SRA_GB(4);
    if (tg == 5) SRA_GB(5);
    if (tg == 6) SRA_GB(6);
    if (tg == 7) SRA_GB(7);
  }
#undef SRA_GB
}

// Slab reduction in a fixed order (deterministic), fp64, two levels:
//  level 1: block (x, g) sums slab entries [g*per, (g+1)*per) of 256 elements;
//  level 2: sums the kRedGroups partials in order and mirrors to N x N.
constexpr int kRedGroups = 32;

template <int NB>
__global__ void __launch_bounds__(256) gram_reduce1_kernel(const float* __restrict__ slab, int64_t nslab,
                                                           double* __restrict__ partial) {
  using C = GramCfg<NB>;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (e >= C::T * 1024) return;
  const int64_t per = (nslab + kRedGroups - 1) / kRedGroups;
  const int64_t w0 = g * per;
  const int64_t w1 = w0 + per < nslab ? w0 + per : nslab;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int64_t w = w0;
  for (; w + 4 <= w1; w += 4) {
    s0 += static_cast<double>(slab[(w + 0) * C::T * 1024 + e]);
    s1 += static_cast<double>(slab[(w + 1) * C::T * 1024 + e]);
    s2 += static_cast<double>(slab[(w + 2) * C::T * 1024 + e]);
    s3 += static_cast<double>(slab[(w + 3) * C::T * 1024 + e]);
  }
  for (; w < w1; ++w) s0 += static_cast<double>(slab[w * C::T * 1024 + e]);
  partial[static_cast<int64_t>(g) * C::T * 1024 + e] = (s0 + s1) + (s2 + s3);
}

template <int NB>
__global__ void __launch_bounds__(256) gram_reduce2_kernel(const double* __restrict__ partial, int n,
                                                           double* __restrict__ G) {
  using C = GramCfg<NB>;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= C::T * 1024) return;
  const int tile = e >> 10;
  const int el = e & 1023;
  const int i = 32 * C::kTileI(tile) + (el >> 5);
  const int j = 32 * C::kTileJ(tile) + (el & 31);
  if (i >= n || j >= n) return;
  // a diagonal tile holds both (i, j) and (j, i), whose MFMA sums may differ in
  // the last bits: only the upper one writes the pair (two writers of one
  // address made G differ from call to call)
  if (C::kTileI(tile) == C::kTileJ(tile) && (el >> 5) > (el & 31)) return;
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < kRedGroups; ++g) s += partial[static_cast<int64_t>(g) * C::T * 1024 + e];
  G[static_cast<int64_t>(i) * n + j] = s;
  G[static_cast<int64_t>(j) * n + i] = s;
}

// Pair path (N > 256): the entries of a virtual pair matrix [block a; block b]
// land at rows off_a + i (i < split) / off_b + i - split of the N x N G; the
// diagonal blocks only where asked (each entry of G is written by one pair).
template <int NB>
__global__ void __launch_bounds__(256) gram_reduce2_pair_kernel(const double* __restrict__ partial, int n, int split,
                                                                int off_a, int off_b, int ldg, int write_aa,
                                                                int write_bb, double* __restrict__ G) {
  using C = GramCfg<NB>;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= C::T * 1024) return;
  const int tile = e >> 10;
  const int el = e & 1023;
  const int i = 32 * C::kTileI(tile) + (el >> 5);
  const int j = 32 * C::kTileJ(tile) + (el & 31);
  if (i >= n || j >= n) return;
  const bool ia = i < split, ja = j < split;
  if ((ia && ja && !write_aa) || (!ia && !ja && !write_bb)) return;
  if (C::kTileI(tile) == C::kTileJ(tile) && (el >> 5) > (el & 31)) return;   // as gram_reduce2_kernel
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < kRedGroups; ++g) s += partial[static_cast<int64_t>(g) * C::T * 1024 + e];
  const int64_t gi = ia ? off_a + i : off_b + i - split;
  const int64_t gj = ja ? off_a + j : off_b + j - split;
  G[gi * ldg + gj] = s;
  G[gj * ldg + gi] = s;
}

// fp32 column mean over the n rows (sequential, like the stage means)
__global__ void __launch_bounds__(256) gram_shift_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                         float* __restrict__ shift) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (j >= d) return;
  float m = 0.f;
  for (int i = 0; i < n; ++i) m += X[static_cast<int64_t>(i) * ldx + j];
  shift[j] = m * (1.0f / static_cast<float>(n));
}

int gram_num_wg(int64_t d) {
  const int64_t stages = cdiv(d, 64);
  return static_cast<int>(stages < 256 ? (stages > 0 ? stages : 1) : 256);
}

// 4 waves (one per SIMD, all tiles of a k-step in one wave: the fragments are
// centred and split once per wave) for N <= 128 -- measured 1.43 vs 1.50 ms
// for 8 waves at N = 128, d = 1e7; 8 waves for larger N (the 4-wave tile
// groups would need more accumulators than a wave holds).
static constexpr int gram_waves(int nb) { return nb <= 4 ? 4 : 8; }

// pair: (off_a, off_b, split, ldg, write_aa, write_bb) of the pair path, or
// nullptr for a whole matrix of n <= 256 rows
struct GramPair {
  const float* X2;
  const float* shift;
  int split, off_a, off_b, ldg, write_aa, write_bb;
};

template <int NB, int WAVES, int STG = 0, int PF = 1, bool WM = false, bool PIPE = false>
static int launch_gram_nbw(const float* X, int n, int64_t d, int64_t ldx, double* G, float* slab, hipStream_t s,
                           const GramPair* pr = nullptr) {
  using C = GramCfg<NB, WAVES, STG>;
  const int nwg = gram_num_wg(d) * (STG == 64 && NB <= 4 ? 2 : 1);
  const int64_t chunk = cdiv(cdiv(d, nwg), C::STAGE) * C::STAGE;
  const size_t lds = sizeof(float) * C::lds_floats;
  const float* X2 = pr ? pr->X2 : X;
  const int split = pr ? pr->split : n;
  const float* shift = pr ? pr->shift : nullptr;
  const bool vec = (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(X2) & 15) == 0);
  if constexpr (PIPE) {
    static_assert(NB == 4 && WAVES == 4 && STG == 0, "pipelined Gram: N in (96, 128], four waves");
    SRA_REQUIRE(pr == nullptr && n == 128 && vec && d % C::STAGE == 0, SRA_ERR_ARG,
                "pipelined Gram needs N == 128, aligned rows and d %% %d == 0", C::STAGE);
    const int rc0 = launch_gram_pipe(X, n, d, ldx, slab, nwg, s);
    if (rc0) return rc0;
  } else if (vec) {
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gram_partial_kernel<NB, WAVES, true, STG, PF, WM>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    hipLaunchKernelGGL((gram_partial_kernel<NB, WAVES, true, STG, PF, WM>), dim3(nwg), dim3(C::THREADS), lds, s, X, X2, split,
                       n, d, ldx, shift, chunk, slab);
  } else {
    SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gram_partial_kernel<NB, WAVES, false, STG, PF, WM>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    hipLaunchKernelGGL((gram_partial_kernel<NB, WAVES, false, STG, PF, WM>), dim3(nwg), dim3(C::THREADS), lds, s, X, X2,
                       split, n, d, ldx, shift, chunk, slab);
  }
  int rc = launch_status("gram_partial_kernel");
  if (rc) return rc;
  double* partial = reinterpret_cast<double*>(slab + static_cast<size_t>(gram_slab_floats_t<NB, WAVES, STG>(nwg)));
  hipLaunchKernelGGL((gram_reduce1_kernel<NB>), dim3(cdiv(C::T * 1024, 256), kRedGroups), dim3(256), 0, s, slab,
                     static_cast<int64_t>(nwg) * C::WK, partial);
  rc = launch_status("gram_reduce1_kernel");
  if (rc) return rc;
  if (pr) {
    hipLaunchKernelGGL((gram_reduce2_pair_kernel<NB>), dim3(cdiv(C::T * 1024, 256)), dim3(256), 0, s, partial, n,
                       pr->split, pr->off_a, pr->off_b, pr->ldg, pr->write_aa, pr->write_bb, G);
    return launch_status("gram_reduce2_pair_kernel");
  }
  hipLaunchKernelGGL((gram_reduce2_kernel<NB>), dim3(cdiv(C::T * 1024, 256)), dim3(256), 0, s, partial, n, G);
  return launch_status("gram_reduce2_kernel");
}

// Kernel choice (DESIGN k2; the losing variants of rounds 2-3 -- two register
// stage sets, 64-coordinate stages, eight-wave per-wave means, phase-B loads --
// are recorded there and no longer built):
//   N == 128, 16-byte aligned rows, d % 128 == 0, 32-bit row offsets: the
//     software-pipelined kernel (gram_pipe.hip);
//   other N <= 128 without a pair: four waves with per-wave column means;
//   pairs (N > 256) and N > 128: the partial-sum means kernel.
template <int NB>
static int launch_gram_nb(const float* X, int n, int64_t d, int64_t ldx, double* G, float* slab, hipStream_t s,
                          const GramPair* pr = nullptr) {
  if constexpr (NB <= 4) {
    if (pr == nullptr) {
      if constexpr (NB == 4) {
        const bool aligned = ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
        if (n == 128 && aligned && d % 128 == 0 && gram_pipe_offsets_fit(ldx))
          return launch_gram_nbw<4, 4, 0, 1, true, true>(X, n, d, ldx, G, slab, s, pr);
      }
      return launch_gram_nbw<NB, 4, 0, 1, true>(X, n, d, ldx, G, slab, s, pr);
    }
  }
  if constexpr (gram_waves(NB) == 4) return launch_gram_nbw<NB, 4>(X, n, d, ldx, G, slab, s, pr);
  return launch_gram_nbw<NB, 8>(X, n, d, ldx, G, slab, s, pr);
}

// Gram of the bucket means (gram_bucket.hip) + the fixed-order fp64 reduction
template <int NB>
static int gram_reduce_slab(const float* slab, int64_t nslab, int n, double* G, hipStream_t s) {
  using C = GramCfg<NB>;
  double* partial = reinterpret_cast<double*>(const_cast<float*>(slab) + nslab * C::T * 1024);
  hipLaunchKernelGGL((gram_reduce1_kernel<NB>), dim3(cdiv(C::T * 1024, 256), kRedGroups), dim3(256), 0, s, slab, nslab,
                     partial);
  const int rc = launch_status("gram_reduce1_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL((gram_reduce2_kernel<NB>), dim3(cdiv(C::T * 1024, 256)), dim3(256), 0, s, partial, n, G);
  return launch_status("gram_reduce2_kernel");
}

int launch_gram_buckets(const float* X, int n, int bs, int64_t d, int64_t ldx, double* G, float* slab,
                        hipStream_t s) {
  const int nb = static_cast<int>(cdiv(n, bs));
  const int nwg = gram_num_wg(d);
  const int rc = launch_gram_bucket_partial(X, n, nb, bs, d, ldx, slab, nwg, s);
  if (rc) return rc;
  switch (cdiv(nb, 32)) {
    case 1: return gram_reduce_slab<1>(slab, nwg, nb, G, s);
    case 2: return gram_reduce_slab<2>(slab, nwg, nb, G, s);
    case 3: return gram_reduce_slab<3>(slab, nwg, nb, G, s);
    case 4: return gram_reduce_slab<4>(slab, nwg, nb, G, s);
    case 5: return gram_reduce_slab<5>(slab, nwg, nb, G, s);
    default: return gram_reduce_slab<6>(slab, nwg, nb, G, s);
  }
}

constexpr int kGramMaxClients = 8192;   // N > 512: pairs of 128-client blocks (Krum without a client ceiling)
constexpr int kGramPairRows = 128;

size_t gram_workspace_bytes(int n, int64_t d) {
  // sized for the larger of the 4- and 8-wave slab layouts (WK <= 8); N > 256:
  // the 256-row pair layout plus the d-vector shift
  const int nb = static_cast<int>(cdiv(n > 256 ? 256 : n, 32));
  const int T = nb * (nb + 1) / 2;
  const size_t base = sizeof(float) * static_cast<size_t>(gram_num_wg(d)) * 2 * 8 * T * 1024 +
                      sizeof(double) * static_cast<size_t>(kRedGroups) * T * 1024;
  return n > 256 ? base + 256 + sizeof(float) * static_cast<size_t>(d) : base;
}

// N in (256, kGramMaxClients]: clients in blocks of 128; one 256-row launch per
// pair of blocks (p, q), p < q, all centred by the same shift (the fp32 mean
// over all N clients) and run in the same configuration (NB = 8), so every
// entry is accumulated alike whichever pair produced it (identical clients
// still get G_ii == G_jj == G_ij).  Cross blocks come from their pair, the
// diagonal block p from (p, p + 1), the last one from the last pair.
static int launch_gram_pairs(const float* X, int n, int64_t d, int64_t ldx, double* G, float* slab, hipStream_t s) {
  const int nblk = static_cast<int>(cdiv(n, kGramPairRows));
  const size_t base = gram_workspace_bytes(256, d);
  float* shift = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(slab) + base + 255) & ~uintptr_t(255));
  hipLaunchKernelGGL(gram_shift_kernel, dim3(cdiv(d, 256)), dim3(256), 0, s, X, n, d, ldx, shift);
  int rc = launch_status("gram_shift_kernel");
  if (rc) return rc;
  for (int p = 0; p < nblk; ++p) {
    for (int q = p + 1; q < nblk; ++q) {
      const int rows_q = q == nblk - 1 ? n - q * kGramPairRows : kGramPairRows;
      GramPair pr{X + static_cast<int64_t>(q) * kGramPairRows * ldx, shift, kGramPairRows, p * kGramPairRows,
                  q * kGramPairRows, n, q == p + 1 ? 1 : 0, (p == nblk - 2 && q == nblk - 1) ? 1 : 0};
      rc = launch_gram_nb<8>(X + static_cast<int64_t>(p) * kGramPairRows * ldx, kGramPairRows + rows_q, d, ldx, G,
                             slab, s, &pr);
      if (rc) return rc;
    }
  }
  return SRA_OK;
}

int launch_gram(const float* X, int n, int64_t d, int64_t ldx, double* G, void* ws, size_t ws_bytes,
                hipStream_t s) {
  SRA_REQUIRE(n >= 1 && n <= kGramMaxClients, SRA_ERR_UNSUPPORTED, "Gram supports 1 <= N <= %d (got %d)",
              kGramMaxClients, n);
  SRA_REQUIRE(ws != nullptr && ws_bytes >= gram_workspace_bytes(n, d), SRA_ERR_WORKSPACE,
              "Gram workspace too small: need %zu bytes", gram_workspace_bytes(n, d));
  float* slab = static_cast<float*>(ws);
  if (n > 256) return launch_gram_pairs(X, n, d, ldx, G, slab, s);
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
  SRA_REQUIRE(n >= 1 && n <= sra::kGramMaxClients && d >= 1, SRA_ERR_UNSUPPORTED, "Gram supports 1 <= N <= %d, d >= 1",
              sra::kGramMaxClients);
  *bytes = sra::gram_workspace_bytes(static_cast<int>(n), d);
  return SRA_OK;
}

extern "C" int sra_gram_f32(const float* X, int64_t n, int64_t d, int64_t ldx, double* G, void* ws, size_t ws_bytes,
                            void* stream) {
  SRA_REQUIRE(X != nullptr && G != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx (%lld/%lld)", (long long)d, (long long)ldx);
  return sra::launch_gram(X, static_cast<int>(n), d, ldx, G, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int sra_gram_buckets_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t bucket_size, double* G,
                                    void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(X != nullptr && G != nullptr && ws != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= (int64_t(1) << 30) && d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad shape");
  SRA_REQUIRE(bucket_size >= 1 && bucket_size <= 4 && sra::cdiv(n, bucket_size) <= 32 * sra::kBucketGramMaxNB,
              SRA_ERR_UNSUPPORTED, "bucket Gram: 1 <= bucket size <= 4 and at most %d buckets",
              32 * sra::kBucketGramMaxNB);
  const int nb = static_cast<int>(sra::cdiv(n, bucket_size));
  SRA_REQUIRE(ws_bytes >= sra::gram_workspace_bytes(nb, d), SRA_ERR_WORKSPACE,
              "bucket Gram workspace too small: need %zu bytes", sra::gram_workspace_bytes(nb, d));
  return sra::launch_gram_buckets(X, static_cast<int>(n), bucket_size, d, ldx, G, static_cast<float*>(ws),
                                  static_cast<hipStream_t>(stream));
}
