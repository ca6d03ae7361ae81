// k2 -- the software-pipelined bf16x3 Gram for N = 128 (the C3 shape), in its
// own file: it is built without SLP vectorisation (Makefile), since packed f32
// VALU between MFMAs costs ~13 cycles more per instruction than two scalar
// ops, while the other Gram kernels (eight waves per CU for N > 128) run
// faster with the packed forms.  Same arithmetic and slab layout as
// gram_partial_kernel<4, 4, VEC, 0, 1, true> (gram.hip); reduced by the same
// gram_reduce kernels.
#include "gram_common.hpp"

namespace sra {

// Software-pipelined Gram for N = 128 (NB = 4, four waves, the C3 shape).
// Same arithmetic as gram_body<4, 4, VEC, 0, 1, true> (per-wave means from a
// fixed butterfly, the exact three-way split, six bf16 MFMAs per tile and
// k-step, tiles accumulated in the same k order), scheduled so that the MFMA
// pipe is never left idle while the wave does its VALU work: each of the 60
// MFMAs of a k-step is followed by one small piece of the NEXT k-step's
// preparation (its LDS reads, the column sums and butterfly, the centring and
// split of one element pair) or of the stage traffic, pinned in place by
// sched_barrier.  (Rounds 3-4 staged each 128-coordinate stage through 64
// VGPRs of register loads and a ds_write pass, one stage in flight per CU;
// round 5 replaced that with the LDS-DMA ring below, bit-identical.)
struct GramOps {
  bf16x8 h[4], m[4], l[4];
};

// ---- round 5: the same pipeline with LDS-DMA staging ----------------------
// global_load_lds_dwordx4 writes a stage straight into LDS (no VGPR landing
// zone, no ds_write pass), so the stage is halved to 64 coordinates (32 KiB)
// and FOUR buffers rotate: the loads of stage t + 3 are issued while stage t's
// MFMAs run and stage t + 1 is prepared, i.e. two to three stages (64-96 KiB
// per CU) are in flight instead of one 64 KiB stage.  One k-step per wave per
// stage; a block walks the same coordinates in the same order as the 128-wide
// pipe (64-stage t = half t & 1 of 128-stage t >> 1), so every wave
// accumulates the same k-steps in the same order: the Gram is bit-identical
// to the register-staged kernel it replaced.
//
// LDS image: lane-linear per instruction (64 lanes x 16 B = four 256-byte
// rows), the 16-byte chunks of row r XOR-swizzled by r & 15 (conflict-free
// ds_read_b128 of 16 rows); each lane loads the source chunk that lands on its
// linear slot (the same involution on both sides).
//
// Ordering: a DMA is a pending LDS write on the VM counter.  After issuing
// stage t + 3, each wave waits vmcnt(8) (its 8 DMAs of stage t + 2 retired,
// t + 3 still in flight) and then a raw s_barrier, so stage t + 2 is complete
// for every wave before phase t + 1 prepares it; stage t + 3's buffer last
// held stage t - 1, read in phase t - 2.
constexpr int kGldsStage = 64;
constexpr int kGldsBuf = 128 * kGldsStage;   // floats per buffer
__device__ __forceinline__ void gram_body_glds(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                               float* __restrict__ slab, float* lds) {
  using C = GramCfg<4, 4, 0>;
  constexpr int T = C::T;   // 10
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int kg = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: the DMA row-block bases in SGPRs
  const int64_t ntiles = d / 128;
  const int nstage = blockIdx.x < ntiles ? static_cast<int>(cdiv(ntiles - blockIdx.x, gridDim.x)) : 0;
  const int nst = 2 * nstage;   // 64-wide stages
  const float inv_n = 1.0f / static_cast<float>(n);
  const int r = lane & 31;
  const int h = lane >> 5;

  f32x16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;

  auto bufp = [&](int t) { return lds + (t & 3) * kGldsBuf; };
  // coordinate base of 64-stage t (clamped: past the end the DMAs re-read the
  // last stage into a buffer nobody reads)
  auto stage_k = [&](int t) -> int64_t {
    const int tc = t < nst ? t : nst - 1;
    return (static_cast<int64_t>(tc >> 1) * gridDim.x + blockIdx.x) * 128 + (tc & 1) * kGldsStage;
  };
  // DMA q (0..7) of this wave: rows 4 rb .. 4 rb + 3, rb = 8 kg + q; lane L
  // fills row 4 rb + L / 16, linear chunk L % 16 <- source chunk
  // (L % 16) ^ (row & 15), and row & 15 = 4 (q & 3) + L / 16
  uint32_t goff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rl = lane >> 4;
    const int c4 = (lane & 15) ^ (4 * q + rl);
    goff[q] = static_cast<uint32_t>((static_cast<int64_t>(rl) * ldx + 4 * c4) * 4);
  }
  auto dma = [&](int t, int q) {
    const int rb = 8 * kg + q;
    const char* src = reinterpret_cast<const char*>(X + static_cast<int64_t>(4 * rb) * ldx + stage_k(t));
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    __builtin_amdgcn_global_load_lds((gvoid*)(src + goff[q & 3]), (lvoid*)(bufp(t) + rb * 256), 16, 0, 0);
  };
  // this lane's two swizzled chunks of its k-step (16 kg + 8 h .. + 7)
  const int sw = r & 15;
  const int offa = 4 * ((4 * kg + 2 * h) ^ sw), offb = 4 * ((4 * kg + 2 * h + 1) ^ sw);

  f32x4 raw0[4], raw1[4], mu0, mu1;
  auto prep_piece = [&](auto pc, const float* b, GramOps& o) {
    constexpr int p = decltype(pc)::value;
    if constexpr (p < 4) {
      const float* rp = b + (32 * p + r) * kGldsStage;
      raw0[p] = *reinterpret_cast<const f32x4*>(rp + offa);
      raw1[p] = *reinterpret_cast<const f32x4*>(rp + offb);
    } else if constexpr (p == 4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) mu0[e] = ((raw0[0][e] + raw0[1][e]) + raw0[2][e]) + raw0[3][e];
    } else if constexpr (p == 5) {
#pragma unroll
      for (int e = 0; e < 4; ++e) mu1[e] = ((raw1[0][e] + raw1[1][e]) + raw1[2][e]) + raw1[3][e];
    } else if constexpr (p < 26) {
      constexpr int q = p - 6;
      constexpr int lvl = q / 4;
      constexpr int v0 = 2 * (q % 4);
#pragma unroll
      for (int vv = v0; vv < v0 + 2; ++vv) {
        float x = vv < 4 ? mu0[vv] : mu1[vv - 4];
        int xi = __builtin_bit_cast(int, x);
        int yi;
        if constexpr (lvl == 0) yi = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);
        else if constexpr (lvl == 1) yi = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);
        else if constexpr (lvl == 2) yi = __builtin_amdgcn_ds_swizzle(xi, 0x101f);
        else if constexpr (lvl == 3) yi = __builtin_amdgcn_ds_swizzle(xi, 0x201f);
        else yi = __builtin_amdgcn_ds_swizzle(xi, 0x401f);
        x += __builtin_bit_cast(float, yi);
        if (vv < 4) mu0[vv] = x; else mu1[vv - 4] = x;
      }
    } else if constexpr (p == 26) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mu0[e] = mu0[e] * inv_n;
        mu1[e] = mu1[e] * inv_n;
      }
    } else if constexpr (p < 43) {
      constexpr int blk = (p - 27) / 4;
      constexpr int e2 = (p - 27) % 4;
      float x0 = e2 < 2 ? raw0[blk][2 * e2] - mu0[2 * e2] : raw1[blk][2 * e2 - 4] - mu1[2 * e2 - 4];
      float x1 = e2 < 2 ? raw0[blk][2 * e2 + 1] - mu0[2 * e2 + 1] : raw1[blk][2 * e2 - 3] - mu1[2 * e2 - 3];
      uint32_t hb, mb, lb;
      split3_pair(x0, x1, hb, mb, lb);
      set_pair(o.h[blk], e2, hb);
      set_pair(o.m[blk], e2, mb);
      set_pair(o.l[blk], e2, lb);
    }
  };
  auto mfma_slot = [&](auto ic, const GramOps& o) {
    constexpr int i = decltype(ic)::value;
    constexpr int t = i / 6, term = i % 6;
    constexpr int ti = C::kTileI(t), tj = C::kTileJ(t);
    if constexpr (term == 0) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.h[ti], o.h[tj], acc[t], 0, 0, 0);
    if constexpr (term == 1) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.h[ti], o.m[tj], acc[t], 0, 0, 0);
    if constexpr (term == 2) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.m[ti], o.h[tj], acc[t], 0, 0, 0);
    if constexpr (term == 3) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.h[ti], o.l[tj], acc[t], 0, 0, 0);
    if constexpr (term == 4) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.l[ti], o.h[tj], acc[t], 0, 0, 0);
    if constexpr (term == 5) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.m[ti], o.m[tj], acc[t], 0, 0, 0);
  };
  auto sync_stage = [&]() {   // this wave's DMAs of the stage two ahead retired, then every wave's
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  GramOps opA, opB;
  if (nst > 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(1, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(2, q);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // stages 0 and 1 landed (this wave's part)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    static_for<0, 43>([&](auto pc) { prep_piece(pc, bufp(0), opA); });
  }
  // phase t: MFMAs of stage t | prepare stage t + 1 | DMAs of stage t + 3
  auto phase = [&](int t, const GramOps& cur, GramOps& nxt) {
    const float* b = bufp(t + 1);
    static_for<0, 60>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      mfma_slot(ic, cur);
      if constexpr (i < 43) prep_piece(ic, b, nxt);
      else if constexpr (i < 51) dma(t + 3, i - 43);
      __builtin_amdgcn_sched_barrier(0);
    });
    sync_stage();
  };
  for (int t = 0; t < nst; t += 2) {
    phase(t, opA, opB);
    phase(t + 1, opB, opA);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing re-read DMAs land before the block ends

  float* my = slab + (static_cast<int64_t>(blockIdx.x) * C::WK + kg) * T * 1024;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    float* o = my + t * 1024;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
      o[row * 32 + r] = acc[t][reg];
    }
  }
}

__global__ void __launch_bounds__(256) gram_glds_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                        float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  gram_body_glds(X, n, d, ldx, slab, lds);
}

int launch_gram_pipe(const float* X, int n, int64_t d, int64_t ldx, float* slab, int nwg, hipStream_t s) {
  using C = GramCfg<4, 4, 0>;
  SRA_REQUIRE(n == 128 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 && d % C::STAGE == 0,
              SRA_ERR_ARG, "pipelined Gram needs N == 128, aligned rows and d %% %d == 0", C::STAGE);
  SRA_REQUIRE(gram_pipe_offsets_fit(ldx), SRA_ERR_ARG,
              "pipelined Gram: the 32-bit lane offsets cannot address rows %lld floats apart", (long long)ldx);
  const size_t lds = sizeof(float) * 4 * kGldsBuf;
  SRA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gram_glds_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  hipLaunchKernelGGL(gram_glds_kernel, dim3(nwg), dim3(256), lds, s, X, n, d, ldx, slab);
  return SRA_OK;
}

}  // namespace sra
