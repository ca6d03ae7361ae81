// Issue rates of the candidate building blocks for a full-rate compare-exchange.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 2048

template <int W>
__global__ void kern(float* out, unsigned long long* clk, float k) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (W == 0) {  // 8x (v_cndmask e32 with vcc)
      asm volatile("v_cmp_gt_f32 vcc, %0, %8\n"
                   "v_cndmask_b32 %0, %0, %8, vcc\nv_cndmask_b32 %1, %1, %8, vcc\nv_cndmask_b32 %2, %2, %8, vcc\nv_cndmask_b32 %3, %3, %8, vcc\n"
                   "v_cndmask_b32 %4, %4, %8, vcc\nv_cndmask_b32 %5, %5, %8, vcc\nv_cndmask_b32 %6, %6, %8, vcc\nv_cndmask_b32 %7, %7, %8, vcc\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k) : "vcc");
    } else if constexpr (W == 1) {  // 8x v_cmp into SGPR pairs
      asm volatile("v_cmp_gt_f32 s[20:21], %0, %8\nv_cmp_gt_f32 s[22:23], %1, %8\nv_cmp_gt_f32 s[24:25], %2, %8\nv_cmp_gt_f32 s[26:27], %3, %8\n"
                   "v_cmp_gt_f32 s[28:29], %4, %8\nv_cmp_gt_f32 s[30:31], %5, %8\nv_cmp_gt_f32 s[32:33], %6, %8\nv_cmp_gt_f32 s[34:35], %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k)
                   : "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35");
    } else if constexpr (W == 2) {  // CE via cmp + 2 cndmask (e64, sgpr masks), 4 independent CEs
      asm volatile("v_cmp_gt_f32 s[20:21], %0, %1\nv_cmp_gt_f32 s[22:23], %2, %3\nv_cmp_gt_f32 s[24:25], %4, %5\nv_cmp_gt_f32 s[26:27], %6, %7\n"
                   "v_cndmask_b32 v250, %0, %1, s[20:21]\nv_cndmask_b32 %1, %1, %0, s[20:21]\n"
                   "v_cndmask_b32 v251, %2, %3, s[22:23]\nv_cndmask_b32 %3, %3, %2, s[22:23]\n"
                   "v_cndmask_b32 v252, %4, %5, s[24:25]\nv_cndmask_b32 %5, %5, %4, s[24:25]\n"
                   "v_cndmask_b32 v253, %6, %7, s[26:27]\nv_cndmask_b32 %7, %7, %6, s[26:27]\n"
                   "v_mov_b32 %0, v250\nv_mov_b32 %2, v251\nv_mov_b32 %4, v252\nv_mov_b32 %6, v253\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :
                   : "s20","s21","s22","s23","s24","s25","s26","s27","v250","v251","v252","v253");
    } else if constexpr (W == 3) {  // 8x v_pk_add_f32 (pairs)
      asm volatile("v_pk_add_f32 v[240:241], v[240:241], v[242:243]\nv_pk_add_f32 v[244:245], v[244:245], v[242:243]\n"
                   "v_pk_add_f32 v[246:247], v[246:247], v[242:243]\nv_pk_add_f32 v[248:249], v[248:249], v[242:243]\n"
                   "v_pk_add_f32 v[240:241], v[240:241], v[242:243]\nv_pk_add_f32 v[244:245], v[244:245], v[242:243]\n"
                   "v_pk_add_f32 v[246:247], v[246:247], v[242:243]\nv_pk_add_f32 v[248:249], v[248:249], v[242:243]\n"
                   ::: "v240","v241","v242","v243","v244","v245","v246","v247","v248","v249");
    } else if constexpr (W == 4) {  // 8x v_mov_b32
      asm volatile("v_mov_b32 %0, %8\nv_mov_b32 %1, %8\nv_mov_b32 %2, %8\nv_mov_b32 %3, %8\n"
                   "v_mov_b32 %4, %8\nv_mov_b32 %5, %8\nv_mov_b32 %6, %8\nv_mov_b32 %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 5) {  // 8x v_pk_max_i16
      asm volatile("v_pk_max_i16 %0, %0, %8\nv_pk_max_i16 %1, %1, %8\nv_pk_max_i16 %2, %2, %8\nv_pk_max_i16 %3, %3, %8\n"
                   "v_pk_max_i16 %4, %4, %8\nv_pk_max_i16 %5, %5, %8\nv_pk_max_i16 %6, %6, %8\nv_pk_max_i16 %7, %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 6) {  // 8x v_sub_f32 + v_xor
      asm volatile("v_sub_f32 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_sub_f32 %2, %2, %8\nv_xor_b32 %3, %3, %8\n"
                   "v_sub_f32 %4, %4, %8\nv_and_b32 %5, %5, %8\nv_sub_f32 %6, %6, %8\nv_or_b32 %7, %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 7) {  // 8x v_max_f16 (VOP2 16-bit)
      asm volatile("v_pk_max_f16 %0, %0, %8\nv_pk_max_f16 %1, %1, %8\nv_pk_max_f16 %2, %2, %8\nv_pk_max_f16 %3, %3, %8\n"
                   "v_pk_max_f16 %4, %4, %8\nv_pk_max_f16 %5, %5, %8\nv_pk_max_f16 %6, %6, %8\nv_pk_max_f16 %7, %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 8) {  // 8x v_max_u32 + v_min_u32 (to compare with f32)
      asm volatile("v_max_u32 %0, %0, %8\nv_min_u32 %1, %1, %8\nv_max_u32 %2, %2, %8\nv_min_u32 %3, %3, %8\n"
                   "v_max_u32 %4, %4, %8\nv_min_u32 %5, %5, %8\nv_max_u32 %6, %6, %8\nv_min_u32 %7, %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 9) {  // 8x v_fma_f32
      asm volatile("v_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\n"
                   "v_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int W>
void run(const char* name, int per_iter, int waves_per_simd) {
  const int blocks = 256 * waves_per_simd;
  float* out; unsigned long long* clk;
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipMalloc(&clk, 16);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  kern<W><<<blocks, 256>>>(out, clk, 1.5f);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  kern<W><<<blocks, 256>>>(out, clk, 1.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
  double ghz = (double)c[0] / ((double)c[1] / 100.0) / 1000.0;
  double instr_per_simd = (double)ITER * per_iter * waves_per_simd;
  printf("%-28s w/SIMD=%d %.3f ms %.2f GHz -> %.2f cyc/instr\n", name, waves_per_simd, ms, ghz,
         ms * 1e-3 * ghz * 1e9 / instr_per_simd);
  hipFree(out); hipFree(clk);
}

int main() {
  for (int w : {2, 4}) {
    run<0>("cmp+8 cndmask(vcc)", 9, w);
    run<1>("8 v_cmp -> sgpr", 8, w);
    run<2>("4 CE cmp+2cndmask+mov", 16, w);
    run<3>("v_pk_add_f32", 8, w);
    run<4>("v_mov_b32", 8, w);
    run<5>("v_pk_max_i16", 8, w);
    run<6>("v_sub/xor/and/or", 8, w);
    run<7>("v_pk_max_f16", 8, w);
    run<8>("v_max_u32/v_min_u32", 8, w);
    run<9>("v_fma_f32", 8, w);
  }
  return 0;
}
