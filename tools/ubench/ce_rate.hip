// Issue rate of compare-exchange forms on gfx950: v_min_f32 + v_max_f32 (the
// network today) against v_min_f32 + v_bitop3_b32 (the max recovered as
// a ^ b ^ min: min returns one of its operands bit for bit, so the xor of all
// three is the other one), and the bitwise op on its own.
// build: hipcc -O3 --offload-arch=gfx950 ce_rate.hip -o bin/ce_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 2048

template <int W>
__global__ void kern(float* out, unsigned long long* clk, float k) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (W == 0) {  // 4 CEs: v_min_f32 + v_max_f32 (VOP2 pair, lo into a temp)
      float l0, l1, l2, l3;
      asm volatile("v_min_f32 %0, %4, %5\nv_max_f32 %5, %4, %5\n"
                   "v_min_f32 %1, %6, %7\nv_max_f32 %7, %6, %7\n"
                   "v_min_f32 %2, %8, %9\nv_max_f32 %9, %8, %9\n"
                   "v_min_f32 %3, %10, %11\nv_max_f32 %11, %10, %11\n"
                   : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3), "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4),
                     "+v"(a5), "+v"(a6), "+v"(a7));
      a0 = l3; a2 = l0; a4 = l1; a6 = l2;
    } else if constexpr (W == 1) {  // 4 CEs: v_min_f32 + v_bitop3_b32 (xor3)
      float l0, l1, l2, l3;
      asm volatile("v_min_f32 %0, %4, %5\nv_bitop3_b32 %5, %4, %5, %0 bitop3:0x96\n"
                   "v_min_f32 %1, %6, %7\nv_bitop3_b32 %7, %6, %7, %1 bitop3:0x96\n"
                   "v_min_f32 %2, %8, %9\nv_bitop3_b32 %9, %8, %9, %2 bitop3:0x96\n"
                   "v_min_f32 %3, %10, %11\nv_bitop3_b32 %11, %10, %11, %3 bitop3:0x96\n"
                   : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3), "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4),
                     "+v"(a5), "+v"(a6), "+v"(a7));
      a0 = l3; a2 = l0; a4 = l1; a6 = l2;
    } else if constexpr (W == 2) {  // 8x v_bitop3_b32
      asm volatile("v_bitop3_b32 %0, %0, %8, %1 bitop3:0x96\nv_bitop3_b32 %1, %1, %8, %2 bitop3:0x96\n"
                   "v_bitop3_b32 %2, %2, %8, %3 bitop3:0x96\nv_bitop3_b32 %3, %3, %8, %4 bitop3:0x96\n"
                   "v_bitop3_b32 %4, %4, %8, %5 bitop3:0x96\nv_bitop3_b32 %5, %5, %8, %6 bitop3:0x96\n"
                   "v_bitop3_b32 %6, %6, %8, %7 bitop3:0x96\nv_bitop3_b32 %7, %7, %8, %0 bitop3:0x96\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 3) {  // 8x v_xor_b32 (VOP2)
      asm volatile("v_xor_b32 %0, %0, %8\nv_xor_b32 %1, %1, %8\nv_xor_b32 %2, %2, %8\nv_xor_b32 %3, %3, %8\n"
                   "v_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %8\nv_xor_b32 %6, %6, %8\nv_xor_b32 %7, %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 4) {  // 8x v_min_f32
      asm volatile("v_min_f32 %0, %0, %8\nv_min_f32 %1, %1, %8\nv_min_f32 %2, %2, %8\nv_min_f32 %3, %3, %8\n"
                   "v_min_f32 %4, %4, %8\nv_min_f32 %5, %5, %8\nv_min_f32 %6, %6, %8\nv_min_f32 %7, %7, %8\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 5) {  // 8x v_xad_u32 (VOP3 xor-add)
      asm volatile("v_xad_u32 %0, %0, %8, %1\nv_xad_u32 %1, %1, %8, %2\nv_xad_u32 %2, %2, %8, %3\nv_xad_u32 %3, %3, %8, %4\n"
                   "v_xad_u32 %4, %4, %8, %5\nv_xad_u32 %5, %5, %8, %6\nv_xad_u32 %6, %6, %8, %7\nv_xad_u32 %7, %7, %8, %0\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (W == 6) {  // 4 CEs: v_min_f32 + 2 v_xor_b32 (VOP2)
      float l0, l1, l2, l3, t0, t1, t2, t3;
      asm volatile("v_min_f32 %0, %8, %9\nv_xor_b32 %4, %8, %9\nv_xor_b32 %9, %4, %0\n"
                   "v_min_f32 %1, %10, %11\nv_xor_b32 %5, %10, %11\nv_xor_b32 %11, %5, %1\n"
                   "v_min_f32 %2, %12, %13\nv_xor_b32 %6, %12, %13\nv_xor_b32 %13, %6, %2\n"
                   "v_min_f32 %3, %14, %15\nv_xor_b32 %7, %14, %15\nv_xor_b32 %15, %7, %3\n"
                   : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3),
                     "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      a0 = l3; a2 = l0; a4 = l1; a6 = l2;
    } else if constexpr (W == 7) {  // 4 CEs: v_min_f32 + v_sub_u32(v_add_u32) mix -- min + max3-free: min3/med3 pair
      float l0, l1, l2, l3;
      asm volatile("v_min3_f32 %0, %4, %5, %6\nv_med3_f32 %5, %4, %5, %6\n"
                   "v_min3_f32 %1, %6, %7, %8\nv_med3_f32 %7, %6, %7, %8\n"
                   "v_min3_f32 %2, %8, %9, %10\nv_med3_f32 %9, %8, %9, %10\n"
                   "v_min3_f32 %3, %10, %11, %4\nv_med3_f32 %11, %10, %11, %4\n"
                   : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3), "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4),
                     "+v"(a5), "+v"(a6), "+v"(a7));
      a0 = l3; a2 = l0; a4 = l1; a6 = l2;
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
  printf("%-32s w/SIMD=%d %.3f ms %.2f GHz -> %.2f cyc/instr\n", name, waves_per_simd, ms, ghz,
         ms * 1e-3 * ghz * 1e9 / instr_per_simd);
  hipFree(out); hipFree(clk);
}

int main() {
  for (int w : {1, 2, 4}) {
    run<0>("4 CE min+max", 8, w);
    run<1>("4 CE min+bitop3(xor3)", 8, w);
    run<6>("4 CE min+2 xor", 12, w);
    run<2>("v_bitop3_b32", 8, w);
    run<3>("v_xor_b32", 8, w);
    run<4>("v_min_f32", 8, w);
    run<5>("v_xad_u32", 8, w);
    run<7>("min3+med3 pairs", 8, w);
  }
  return 0;
}
