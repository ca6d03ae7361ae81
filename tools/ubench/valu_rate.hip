// VALU issue-rate microbenchmark for the k-select compare-exchange ops on gfx950.
// Each thread runs ITER iterations of 16 independent ops (8 chains x 2) in
// inline asm; we report wave-instructions per SIMD per ns and implied cycles
// per instruction at the measured clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 4096

#define BODY(OP)                                                                     \
  for (int it = 0; it < ITER; ++it) {                                                \
    asm volatile(OP " %0, %0, %8\n" OP " %1, %1, %8\n" OP " %2, %2, %8\n" OP " %3, %3, %8\n" \
                 OP " %4, %4, %8\n" OP " %5, %5, %8\n" OP " %6, %6, %8\n" OP " %7, %7, %8\n" \
                 OP " %0, %0, %8\n" OP " %1, %1, %8\n" OP " %2, %2, %8\n" OP " %3, %3, %8\n" \
                 OP " %4, %4, %8\n" OP " %5, %5, %8\n" OP " %6, %6, %8\n" OP " %7, %7, %8\n" \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k)); \
  }
#define BODY3(OP)                                                                     \
  for (int it = 0; it < ITER; ++it) {                                                \
    asm volatile(OP " %0, %0, %8, %8\n" OP " %1, %1, %8, %8\n" OP " %2, %2, %8, %8\n" OP " %3, %3, %8, %8\n" \
                 OP " %4, %4, %8, %8\n" OP " %5, %5, %8, %8\n" OP " %6, %6, %8, %8\n" OP " %7, %7, %8, %8\n" \
                 OP " %0, %0, %8, %8\n" OP " %1, %1, %8, %8\n" OP " %2, %2, %8, %8\n" OP " %3, %3, %8, %8\n" \
                 OP " %4, %4, %8, %8\n" OP " %5, %5, %8, %8\n" OP " %6, %6, %8, %8\n" OP " %7, %7, %8, %8\n" \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k)); \
  }

template <int W>
__global__ void kern(float* out, unsigned long long* clk, float k) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (W == 0) { BODY("v_min_f32") }
  if constexpr (W == 1) { BODY3("v_minimum3_f32") }
  if constexpr (W == 2) { BODY("v_add_f32") }
  if constexpr (W == 3) { BODY3("v_min3_f32") }
  if constexpr (W == 4) { BODY3("v_med3_f32") }
  if constexpr (W == 5) { BODY("v_min_i32") }
  if constexpr (W == 6) { BODY3("v_maximum3_f32") }
  if constexpr (W == 7) {   // fp64 FMA (the spectral-filter solver's matvec)
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7, dk = k;
    for (int it = 0; it < ITER; ++it) {
      asm volatile("v_fma_f64 %0, %0, %8, %8\nv_fma_f64 %1, %1, %8, %8\nv_fma_f64 %2, %2, %8, %8\nv_fma_f64 %3, %3, %8, %8\n"
                   "v_fma_f64 %4, %4, %8, %8\nv_fma_f64 %5, %5, %8, %8\nv_fma_f64 %6, %6, %8, %8\nv_fma_f64 %7, %7, %8, %8\n"
                   "v_fma_f64 %0, %0, %8, %8\nv_fma_f64 %1, %1, %8, %8\nv_fma_f64 %2, %2, %8, %8\nv_fma_f64 %3, %3, %8, %8\n"
                   "v_fma_f64 %4, %4, %8, %8\nv_fma_f64 %5, %5, %8, %8\nv_fma_f64 %6, %6, %8, %8\nv_fma_f64 %7, %7, %8, %8\n"
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "v"(dk));
    }
    a0 = (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int W>
void run(const char* name, int waves_per_simd) {
  const int blocks = 256 * waves_per_simd;  // 256-thread blocks = 1 wave per SIMD each
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
  double ghz = (double)c[0] / ((double)c[1] / 100.0) / 1000.0;  // memrealtime = 100 MHz
  double instr_per_simd = (double)ITER * 16 * waves_per_simd;
  double cyc = ms * 1e-3 * ghz * 1e9 / instr_per_simd;
  printf("%-16s waves/SIMD=%d  %.3f ms  clock %.2f GHz  -> %.2f cycles per wave-instruction per SIMD\n", name,
         waves_per_simd, ms, ghz, cyc);
  hipFree(out); hipFree(clk);
}

int main() {
  for (int w : {1, 2, 4, 8}) {
    run<0>("v_min_f32", w);
    run<1>("v_minimum3_f32", w);
    run<6>("v_maximum3_f32", w);
    run<2>("v_add_f32", w);
    run<3>("v_min3_f32", w);
    run<4>("v_med3_f32", w);
    run<5>("v_min_i32", w);
    run<7>("v_fma_f64", w);
  }
  return 0;
}
