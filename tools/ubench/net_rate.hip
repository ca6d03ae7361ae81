// The north-star trimmed-mean network (sort4 blocks + pruned odd-even merges
// for N = 128, kept ranks [12, 116)) on register-resident columns, no memory
// traffic: cycles per 64-coordinate tile for each compare-exchange form of
// network_plain (csrc/sra_common.hpp, CEF 0 / 1) at 1 and 2 waves per SIMD.
// Round 6 (one box): 12,149-12,333 vs 11,954-11,992 cycles per tile at two
// waves (a plan group's mins issued before its xors: 11,869-11,877).
// build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -I../../include net_rate.hip -o bin/net_rate
#include "../../secure-robust-federated-learning_amd/csrc/sra_common.hpp"

#include <cstdio>

using namespace sra;
constexpr int ITER = 64;

template <int CEF>
__global__ void __launch_bounds__(256) kern(const float* __restrict__ in, float* out, unsigned long long* clk) {
  float v[128];
  const int t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 128; ++i) v[i] = in[(i * 977 + t) & 65535];
  float acc = 0.f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 128; ++i) asm volatile("" : "+v"(v[i]));
    sort4_blocks<128>(v);
    network_plain<128, 128, 12, 116, kNetFrom4, CEF>(v);
    float s = 0.f;
#pragma unroll
    for (int p = 12; p < 116; ++p) s += v[p];
    acc += s;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[t] = acc;
  if (t == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int CEF>
void run(const char* name, int waves_per_simd, const float* in) {
  const int blocks = 256 * waves_per_simd;
  float* out; unsigned long long* clk;
  (void)hipMalloc(&out, sizeof(float) * blocks * 256);
  (void)hipMalloc(&clk, 16);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  kern<CEF><<<blocks, 256>>>(in, out, clk);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  kern<CEF><<<blocks, 256>>>(in, out, clk);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c[2]; (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
  double ghz = (double)c[0] / ((double)c[1] / 100.0) / 1000.0;
  // tiles per SIMD: blocks * 4 waves / 1024 SIMDs * ITER
  double tiles_per_simd = (double)blocks * 4 / 1024 * ITER;
  printf("%-26s w/SIMD=%d %.3f ms %.2f GHz -> %.0f cycles per tile\n", name, waves_per_simd, ms, ghz,
         ms * 1e-3 * ghz * 1e9 / tiles_per_simd);
  (void)hipFree(out); (void)hipFree(clk);
}

int main() {
  float* in; (void)hipMalloc(&in, 65536 * 4);
  float h[65536];
  for (int i = 0; i < 65536; ++i) h[i] = (float)((i * 2654435761u) % 100003) * 1e-3f;
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep)
    for (int w : {1, 2}) {
      run<0>("min+max (VOP2)", w, in);
      run<1>("min+bitop3", w, in);
    }
  return 0;
}
