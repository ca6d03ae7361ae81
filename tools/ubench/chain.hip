// Latency of one serial fp64 recurrence step g' = fma(x - a_k, g, -b_k * g0) on
// gfx950, one wave alone, by where the per-step coefficients (a_k, b_k) come from:
//   V0 constants in VGPRs (pure dependency chain);
//   V1 v_readlane from a register-resident table (lane k holds a_k, b_k);
//   V2 LDS broadcast loads (every lane reads the same address) issued 4 ahead;
//   V3 V1 unrolled by 8 with the readlanes of the next 8 steps issued first.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double rl(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), l);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

template <int V>
__global__ void chain(double* out, long long* cyc, int steps) {
  __shared__ double2 tab[64 + 8];
  const int lane = threadIdx.x;
  const double a = 1.0 + 1e-3 * lane, b = 0.25 + 1e-4 * lane;
  tab[lane] = make_double2(a, b);
  if (lane < 8) tab[64 + lane] = make_double2(a, b);
  __syncthreads();
  const double x = 1.5 + 1e-6 * lane;
  double g1 = 1.0, g0 = 0.5;
  long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (V == 0) {
    for (int k = 0; k < steps; ++k) {
      const double gn = fma(x - a, g1, -(b * g0));
      g0 = g1;
      g1 = gn * 0.5;
    }
  } else if constexpr (V == 1) {
    for (int k = 0; k < steps; ++k) {
      const double gn = fma(x - rl(a, k & 63), g1, -(rl(b, k & 63) * g0));
      g0 = g1;
      g1 = gn * 0.5;
    }
  } else if constexpr (V == 2) {
    double2 c0 = tab[0], c1 = tab[1], c2 = tab[2], c3 = tab[3];
    for (int k = 0; k < steps; k += 4) {
      const int q = (k + 4) & 63;
      const double2 n0 = tab[q], n1 = tab[q + 1], n2 = tab[q + 2], n3 = tab[q + 3];
      double gn = fma(x - c0.x, g1, -(c0.y * g0)); g0 = g1; g1 = gn * 0.5;
      gn = fma(x - c1.x, g1, -(c1.y * g0)); g0 = g1; g1 = gn * 0.5;
      gn = fma(x - c2.x, g1, -(c2.y * g0)); g0 = g1; g1 = gn * 0.5;
      gn = fma(x - c3.x, g1, -(c3.y * g0)); g0 = g1; g1 = gn * 0.5;
      c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
  } else {
    for (int k = 0; k < steps; k += 8) {
      double ca[8], cb[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        ca[t] = x - rl(a, (k + t) & 63);
        cb[t] = rl(b, (k + t) & 63);
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const double gn = fma(ca[t], g1, -(cb[t] * g0));
        g0 = g1;
        g1 = gn * 0.5;
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = g1;
  if (lane == 0) cyc[0] = (t1 - t0) / steps;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8);
  const char* names[4] = {"VGPR constants", "v_readlane per step", "LDS broadcast, 4 ahead", "readlane x8 batched"};
  for (int v = 0; v < 4; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      if (v == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, out, cyc, 4096);
      if (v == 1) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, out, cyc, 4096);
      if (v == 2) hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, out, cyc, 4096);
      if (v == 3) hipLaunchKernelGGL(chain<3>, dim3(1), dim3(64), 0, 0, out, cyc, 4096);
      hipDeviceSynchronize();
    }
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-26s %lld cycles per step\n", names[v], c);
  }
  return 0;
}
