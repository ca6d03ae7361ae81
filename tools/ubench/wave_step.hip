// Microbenchmark of the round-5 one-wave Lanczos step (csrc/wave_sym.hpp):
// a 128 x 128 symmetric fp64 matrix in circulant-half form held by ONE wave
// (KV diagonals in VGPRs, the rest in LDS), y = C z with wave-local
// reductions only.  Checks y against the host product, then reports cycles
// per plain-Lanczos step (s_memtime, workgroup 0) and ns per step per
// chunk slot at 1 .. 6 waves per CU.  Also measures the dependent-chain
// latency of v_fma_f64 for one wave.
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -I../../secure-robust-federated-learning_amd/csrc wave_step.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#include "wave_sym.hpp"

using namespace sra;

__device__ __forceinline__ double dpp_sum(double v) {
  auto d = [](double x, int ctrl) {
    const long long b = __builtin_bit_cast(long long, x);
    int lo, hi;
    switch (ctrl) {
      case 0: lo = __builtin_amdgcn_mov_dpp((int)b, 0xB1, 0xF, 0xF, false);
              hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0xB1, 0xF, 0xF, false); break;
      case 1: lo = __builtin_amdgcn_mov_dpp((int)b, 0x4E, 0xF, 0xF, false);
              hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x4E, 0xF, 0xF, false); break;
      case 2: lo = __builtin_amdgcn_mov_dpp((int)b, 0x141, 0xF, 0xF, false);
              hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x141, 0xF, 0xF, false); break;
      default: lo = __builtin_amdgcn_mov_dpp((int)b, 0x140, 0xF, 0xF, false);
               hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x140, 0xF, 0xF, false); break;
    }
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
  };
  v += d(v, 0);
  v += d(v, 1);
  v += d(v, 2);
  v += d(v, 3);
  auto rl = [](double x, int l) {
    const long long b = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
  };
  return (rl(v, 0) + rl(v, 16)) + (rl(v, 32) + rl(v, 48));
}

template <int KV>
__global__ void __launch_bounds__(64, 1) wave_step_kernel(const double* C, const double* xin, double* yout, double* out,
                                                          long long* cyc, int steps) {
  constexpr int KL = wsym::NK - KV;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* zd = sm;
  double* tb = zd + wsym::kZd;
  double* cl = tb + wsym::kTb;
  const int lane = threadIdx.x;
  wsym::Packed<KV> P;
  wsym::sfor<wsym::NK>([&](auto K) {
    constexpr int k = decltype(K)::value;
    const int m0 = 2 * lane, m1 = 2 * lane + 1;
    const double v0 = C[m0 * 128 + ((m0 + k) & 127)], v1 = C[m1 * 128 + ((m1 + k) & 127)];
    if constexpr (k < KV) {
      P.cv[k][0] = v0;
      P.cv[k][1] = v1;
    } else {
      cl[(k - KV) * 128 + m0] = v0;
      cl[(k - KV) * 128 + m1] = v1;
    }
  });
  (void)KL;
  // correctness: y = C x
  {
    const double x0 = xin[2 * lane], x1 = xin[2 * lane + 1];
    wsym::put_operand(zd, x0, x1);
    double y0, y1;
    wsym::matvec<KV>(P, cl, zd, tb, x0, x1, y0, y1);
    if (blockIdx.x == 0) {
      yout[2 * lane] = y0;
      yout[2 * lane + 1] = y1;
    }
  }
  // plain Lanczos steps
  double r0 = 1.0 + 0.01 * (2 * lane), r1 = 1.0 + 0.01 * (2 * lane + 1), p0 = 0.0, p1 = 0.0;
  double nrm2 = dpp_sum(r0 * r0 + r1 * r1);
  long long t0 = 0;
  double asum = 0.0;
  for (int j = 0; j < steps; ++j) {
    if (j == 2) t0 = __builtin_amdgcn_s_memtime();
    const double bet = sqrt(nrm2);
    wsym::put_operand(zd, r0, r1);
    double y0, y1;
    wsym::matvec<KV>(P, cl, zd, tb, r0, r1, y0, y1);
    const double ib = 1.0 / bet;
    const double q0 = r0 * ib, q1 = r1 * ib;
    const double m0 = y0 * ib, m1 = y1 * ib;
    const double aj = dpp_sum(q0 * m0 + q1 * m1);
    const double n0 = m0 - aj * q0 - (j > 0 ? bet * p0 : 0.0);
    const double n1 = m1 - aj * q1 - (j > 0 ? bet * p1 : 0.0);
    p0 = q0;
    p1 = q1;
    r0 = n0;
    r1 = n1;
    nrm2 = dpp_sum(r0 * r0 + r1 * r1);
    asum += aj;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[blockIdx.x] = asum;
    if (blockIdx.x == 0) cyc[0] = (t1 - t0) / (steps - 2);
  }
}

// dependent v_fma_f64 chain, one wave
__global__ void fma_chain_kernel(double* out, long long* cyc, int n) {
  double a = threadIdx.x * 1e-3, b = 0.999999, c = 1e-7;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    a = fma(a, b, c);
    a = fma(a, b, c);
    a = fma(a, b, c);
    a = fma(a, b, c);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[1] = (t1 - t0) / (4ll * n);
}

template <int KV>
void run(const double* dC, const double* dx, double* dy, double* dout, long long* dcyc, const std::vector<double>& C,
         const std::vector<double>& x) {
  const size_t lds = sizeof(double) * (wsym::kZd + wsym::kTb + (wsym::NK - KV) * 128);
  hipFuncSetAttribute(reinterpret_cast<const void*>(wave_step_kernel<KV>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  const int steps = 2000;
  for (int grid : {1, 256, 512, 768, 1024, 1280, 1536}) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(wave_step_kernel<KV>, dim3(grid), dim3(64), lds, 0, dC, dx, dy, dout, dcyc, steps);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(wave_step_kernel<KV>, dim3(grid), dim3(64), lds, 0, dC, dx, dy, dout, dcyc, steps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c;
    hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
    std::vector<double> y(128);
    hipMemcpy(y.data(), dy, 128 * 8, hipMemcpyDeviceToHost);
    double err = 0.0, ymax = 0.0;
    for (int i = 0; i < 128; ++i) {
      double s = 0.0;
      for (int j = 0; j < 128; ++j) s += C[i * 128 + j] * x[j];
      err = fmax(err, fabs(s - y[i]));
      ymax = fmax(ymax, fabs(s));
    }
    printf("KV %2d lds %5zu B grid %4d: %lld cyc/step (WG 0), %.3f ms -> %.1f ns per step per CU-slot "
           "(%.1f ns per chunk-step per CU), matvec rel err %.2e\n",
           KV, lds, grid, c, ms, ms * 1e6 / steps, ms * 1e6 / steps / (grid / 256.0 > 1 ? grid / 256.0 : 1), err / ymax);
  }
}

int main() {
  std::vector<double> C(128 * 128), x(128);
  unsigned s = 1;
  for (int i = 0; i < 128; ++i)
    for (int j = 0; j <= i; ++j) {
      s = s * 1664525u + 1013904223u;
      const double v = ((s >> 8) / 16777216.0 - 0.5) * 0.02 + (i == j ? 1.0 : 0.0);
      C[i * 128 + j] = C[j * 128 + i] = v;
    }
  for (int i = 0; i < 128; ++i) {
    s = s * 1664525u + 1013904223u;
    x[i] = (s >> 8) / 16777216.0 - 0.5;
  }
  double *dC, *dx, *dy, *dout;
  long long* dcyc;
  hipMalloc(&dC, C.size() * 8);
  hipMalloc(&dx, 128 * 8);
  hipMalloc(&dy, 128 * 8);
  hipMalloc(&dout, 8192 * 8);
  hipMalloc(&dcyc, 16);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dx, x.data(), 128 * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(fma_chain_kernel, dim3(1), dim3(64), 0, 0, dout, dcyc, 4096);
  hipDeviceSynchronize();
  long long cc[2];
  hipMemcpy(cc, dcyc, 16, hipMemcpyDeviceToHost);
  printf("v_fma_f64 dependent chain, one wave: %lld cycles per fma\n", cc[1]);
  run<32>(dC, dx, dy, dout, dcyc, C, x);
  run<40>(dC, dx, dy, dout, dcyc, C, x);
  run<48>(dC, dx, dy, dout, dcyc, C, x);
  return 0;
}
