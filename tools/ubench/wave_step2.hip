// Variants of the one-wave matvec (csrc/wave_sym.hpp) measured inside the
// plain-Lanczos step of wave_step.hip: V = 0 the production matvec; V = 1 the
// b part's one-row rotation through ds_bpermute (the LDS crossbar) instead of
// two v_mov_b32_dpp per double; V = 2 the a part in eight accumulators per
// slot instead of four (more independent fma chains for one wave per SIMD).
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -I../../secure-robust-federated-learning_amd/csrc wave_step2.hip
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

namespace v2 {
using namespace sra::wsym;
__device__ __forceinline__ double ror1_bp(double v, int addr) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(b));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(b >> 32));
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
template <int KV, int V>
__device__ __forceinline__ void matvec(const Packed<KV>& P, const double* __restrict__ cl, const double* zd,
                                       double* tb, double z0, double z1, double& y0, double& y1) {
  const int lane = threadIdx.x & 63;
  const int addr = ((lane + 63) & 63) * 4;   // ds_bpermute source lane l - 1
  const double2* xp = reinterpret_cast<const double2*>(zd) + lane;
  constexpr int NA = V == 2 ? 2 : 1;          // accumulators per group and slot
  double a[4][NA][2];
  double h[4][2];
  double2 xw[4][2];
  {
    const double2 c0 = diag<KV, 0>(P, cl, lane);
    for (int g = 0; g < 4; ++g)
      for (int q = 0; q < NA; ++q) a[g][q][0] = a[g][q][1] = 0.0;
    a[0][0][0] = c0.x * z0;
    a[0][0][1] = c0.y * z1;
  }
  sfor<16>([&](auto R) {
    constexpr int r = decltype(R)::value;
    constexpr int q = NA == 2 ? (r & 1) : 0;
    sfor<4>([&](auto Gi) {
      constexpr int g = decltype(Gi)::value;
      constexpr int k = 16 * g + 16 - r;
      constexpr int j = k / 2;
      const double2 c = diag<KV, k>(P, cl, lane);
      if constexpr (r == 0) {
        xw[g][0] = xp[j];
        if constexpr (k & 1) xw[g][1] = xp[j + 1];
      } else if constexpr (k & 1) {
        xw[g][1] = xw[g][0];
        xw[g][0] = xp[j];
      }
      if constexpr ((k & 1) == 0) {
        a[g][q][0] = fma(c.x, xw[g][0].x, a[g][q][0]);
        a[g][q][1] = fma(c.y, xw[g][0].y, a[g][q][1]);
      } else {
        a[g][q][0] = fma(c.x, xw[g][0].y, a[g][q][0]);
        a[g][q][1] = fma(c.y, xw[g][1].x, a[g][q][1]);
      }
      if constexpr (k <= 63) {
        constexpr int ktop = 16 * g + 16 < 63 ? 16 * g + 16 : 63;
        if constexpr (k == ktop) {
          h[g][0] = c.x * z0;
          h[g][1] = c.y * z1;
        } else {
          const double t = V == 1 ? ror1_bp(h[g][1], addr) : ror1(h[g][1]);
          const double n1 = fma(c.y, z1, h[g][0]);
          h[g][0] = fma(c.x, z0, t);
          h[g][1] = n1;
        }
      }
    });
  });
  double s0 = 0.0, s1 = 0.0;
  sfor<4>([&](auto Gi) {
    constexpr int g = decltype(Gi)::value;
    const double d0 = ror1(h[g][1]), d1 = h[g][0];
    if constexpr (g == 0) {
      s0 = d0;
      s1 = d1;
    } else {
      reinterpret_cast<double2*>(tb + (g - 1) * NP)[(lane + 8 * g) & 63] = double2{d0, d1};
    }
  });
  lds_order();
  sfor<3>([&](auto Gi) {
    constexpr int g = decltype(Gi)::value;
    const double2 v = reinterpret_cast<const double2*>(tb + g * NP)[lane];
    s0 += v.x;
    s1 += v.y;
  });
  double b0[4], b1[4];
  for (int g = 0; g < 4; ++g) {
    b0[g] = NA == 2 ? a[g][0][0] + a[g][NA - 1][0] : a[g][0][0];
    b1[g] = NA == 2 ? a[g][0][1] + a[g][NA - 1][1] : a[g][0][1];
  }
  y0 = ((b0[0] + b0[1]) + (b0[2] + b0[3])) + s0;
  y1 = ((b1[0] + b1[1]) + (b1[2] + b1[3])) + s1;
}
}  // namespace v2

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

template <int KV, int V>
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
    v2::matvec<KV, V>(P, cl, zd, tb, x0, x1, y0, y1);
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
    v2::matvec<KV, V>(P, cl, zd, tb, r0, r1, y0, y1);
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

template <int KV, int V>
void run(const double* dC, const double* dx, double* dy, double* dout, long long* dcyc, const std::vector<double>& C,
         const std::vector<double>& x) {
  const size_t lds = sizeof(double) * (wsym::kZd + wsym::kTb + (wsym::NK - KV) * 128);
  hipFuncSetAttribute(reinterpret_cast<const void*>(wave_step_kernel<KV, V>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  const int steps = 2000;
  for (int grid : {1, 1024}) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((wave_step_kernel<KV, V>), dim3(grid), dim3(64), lds, 0, dC, dx, dy, dout, dcyc, steps);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL((wave_step_kernel<KV, V>), dim3(grid), dim3(64), lds, 0, dC, dx, dy, dout, dcyc, steps);
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
    printf("V %d KV %2d lds %5zu B grid %4d: %lld cyc/step (WG 0), %.3f ms -> %.1f ns per step per CU-slot "
           "(%.1f ns per chunk-step per CU), matvec rel err %.2e\n",
           V, KV, lds, grid, c, ms, ms * 1e6 / steps, ms * 1e6 / steps / (grid / 256.0 > 1 ? grid / 256.0 : 1), err / ymax);
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
  for (int rep = 0; rep < 2; ++rep) {
    run<36, 0>(dC, dx, dy, dout, dcyc, C, x);
    run<36, 1>(dC, dx, dy, dout, dcyc, C, x);
    run<36, 2>(dC, dx, dy, dout, dcyc, C, x);
  }
  return 0;
}
