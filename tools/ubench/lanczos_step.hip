// Microbenchmark of one plain-Lanczos step of the spectral-filter solver on a
// 128 x 128 fp64 matrix held in registers by one 256-thread workgroup:
//   V0: lane pair per row (row = tid / 2, half = tid & 1), x broadcast from LDS
//       by 32 ds_read_b128 per lane (the round-2 lanczos_solve_kernel gmv);
//   V1: row halves in lanes l and l + 32 of a wave, each lane loads 4 x values
//       (2 ds_read_b128) and the matvec takes x by v_fmac_f64_dpp row_newbcast
//       (no per-element LDS traffic); halves combined by v_permlane32_swap.
// Both then run the step's two block reductions (alpha, |r|^2) and the vector
// update exactly like the solver.  Reports cycles per step (s_memtime on
// workgroup 0) alone on the chip and with 2 workgroups per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), l);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  v += dpp_f64<0x140>(v);
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}
__device__ __forceinline__ double swap32(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const auto lo = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(b), static_cast<unsigned>(b), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(b >> 32), static_cast<unsigned>(b >> 32),
                                                   false, false);
  const bool up = (threadIdx.x & 63) >= 32;
  const unsigned l = up ? lo[0] : lo[1], h = up ? hi[0] : hi[1];
  return __builtin_bit_cast(double, (static_cast<unsigned long long>(h) << 32) | l);
}

#define FMAC_DPP(K, J) \
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #K " row_mask:0xf bank_mask:0xf" \
               : "+v"(acc[J]) : "v"(xr[J]), "v"(g[4 * K + J]))

template <int V>
__global__ void __launch_bounds__(256, 2) step_kernel(const double* G, double* out, long long* cyc, int steps) {
  __shared__ __attribute__((aligned(16))) double xbuf[136];
  __shared__ double red[2][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = V == 0 ? tid >> 1 : 32 * wave + (lane & 31);
  const int half = V == 0 ? tid & 1 : lane >> 5;
  const bool own = half == 0;
  double g[64];
  for (int c = 0; c < 64; ++c) g[c] = G[row * 128 + 64 * half + c];
  int rslot = 0;
  auto reduce = [&](double v) -> double {
    v = wave_sum(v);
    double* R = red[rslot];
    if (lane == 0) R[wave] = v;
    __syncthreads();
    rslot ^= 1;
    return (R[0] + R[1]) + (R[2] + R[3]);
  };
  auto gmv = [&]() -> double {
    if constexpr (V == 0) {
      const double2* xh = reinterpret_cast<const double2*>(xbuf + 64 * half);
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
      for (int c = 0; c < 32; c += 2) {
        const double2 a = xh[c], b = xh[c + 1];
        p0 = fma(g[2 * c], a.x, p0);
        p1 = fma(g[2 * c + 1], a.y, p1);
        p2 = fma(g[2 * c + 2], b.x, p2);
        p3 = fma(g[2 * c + 3], b.y, p3);
        if ((c & 6) == 6) asm volatile("" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)::"memory");
      }
      const double p = (p0 + p1) + (p2 + p3);
      return p + dpp_f64<0xB1>(p);
    } else {
      const double2* xp = reinterpret_cast<const double2*>(xbuf + 64 * half + 4 * (lane & 15));
      const double2 a = xp[0], b = xp[1];
      double xr[4] = {a.x, a.y, b.x, b.y};
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      FMAC_DPP(0, 0); FMAC_DPP(0, 1); FMAC_DPP(0, 2); FMAC_DPP(0, 3);
      FMAC_DPP(1, 0); FMAC_DPP(1, 1); FMAC_DPP(1, 2); FMAC_DPP(1, 3);
      FMAC_DPP(2, 0); FMAC_DPP(2, 1); FMAC_DPP(2, 2); FMAC_DPP(2, 3);
      FMAC_DPP(3, 0); FMAC_DPP(3, 1); FMAC_DPP(3, 2); FMAC_DPP(3, 3);
      FMAC_DPP(4, 0); FMAC_DPP(4, 1); FMAC_DPP(4, 2); FMAC_DPP(4, 3);
      FMAC_DPP(5, 0); FMAC_DPP(5, 1); FMAC_DPP(5, 2); FMAC_DPP(5, 3);
      FMAC_DPP(6, 0); FMAC_DPP(6, 1); FMAC_DPP(6, 2); FMAC_DPP(6, 3);
      FMAC_DPP(7, 0); FMAC_DPP(7, 1); FMAC_DPP(7, 2); FMAC_DPP(7, 3);
      FMAC_DPP(8, 0); FMAC_DPP(8, 1); FMAC_DPP(8, 2); FMAC_DPP(8, 3);
      FMAC_DPP(9, 0); FMAC_DPP(9, 1); FMAC_DPP(9, 2); FMAC_DPP(9, 3);
      FMAC_DPP(10, 0); FMAC_DPP(10, 1); FMAC_DPP(10, 2); FMAC_DPP(10, 3);
      FMAC_DPP(11, 0); FMAC_DPP(11, 1); FMAC_DPP(11, 2); FMAC_DPP(11, 3);
      FMAC_DPP(12, 0); FMAC_DPP(12, 1); FMAC_DPP(12, 2); FMAC_DPP(12, 3);
      FMAC_DPP(13, 0); FMAC_DPP(13, 1); FMAC_DPP(13, 2); FMAC_DPP(13, 3);
      FMAC_DPP(14, 0); FMAC_DPP(14, 1); FMAC_DPP(14, 2); FMAC_DPP(14, 3);
      FMAC_DPP(15, 0); FMAC_DPP(15, 1); FMAC_DPP(15, 2); FMAC_DPP(15, 3);
      const double p = (acc[0] + acc[1]) + (acc[2] + acc[3]);
      return p + swap32(p);
    }
  };
  const int xi = row;
  double rt = 1.0 + 0.01 * row, qprev = 0.0, nrm2 = 0.0;
  if (own) xbuf[xi] = rt;
  nrm2 = reduce(own ? rt * rt : 0.0);
  long long t0 = 0;
  double asum = 0.0;
  for (int j = 0; j < steps; ++j) {
    if (j == 2) t0 = __builtin_amdgcn_s_memtime();
    const double bet = sqrt(nrm2);
    const double y = gmv();
    const double ib = 1.0 / bet;
    const double q = rt * ib;
    const double mq = y * ib;
    const double aj = reduce(own ? q * mq : 0.0);
    const double r = mq - aj * q - (j > 0 ? bet * qprev : 0.0);
    qprev = q;
    rt = r;
    if (own) xbuf[xi] = r;
    nrm2 = reduce(own ? r * r : 0.0);
    asum += aj;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) {
    out[blockIdx.x] = asum;
    if (blockIdx.x == 0) cyc[0] = (t1 - t0) / (steps - 2);
  }
}

int main() {
  std::vector<double> h(128 * 128);
  unsigned s = 1;
  for (int i = 0; i < 128; ++i)
    for (int j = 0; j <= i; ++j) {
      s = s * 1664525u + 1013904223u;
      const double v = ((s >> 8) / 16777216.0 - 0.5) * 0.02 + (i == j ? 1.0 : 0.0);
      h[i * 128 + j] = h[j * 128 + i] = v;
    }
  double *G, *out;
  long long* cyc;
  hipMalloc(&G, h.size() * 8);
  hipMalloc(&out, 4096 * 8);
  hipMalloc(&cyc, 8);
  hipMemcpy(G, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  const int steps = 2000;
  for (int grid : {1, 256, 512, 768}) {
    for (int v = 0; v < 2; ++v) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      auto launch = [&]() {
        if (v == 0) hipLaunchKernelGGL(step_kernel<0>, dim3(grid), dim3(256), 0, 0, G, out, cyc, steps);
        else hipLaunchKernelGGL(step_kernel<1>, dim3(grid), dim3(256), 0, 0, G, out, cyc, steps);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      long long c;
      double o;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      hipMemcpy(&o, out, 8, hipMemcpyDeviceToHost);
      printf("V%d grid %4d: %lld cycles/step (WG 0), %.3f ms -> %.1f ns per step per WG-slot (alpha sum %.6f)\n", v,
             grid, c, ms, ms * 1e6 / steps, o);
    }
  }
  return 0;
}
