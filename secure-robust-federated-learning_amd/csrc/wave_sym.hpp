// One-wave symmetric matrix-vector product for the spectral-filter solver
// (k6, round 5).  A 128 x 128 symmetric fp64 matrix C (the chunk's centred
// client Gram, client space) is held by ONE wave in circulant-half form:
// lane l owns rows m = 2l (slot 0) and 2l + 1 (slot 1) and, for each
// diagonal offset k = 0 .. 64, the entry C[m][(m + k) mod 128].  Every entry
// of the upper half is stored once (k = 64 twice: C[m][m+64] = C[m+64][m]),
// 130 doubles per lane against 256 for whole rows, so a chunk fits one wave
// (the first KV diagonals in VGPRs, the other 65 - KV in LDS) and the
// filter's reductions are wave-local (DPP), never a workgroup barrier.
//
//   y_m = sum_{k=0}^{64} C[m][m+k] z_{m+k}            ("a" part)
//       + sum_{k=1}^{63} C[m-k][m] z_{m-k}            ("b" part, transposed)
//
// a part: z doubled in LDS (zd[i] = z_{i mod 128}, 256 entries); lane l reads
// (z_{2l+2j}, z_{2l+2j+1}) with one ds_read_b128 per j = 0 .. 32 and takes
// both slots' terms of k = 2j and 2j + 1 from it (slot 1 of an odd k uses the
// next read).
// b part: b_k = C[m][m+k] z_m belongs to row m + k, i.e. S = sum_k D^k b_k
// with D the shift by one row (row m takes row m - 1).  In this layout
// D(v0, v1) = (ror1(v1), v0): ONE cross-lane double (two v_mov_b32_dpp
// wave_ror:1, lane 0 takes lane 63 = the circulant wrap), so S is evaluated
// by Horner's rule in four independent groups of 16 diagonals (k descending),
// and the groups' results are shifted by 16 g rows through LDS.
#pragma once
#include <utility>

namespace sra {
namespace wsym {

constexpr int NP = 128;
constexpr int NK = 65;   // diagonals 0 .. 64

template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<0>), ..., f(integral_constant<N-1>), fully unrolled
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// Compiler-level ordering of one wave's LDS traffic.  A lane reads slots that
// OTHER lanes of the same wave wrote: the hardware runs a wave's LDS
// instructions in order, but the compiler reasons per thread, sees different
// addresses and may hoist the read above the write (wave_barrier is no memory
// fence).  Every cross-lane LDS hand-off of the one-wave solver goes through
// this.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// lane l + 1's value (lane 63 takes lane 0): DPP wave_rol:1
__device__ __forceinline__ double rol1(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b), 0x134, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), 0x134, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// lane l - 1's value (lane 0 takes lane 63)
__device__ __forceinline__ double ror1(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b), 0x13C, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), 0x13C, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// LDS words of one wave's operator scratch besides the matrix part:
// zd [256] doubled operand, tb [3][128] group shifts
constexpr int kZd = 2 * NP;
constexpr int kTb = 3 * NP;

// Packed storage of diagonal k in LDS: cl[(k - KV) * NP + m] for m = 2l + s
template <int KV>
struct Packed {
  static constexpr int KL = NK - KV;
  double cv[KV][2];
};

// C[m][(m+k) mod 128] of diagonal k for this lane's two rows
template <int KV, int K>
__device__ __forceinline__ double2 diag(const Packed<KV>& P, const double* __restrict__ cl, int lane) {
  if constexpr (K < KV) return double2{P.cv[K][0], P.cv[K][1]};
  else return reinterpret_cast<const double2*>(cl + (K - KV) * NP)[lane];
}

// y = C z.  zd: LDS [256], z doubled, already written (this wave); z0, z1 the
// lane's own entries; tb: LDS scratch [3][128]; cl: LDS part of C.
template <int KV>
__device__ __forceinline__ void matvec(const Packed<KV>& P, const double* __restrict__ cl, const double* zd,
                                       double* tb, double z0, double z1, double& y0, double& y1) {
  const int lane = threadIdx.x & 63;
  const double2* xp = reinterpret_cast<const double2*>(zd) + lane;   // xp[j] = (z_{2l+2j}, z_{2l+2j+1})
  double a[4][2];
  double h[4][2];
  // operand window of each group: xw[g][0] = X_j, xw[g][1] = X_{j+1} for the
  // group's current diagonal k (j = k / 2); every X is one aligned b128 read
  double2 xw[4][2];
  {
    const double2 c0 = diag<KV, 0>(P, cl, lane);
    a[0][0] = c0.x * z0;
    a[0][1] = c0.y * z1;
    a[1][0] = a[1][1] = a[2][0] = a[2][1] = a[3][0] = a[3][1] = 0.0;
  }
  // round r takes k = 16 g + 16 - r of every group g (k descending inside a group)
  sfor<16>([&](auto R) {
    constexpr int r = decltype(R)::value;
    sfor<4>([&](auto Gi) {
      constexpr int g = decltype(Gi)::value;
      constexpr int k = 16 * g + 16 - r;
      constexpr int j = k / 2;
      const double2 c = diag<KV, k>(P, cl, lane);
      // ---- a part: k even uses X_j; k odd uses X_j.y and X_{j+1}.x.  Going
      // down, an odd k loads X_j (X_{j+1} is the previous round's), the even
      // k = 2j that follows reuses it; a group's first k loads what it needs.
      if constexpr (r == 0) {
        xw[g][0] = xp[j];
        if constexpr (k & 1) xw[g][1] = xp[j + 1];
      } else if constexpr (k & 1) {
        xw[g][1] = xw[g][0];
        xw[g][0] = xp[j];
      }
      if constexpr ((k & 1) == 0) {
        a[g][0] = fma(c.x, xw[g][0].x, a[g][0]);
        a[g][1] = fma(c.y, xw[g][0].y, a[g][1]);
      } else {
        a[g][0] = fma(c.x, xw[g][0].y, a[g][0]);
        a[g][1] = fma(c.y, xw[g][1].x, a[g][1]);
      }
      // ---- b part (k <= 63), Horner from the group's top diagonal down
      if constexpr (k <= 63) {
        constexpr int ktop = 16 * g + 16 < 63 ? 16 * g + 16 : 63;
        if constexpr (k == ktop) {
          h[g][0] = c.x * z0;
          h[g][1] = c.y * z1;
        } else {
          const double t = ror1(h[g][1]);
          const double n1 = fma(c.y, z1, h[g][0]);
          h[g][0] = fma(c.x, z0, t);
          h[g][1] = n1;
        }
      }
    });
  });
  // group g's contribution is D^{16 g + 1} h_g: one D here, 16 g rows (8 g
  // lanes) through LDS
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
  y0 = ((a[0][0] + a[1][0]) + (a[2][0] + a[3][0])) + s0;
  y1 = ((a[0][1] + a[1][1]) + (a[2][1] + a[3][1])) + s1;
}

// Write this lane's rows of z into the doubled operand buffer.
__device__ __forceinline__ void put_operand(double* zd, double z0, double z1) {
  const int lane = threadIdx.x & 63;
  lds_order();   // after every earlier cross-lane read of the buffer
  reinterpret_cast<double2*>(zd)[lane] = double2{z0, z1};
  reinterpret_cast<double2*>(zd + NP)[lane] = double2{z0, z1};
  lds_order();
}

}  // namespace wsym
}  // namespace sra
