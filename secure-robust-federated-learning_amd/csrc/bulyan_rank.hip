// k4 rounds without a sort per round: persistent per-coordinate ranks.
//
// Bulyan's median / trimmed-mean selection (src/robust_estimator.py:297-322)
// runs theta rounds; round t aggregates the N - t remaining clients
// coordinate-wise (np.median / the sorted window's sequential fp32 mean) and
// removes the client nearest to that aggregate.  Removing one client changes
// each coordinate's sorted order by deleting one entry, so the order is kept
// instead of rebuilt: rank[i][k] (uint8, clients x coordinates) is client i's
// position in coordinate k's ascending order among the remaining clients (NaN
// last, ties by client index, the order np.sort's output takes up to equal
// values, which the aggregates cannot tell apart).
//
//   rank_init_kernel: one sort of every column's order-preserving keys, then
//     each client's rank by binary search in the sorted keys (ties by index).
//   rank_round_kernel: per 256-coordinate tile, one lane per coordinate, every
//     remaining row is loaded ONCE (x in registers, its rank byte); the ranks
//     drop by one above the previous round's removed client (r > r*) and are
//     stored back; the aggregate is the value of rank (m-1)/2 (or the mean of
//     ranks m/2 - 1, m/2) -- the median -- or the sequential fp32 sum of the
//     values of ranks [lo, hi) in rank order (scattered to a per-wave LDS slot
//     array, 64 ranks per pass) -- the trimmed mean / the DBA lower median;
//     then the squared distances of the remaining rows to it from the SAME
//     registers, with select_dist_rows_kernel's arithmetic (LDS transpose,
//     fp32 chains per 32-coordinate half, waves in order, fp32 across a
//     block's tiles), so the rounds' aggregates and distances are the bits the
//     sorting kernel produces.
// Per round: 4 bytes per remaining value read once + 2 rank bytes (read and
// write) against the sorting kernel's two reads of every value, and a few
// VALU operations per value instead of a compare-exchange network.
#include "sra_common.hpp"

namespace sra {

namespace {

__device__ __forceinline__ const char* uniform_ptr_r(const char* p) {
  const uint64_t r = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r >> 32));
  return reinterpret_cast<const char*>((static_cast<uint64_t>(hi) << 32) | lo);
}

typedef const __attribute__((address_space(1))) float gfloat_c;
typedef const __attribute__((address_space(1))) uint8_t gbyte_c;
typedef __attribute__((address_space(1))) uint8_t gbyte;

// ascending float order as unsigned keys; every NaN after +inf
__device__ __forceinline__ uint32_t order_key(float x) {
  const uint32_t b = __builtin_bit_cast(uint32_t, x);
  if (x != x) return 0xffffffffu;
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// bitonic sort of u32 keys in registers, ascending; every index compile-time
template <int P2, int KK, int J>
__device__ __forceinline__ void bitonic_pass(uint32_t (&key)[P2]) {
#pragma unroll
  for (int i = 0; i < P2; ++i) {
    const int l = i ^ J;
    if (l > i) {
      const uint32_t a = key[i], b = key[l];
      const uint32_t mn = a < b ? a : b, mx = a < b ? b : a;
      const bool up = (i & KK) == 0;
      key[i] = up ? mn : mx;
      key[l] = up ? mx : mn;
    }
  }
  if constexpr (J > 1) bitonic_pass<P2, KK, J / 2>(key);
}

template <int P2, int KK>
__device__ __forceinline__ void bitonic_stage(uint32_t (&key)[P2]) {
  bitonic_pass<P2, KK, KK / 2>(key);
  if constexpr (KK < P2) bitonic_stage<P2, KK * 2>(key);
}

}  // namespace

// ---------------------------------------------------------------------------
// initial ranks: n <= P2 <= 128 clients, one wave (64 coordinates) per block.
// The column's order keys are sorted in registers (u32 min / max network),
// stored to this wave's LDS, and each client takes lower_bound(its key) plus
// the number of earlier clients with the same key (a per-position counter in
// LDS, clients visited in index order): ascending order, ties by index.
// ---------------------------------------------------------------------------
template <int P2>
__global__ void __launch_bounds__(64) rank_init_kernel(const float* __restrict__ X, int64_t ldx, int n, int64_t d,
                                                       uint8_t* __restrict__ ranks) {
  __shared__ uint32_t sk[P2][64];
  __shared__ uint8_t cnt[P2][64];
  const int t = threadIdx.x;
  const int64_t k = static_cast<int64_t>(blockIdx.x) * 64 + t;
  const int64_t kc = k < d ? k : d - 1;
  uint32_t key[P2];
#pragma unroll
  for (int i = 0; i < P2; ++i) {
    key[i] = i < n ? order_key(X[static_cast<int64_t>(i) * ldx + kc]) : 0xffffffffu;
    cnt[i][t] = 0;
  }
  bitonic_stage<P2, 2>(key);
#pragma unroll
  for (int p = 0; p < P2; ++p) sk[p][t] = key[p];
  for (int i = 0; i < n; ++i) {
    const uint32_t ki = order_key(X[static_cast<int64_t>(i) * ldx + kc]);
    int lb = 0;
#pragma unroll
    for (int step = P2 / 2; step >= 1; step >>= 1)
      if (sk[lb + step - 1][t] < ki) lb += step;
    const int c = cnt[lb][t];
    cnt[lb][t] = static_cast<uint8_t>(c + 1);
    if (k < d) ranks[static_cast<int64_t>(i) * d + k] = static_cast<uint8_t>(lb + c);
  }
}

// ---------------------------------------------------------------------------
// one round over the listed rows (n in (P - 16, P], P <= 128)
// ---------------------------------------------------------------------------
template <int P, int MODE>   // MODE 0: median; 1: the sequential mean of ranks [lo, hi)
__global__ void __launch_bounds__(256, 2) rank_round_kernel(const float* __restrict__ X, int64_t ldx,
                                                            const int* __restrict__ rows, int nrows_x, int n_arg,
                                                            int64_t d, int lo, int hi, uint8_t* __restrict__ ranks,
                                                            const int* __restrict__ picked, float* __restrict__ out,
                                                            float* __restrict__ bpart, int nb, int tpb) {
  constexpr int RW = (P + 63) / 64;
  constexpr int CH = 64;                     // window ranks per scatter pass
  constexpr int WREG = MODE == 1 ? CH * 64 : 32 * 68;   // per-wave LDS floats: slots, or the distance tile
  __shared__ float lds[4 * (WREG > 32 * 68 ? WREG : 32 * 68)];
  __shared__ float wsum[4][P];
  const unsigned t = threadIdx.x;
  const unsigned lane = t & 63u;
  const unsigned w = t >> 6;
  constexpr int WSTRIDE = WREG > 32 * 68 ? WREG : 32 * 68;
  float* wl = lds + w * WSTRIDE;   // this wave's private LDS region
  int rl[RW];
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int li = 64 * q + static_cast<int>(lane);
    rl[q] = rows[li < n_arg ? li : n_arg - 1];
  }
  // the previous round's removed client (none before the first round)
  const int removed = picked != nullptr ? checked_row(*picked, nrows_x) : -1;
  float bs = 0.f;
  const int64_t ntiles = cdiv(d, 256);
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * tpb;
  const int64_t t1 = t0 + tpb < ntiles ? t0 + tpb : ntiles;
  for (int64_t tile = t0; tile < t1; ++tile) {
    const int64_t base = tile * 256;
    const int64_t rem = d - base;
    const unsigned last = rem < 256 ? static_cast<unsigned>(rem - 1) : 255u;
    const unsigned tc = t < last ? t : last;
    const bool valid = t < rem;
#pragma unroll
    for (int q = 0; q < RW; ++q) asm volatile("" : "+v"(rl[q]));
    int n = n_arg;
    asm volatile("" : "+s"(n));
    int rstar = 255;   // ranks above it drop by one
    if (removed >= 0) {
      const char* rp = uniform_ptr_r(reinterpret_cast<const char*>(ranks + static_cast<int64_t>(removed) * d + base));
      rstar = *reinterpret_cast<gbyte_c*>(reinterpret_cast<uint64_t>(rp) + tc);
    }
    float v[P];
    uint32_t pk[(P + 3) / 4];   // the updated ranks, four per register (MODE 1)
    float sel0 = 0.f, sel1 = 0.f, top = 0.f;
    const int m = n;
    const int p0 = MODE == 0 ? ((m & 1) ? (m - 1) / 2 : m / 2 - 1) : 0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (i < n) {
        const int row = checked_row(__builtin_amdgcn_readlane(rl[i / 64], i % 64), nrows_x);
        const char* xp = uniform_ptr_r(reinterpret_cast<const char*>(X + static_cast<int64_t>(row) * ldx + base));
        const char* rp = uniform_ptr_r(reinterpret_cast<const char*>(ranks + static_cast<int64_t>(row) * d + base));
        const float x = *reinterpret_cast<gfloat_c*>(reinterpret_cast<uint64_t>(xp) + 4u * tc);
        int r = *reinterpret_cast<gbyte_c*>(reinterpret_cast<uint64_t>(rp) + tc);
        __builtin_amdgcn_sched_barrier(0);
        r -= r > rstar ? 1 : 0;
        if (removed >= 0 && valid) *reinterpret_cast<gbyte*>(reinterpret_cast<uint64_t>(rp) + tc) = static_cast<uint8_t>(r);
        v[i] = x;
        if constexpr (MODE == 0) {
          sel0 = r == p0 ? x : sel0;
          sel1 = r == p0 + 1 ? x : sel1;
          top = r == m - 1 ? x : top;
        } else {
          if ((i & 3) == 0) pk[i / 4] = static_cast<uint32_t>(r);
          else pk[i / 4] |= static_cast<uint32_t>(r) << (8 * (i & 3));
        }
      } else {
        v[i] = 0.f;
      }
    }
    float res;
    if constexpr (MODE == 0) {
      res = (m & 1) ? sel0 : (sel0 + sel1) * 0.5f;
      if (top != top) res = qnan();   // NaN ranks last: one NaN anywhere -> np.median is NaN
    } else {
      int lo_t = lo, hi_t = hi;
      asm volatile("" : "+s"(lo_t), "+s"(hi_t));
      const int W = hi_t - lo_t;
      float acc = 0.f;
      for (int c0 = 0; c0 < W; c0 += CH) {   // wave-uniform
        const int wc = W - c0 < CH ? W - c0 : CH;
#pragma unroll
        for (int i = 0; i < P; ++i) {
          if (i < n) {
            const int r = static_cast<int>((pk[i / 4] >> (8 * (i & 3))) & 0xffu);
            const unsigned q = static_cast<unsigned>(r - lo_t - c0);
            if (q < static_cast<unsigned>(wc)) wl[q * 64 + lane] = v[i];
          }
        }
        for (int q = 0; q < wc; ++q) acc += wl[q * 64 + lane];   // ascending rank order
      }
      res = acc / static_cast<float>(W);
    }
    if (valid) out[base + t] = res;
    // squared distances over this wave's 64 coordinates: select_dist_rows_kernel's
    // arithmetic (32-row chunks through an LDS tile read transposed)
    const unsigned ti = lane & 31u, th = lane >> 5;
    float* dl = wl;   // [32][68], this wave's region
#pragma unroll
    for (int c = 0; c < RW * 2; ++c) {
      if (32 * c >= n) break;   // wave-uniform
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();   // every lane done with the slot array / the previous chunk's reads
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        if (32 * c + i < P) dl[i * 68 + lane] = res - v[32 * c + i];
      }
      if (rem < 256 && !valid) {
#pragma unroll
        for (int i = 0; i < 32; ++i) dl[i * 68 + lane] = 0.f;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float sh = 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(&dl[ti * 68 + 32 * th + 4 * u]);
        sh = __builtin_fmaf(q[0], q[0], sh);
        sh = __builtin_fmaf(q[1], q[1], sh);
        sh = __builtin_fmaf(q[2], q[2], sh);
        sh = __builtin_fmaf(q[3], q[3], sh);
      }
      const float so = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(static_cast<int>((lane ^ 32u) * 4u),
                                                                              __builtin_bit_cast(int, sh)));
      const float st = th == 0 ? sh + so : so + sh;
      if (th == 0 && 32 * c + static_cast<int>(ti) < n) wsum[w][32 * c + ti] = st;
    }
    __syncthreads();
    if (static_cast<int>(t) < n) bs += (wsum[0][t] + wsum[1][t]) + (wsum[2][t] + wsum[3][t]);
    __syncthreads();
  }
  if (static_cast<int>(t) < n_arg) bpart[static_cast<int64_t>(t) * nb + blockIdx.x] = bs;
}

int launch_rank_init(const float* X, int64_t ldx, int n, int64_t d, uint8_t* ranks, hipStream_t s) {
  SRA_REQUIRE(n >= 1 && n <= 128, SRA_ERR_UNSUPPORTED, "rank rounds: N <= 128 (got %d)", n);
  const dim3 g(static_cast<unsigned>(cdiv(d, 64)));
  if (n <= 32) hipLaunchKernelGGL(rank_init_kernel<32>, g, dim3(64), 0, s, X, ldx, n, d, ranks);
  else if (n <= 64) hipLaunchKernelGGL(rank_init_kernel<64>, g, dim3(64), 0, s, X, ldx, n, d, ranks);
  else hipLaunchKernelGGL(rank_init_kernel<128>, g, dim3(64), 0, s, X, ldx, n, d, ranks);
  return launch_status("rank_init_kernel");
}

int launch_rank_round(const float* X, int64_t ldx, const int* rows, int nrows_x, int n, int64_t d, bool median,
                      int lo, int hi, uint8_t* ranks, const int* picked, float* out, float* bpart, int nb, int tpb,
                      hipStream_t s) {
  const int P = static_cast<int>(cdiv(n, 16) * 16);
#define SRA_RR(PP)                                                                                              \
  case PP:                                                                                                      \
    if (median)                                                                                                 \
      hipLaunchKernelGGL((rank_round_kernel<PP, 0>), dim3(nb), dim3(256), 0, s, X, ldx, rows, nrows_x, n, d, lo, \
                         hi, ranks, picked, out, bpart, nb, tpb);                                              \
    else                                                                                                        \
      hipLaunchKernelGGL((rank_round_kernel<PP, 1>), dim3(nb), dim3(256), 0, s, X, ldx, rows, nrows_x, n, d, lo, \
                         hi, ranks, picked, out, bpart, nb, tpb);                                              \
    return launch_status("rank_round_kernel");
  switch (P) {
    SRA_RR(16) SRA_RR(32) SRA_RR(48) SRA_RR(64) SRA_RR(80) SRA_RR(96) SRA_RR(112) SRA_RR(128)
    default: break;
  }
#undef SRA_RR
  set_error("rank rounds support N <= 128 (got %d)", n);
  return SRA_ERR_UNSUPPORTED;
}

}  // namespace sra
