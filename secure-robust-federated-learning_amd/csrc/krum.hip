// k3 — Krum scoring in client space (N x N), from the centred Gram of k2.
//
// Replaces the O(N^2 d) Python double loop of krum_ (src/robust_estimator.py:
// 234-244), krum's argmin (:246-249) and the theta selection rounds of
// bulyan(aggsubfunc='krum') (:286-296), which call krum on the remaining set
// with f fixed and delete the chosen client by identity.
//
//   d_ij  = fp32(sqrt(max(G_ii + G_jj - 2 G_ij, 0)))      (fp64 arithmetic)
//   score = numpy pairwise fp32 sum of the m smallest d_ij, j != i, j alive,
//           in ascending order, m = Python-slice count of (n_alive - f - 2)
//   pick  = first index (in client order) of the minimum score
//
// Each row is sorted once (bitonic in LDS, ties by j); a round then compacts
// the first m alive entries of each row and reduces them in numpy's order, so
// a theta-round Bulyan-Krum costs theta * N^2 instead of theta * N^2 log N.
// Everything runs in one workgroup: N-space work is microseconds and needs no
// host synchronisation between rounds.
#include "gram_common.hpp"

namespace sra {

constexpr int kMaxClients = 512;

// numpy's pairwise summation (numpy/_core/src/umath/loops_utils.h.src) for
// float32, n elements at a[0..n): < 8 sequential from 0; <= 128 eight
// accumulators then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail;
// otherwise split at n/2 rounded down to a multiple of 8 (wave_pairwise_f32).

// distance matrix (fp32) from the fp64 Gram.  A non-finite diagonal entry
// means a NaN / inf somewhere in the data (the centring spreads it over every
// entry): *nonfinite is set and the exact per-pair route below takes over.
// acc (n x n fp64) and cls (n x n int32 class bits), optional, are zeroed for
// that route.
__global__ void krum_dist_kernel(const double* __restrict__ G, int n, float* __restrict__ D, int* __restrict__ nonfinite,
                                 double* __restrict__ acc, int* __restrict__ cls) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * n) return;
  const int i = e / n, j = e - (e / n) * n;
  double sq = G[(int64_t)i * n + i] + G[(int64_t)j * n + j] - 2.0 * G[e];
  if (i == j) {
    if (nonfinite != nullptr && !__builtin_isfinite(G[e])) atomicOr(nonfinite, 1);
    sq = 0.0;
  }
  // a squared distance near fp32's range: the reference's fp32 norm overflows
  if (nonfinite != nullptr && sq > 3.0e38) atomicOr(nonfinite, 1);
  if (acc != nullptr) {
    acc[e] = 0.0;
    cls[e] = 0;
  }
  D[e] = static_cast<float>(sqrt(sq > 0.0 ? sq : 0.0));
}

// The exact route for data with NaN / inf (or fp32-overflowing distances):
// acc[i][j] (i < j) = sum_k fp32(x_ik - x_jk)^2 in fp64 -- the reference's
// np.linalg.norm of the fp32 difference (robust_estimator.py:242), whose NaN /
// inf classes (a NaN anywhere, inf - inf = NaN, inf - finite = inf) IEEE
// arithmetic reproduces; the pair's fp32 distance is sqrt(fp32(acc)).  Runs
// only when krum_dist_kernel flagged the Gram (every block exits at once
// otherwise).  Grid: (32 x 32 row-tile pairs I <= J) x d-slices; each thread
// owns 4 pairs of its tile pair.  Finite fp64 partials are added atomically;
// a NaN / inf partial only sets its pair's class bit (1 NaN, 2 inf) -- the
// class of a sum of non-negative squares is NaN if any term is, else inf if
// any term is -- so no special value ever goes through the float atomic.
constexpr int kDirTile = 32;
constexpr int kDirK = 64;
constexpr int64_t kExactMaxD = 1024;
// element k of row i of the matrix Krum scores: X itself (bs == 1), or the
// mean of the bucket of clients [i*bs, min((i+1)*bs, nx)) with bucket.hip's
// expression (mom_krum's fused route, which never writes the bucket means)
__device__ __forceinline__ float row_value(const float* __restrict__ X, int64_t ldx, int nx, int bs, int i,
                                           int64_t k) {
  if (bs == 1) return X[static_cast<int64_t>(i) * ldx + k];
  const int lo = i * bs;
  const int hi = lo + bs < nx ? lo + bs : nx;
  float acc = 0.f;
  for (int q = lo; q < hi; ++q) acc += X[static_cast<int64_t>(q) * ldx + k];
  return acc / static_cast<float>(hi - lo);
}

__global__ void __launch_bounds__(256) krum_direct_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                          int nx, int bs, const int* __restrict__ nonfinite,
                                                          double* __restrict__ acc, int* __restrict__ cls,
                                                          int nslices) {
  if (*nonfinite == 0) return;
  __shared__ float ta[kDirTile][kDirK + 1];
  __shared__ float tb[kDirTile][kDirK + 1];
  const int nt = static_cast<int>(cdiv(n, kDirTile));
  int I = 0, rem = blockIdx.y;
  while (rem >= nt - I) { rem -= nt - I; ++I; }
  const int J = I + rem;
  const int tid = threadIdx.x;
  const int ti = tid >> 3;              // row of tile I
  const int tj = (tid & 7) * 4;         // first of 4 rows of tile J
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t per = cdiv(cdiv(d, kDirK), nslices) * kDirK;
  const int64_t k0 = static_cast<int64_t>(blockIdx.x) * per;
  const int64_t k1 = k0 + per < d ? k0 + per : d;
  for (int64_t kb = k0; kb < k1; kb += kDirK) {
    for (int e = tid; e < kDirTile * kDirK; e += 256) {
      const int r = e / kDirK, c = e % kDirK;
      const int64_t k = kb + c;
      const int ra = I * kDirTile + r, rb = J * kDirTile + r;
      ta[r][c] = (ra < n && k < k1) ? row_value(X, ldx, nx, bs, ra, k) : 0.f;
      tb[r][c] = (rb < n && k < k1) ? row_value(X, ldx, nx, bs, rb, k) : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int c = 0; c < kDirK; ++c) {
      const float a = ta[ti][c];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double df = static_cast<double>(a - tb[tj + q][c]);   // the fp32 difference, squared in fp64
        s[q] = fma(df, df, s[q]);
      }
    }
    __syncthreads();
  }
  const int i = I * kDirTile + ti;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = J * kDirTile + tj + q;
    if (i < n && j < n && (I < J || i < j)) {
      const int64_t e = static_cast<int64_t>(i) * n + j;
      if (s[q] != s[q]) atomicOr(&cls[e], 1);
      else if (__builtin_isinf(s[q])) atomicOr(&cls[e], 2);
      else if (s[q] != 0.0) atomicAdd(&acc[e], s[q]);
    }
  }
}

// Sort every row's off-diagonal distances ascending (ties by j): one workgroup
// per row, bitonic network in LDS over next_pow2(n-1) slots.  With the exact
// route flagged, the distances come from acc instead of D.
// Dynamic LDS: next_pow2(n - 1) (value, index) pairs, at most 64 KiB.
__global__ void __launch_bounds__(256) krum_rowsort_kernel(const float* __restrict__ D, int n,
                                                           float* __restrict__ S, int* __restrict__ J,
                                                           const int* __restrict__ nonfinite,
                                                           const double* __restrict__ acc,
                                                           const int* __restrict__ cls) {
  extern __shared__ __attribute__((aligned(16))) char rs_smem[];
  const int i = blockIdx.x;
  const int m = n - 1;
  const bool direct = nonfinite != nullptr && *nonfinite != 0;
  int pn = 1;
  while (pn < m) pn <<= 1;
  float* kv = reinterpret_cast<float*>(rs_smem);
  int* kj = reinterpret_cast<int*>(kv + pn);
  for (int p = threadIdx.x; p < pn; p += blockDim.x) {
    if (p < m) {
      const int j = p < i ? p : p + 1;
      if (direct) {
        const int64_t e = i < j ? (int64_t)i * n + j : (int64_t)j * n + i;
        // (cls == nullptr: acc is class-coded itself, NaN / inf in place --
        // the sharded route's summed partials, launch_krum_from_pairs)
        const int c = cls != nullptr ? cls[e] : 0;
        // np.sqrt of the fp32 squared norm (inf on fp32 overflow)
        kv[p] = (c & 1) ? __builtin_nanf("") : (c & 2) ? __builtin_inff() : sqrtf(static_cast<float>(acc[e]));
      } else {
        kv[p] = D[(int64_t)i * n + j];
      }
      kj[p] = j;
    } else {
      kv[p] = __builtin_inff();
      kj[p] = 0x7fffffff;
    }
  }
  __syncthreads();
  for (int k = 2; k <= pn; k <<= 1) {
    for (int s = k >> 1; s > 0; s >>= 1) {
      for (int h = threadIdx.x; h < pn / 2; h += blockDim.x) {
        const int a = (h / s) * (2 * s) + (h % s);
        const int b = a + s;
        const bool up = (a & k) == 0;
        const float va = kv[a], vb = kv[b];
        const int ja = kj[a], jb = kj[b];
        // order (class, value, j): numbers ascending (inf included), then NaN
        // (argsort's NaN-last), then the padding slots (j = INT_MAX)
        const int ca = ja == 0x7fffffff ? 2 : (va != va ? 1 : 0);
        const int cb = jb == 0x7fffffff ? 2 : (vb != vb ? 1 : 0);
        const bool a_gt = ca != cb ? ca > cb : (ca == 0 ? (va > vb || (va == vb && ja > jb)) : ja > jb);
        if (a_gt == up) {
          kv[a] = vb; kv[b] = va;
          kj[a] = jb; kj[b] = ja;
        }
      }
      __syncthreads();
    }
  }
  for (int p = threadIdx.x; p < m; p += blockDim.x) {
    S[(int64_t)i * n + p] = kv[p];
    J[(int64_t)i * n + p] = kj[p];
  }
}

// Python slice length of a[:size_] for a length-`len` array.
__device__ __forceinline__ int slice_count(int size_, int len) {
  if (size_ >= 0) return size_ < len ? size_ : len;
  const int c = len + size_;
  return c > 0 ? c : 0;
}

// numpy's eight-accumulator pairwise block (n <= 128) of a[0..n) over one
// wave: lanes 0..7 run the eight accumulators (a[k], a[k+8], ... in order),
// then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) and the tail, every lane computing
// the same value; n < 8 is the plain sequential sum.
__device__ __forceinline__ float wave_pw_block_f32(const float* a, int n) {
  const int lane = threadIdx.x & 63;
  if (n < 8) {
    float res = 0.f;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  const int n8 = n - (n % 8);
  float r = 0.f;
  if (lane < 8) {
    r = a[lane];
    for (int q = lane + 8; q < n8; q += 8) r += a[q];
  }
  auto rl = [&](int k) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r), k)); };
  float res = ((rl(0) + rl(1)) + (rl(2) + rl(3))) + ((rl(4) + rl(5)) + (rl(6) + rl(7)));
  for (int q = n8; q < n; ++q) res += a[q];
  return res;
}

// np_pairwise_f32 over one wave, n <= 512.  numpy splits while a piece holds
// more than 128 elements; from n <= 512 the largest piece after three splits
// is <= 76, so three levels are exact (n = 505: 248 + (128 + (64 + 65))).
__device__ __forceinline__ float wave_pairwise_f32(const float* a, int n) {
  if (n <= 128) return wave_pw_block_f32(a, n);
  auto quarter = [&](const float* b, int m) -> float {
    if (m <= 128) return wave_pw_block_f32(b, m);
    int q = m / 2;
    q -= q % 8;
    return wave_pw_block_f32(b, q) + wave_pw_block_f32(b + q, m - q);
  };
  auto half = [&](const float* b, int m) -> float {
    if (m <= 128) return wave_pw_block_f32(b, m);
    int q = m / 2;
    q -= q % 8;
    return quarter(b, q) + quarter(b + q, m - q);
  };
  int n2 = n / 2;
  n2 -= n2 % 8;
  return half(a, n2) + half(a + n2, n - n2);
}

// `rounds` Krum selections over a shrinking alive set (rounds = 1: plain krum).
// order[t] = client chosen in round t; scores (round 0, all N) optional.
// One workgroup of 16 waves.  For N <= 128 the sorted rows (S fp32, J as
// bytes) are staged in LDS once, so a round is LDS-only.  Per round a wave
// takes its alive rows eight at a time: a ballot compaction of each row's
// first m alive entries, then the eight rows' pairwise sums at once (lanes
// 8u..8u+7 run row u's eight accumulators, lane 8u combines them and adds the
// tail), then a wave-parallel first minimum.  (Round 1 summed on one lane per
// row from global memory: 2.5 ms for Bulyan's 88 rounds at N = 128.)
constexpr int kKrumGStaged = 128;   // compacted-row stride (m <= 125 for N <= 128)
constexpr int kKrumGGlobal = 256;   // N <= 258 (m <= 256), eight rows per wave batch
constexpr int kKrumGBig = 512;      // N <= kMaxClients, two rows per wave batch (LDS)

// U: rows compacted per wave batch (eight, or two for the 512-wide rows)
template <bool STAGED, int GS = STAGED ? kKrumGStaged : kKrumGGlobal, int U = 8>
__global__ void __launch_bounds__(1024) krum_rounds_kernel(const float* __restrict__ Sg, const int* __restrict__ Jg,
                                                           int n, int f, int rounds, int* __restrict__ order,
                                                           float* __restrict__ scores0, int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) char kr_smem[];
  static_assert(U == 8 || !STAGED, "the staged kernel compacts eight rows per batch");
  __shared__ unsigned char alive[kMaxClients];
  __shared__ float score[kMaxClients];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nwaves = blockDim.x >> 6;
  float* gath = reinterpret_cast<float*>(kr_smem);                            // [16][U][GS]
  float* Ss = gath + 16 * U * GS;                                            // [n][n] when staged
  unsigned char* Js = reinterpret_cast<unsigned char*>(Ss + (STAGED ? n * n : 0));
  if constexpr (STAGED) {
    for (int e = tid; e < n * n; e += blockDim.x) {
      Ss[e] = Sg[e];
      Js[e] = static_cast<unsigned char>(Jg[e]);
    }
  }
  for (int i = tid; i < n; i += blockDim.x) alive[i] = 1;
  __syncthreads();
  float* gw = gath + wave * U * GS;
  const int u_me = lane >> 3, k_me = lane & 7;
  for (int t = 0; t < rounds; ++t) {
    const int nr = n - t;
    const int m = slice_count(nr - f - 2, nr - 1);
    for (int u0 = 0; wave + nwaves * u0 < n; u0 += U) {
      // compaction of up to U rows
      if constexpr (STAGED) {
        // N <= 128: each row is two 64-entry pieces.  All 2U pieces' LDS
        // reads are issued before any write (the compiler cannot tell the
        // compaction buffer from the staged rows, so a write between them
        // would serialise every piece on three LDS latencies); lanes with
        // nothing to keep write the row's spare last slot (m <= n - 2 < GS - 1)
        constexpr int NPC = 2 * U;
        int js[NPC], ev[NPC];
        bool rv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = wave + nwaves * (u0 + u);
          rv[u] = (i < n) & (alive[i < n ? i : 0] != 0);   // wave-uniform
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int p = 64 * h2 + lane;
            const int e = (i < n ? i : 0) * n + p;
            ev[2 * u + h2] = p < n - 1 ? e : 0;
            js[2 * u + h2] = Js[ev[2 * u + h2]];
          }
        }
        bool okv[NPC];
        float sv[NPC];
#pragma unroll
        for (int q = 0; q < NPC; ++q) {
          const int p = 64 * (q & 1) + lane;
          okv[q] = rv[q >> 1] & (p < n - 1) & (alive[js[q]] != 0);
          sv[q] = Ss[ev[q]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          int c = 0;
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const bool ok = okv[2 * u + h2];
            const unsigned long long bal = __builtin_amdgcn_ballot_w64(ok);
            const int pre = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(bal >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(bal), 0));
            const int dst = ok && c + pre < m ? c + pre : GS - 1;
            gw[u * GS + dst] = sv[2 * u + h2];
            c += __builtin_popcountll(bal);
          }
        }
      } else {
#pragma unroll 1
        for (int u = 0; u < U; ++u) {
          const int i = wave + nwaves * (u0 + u);
          if (i >= n || !alive[i]) continue;   // wave-uniform
          int c = 0;
          for (int p0 = 0; p0 < n - 1 && c < m; p0 += 64) {
            const int p = p0 + lane;
            const int64_t e = static_cast<int64_t>(i) * n + p;
            const bool ok = p < n - 1 && alive[Jg[e]];
            const unsigned long long bal = __builtin_amdgcn_ballot_w64(ok);
            const int pre = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(bal >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(bal), 0));
            if (ok && c + pre < m) gw[u * GS + c + pre] = Sg[e];
            c += __builtin_popcountll(bal);
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      // numpy pairwise sums of the eight compacted rows
      const int i_me = wave + nwaves * (u0 + u_me);
      const bool row_ok = u_me < U && i_me < n && alive[i_me];
      const float* a = gw + (u_me < U ? u_me : 0) * GS;
      float sc = 0.f;
      if (m <= 128) {
        const int n8 = m - (m % 8);
        float r = 0.f;
        if (m >= 8 && row_ok) {
          r = a[k_me];
          int q = k_me + 8;
          // four loads in flight, added in the same sequential order
          for (; q + 24 < n8; q += 32) {
            const float x0 = a[q], x1 = a[q + 8], x2 = a[q + 16], x3 = a[q + 24];
            r += x0;
            r += x1;
            r += x2;
            r += x3;
          }
          for (; q < n8; q += 8) r += a[q];
        }
        const int g = lane & ~7;
        const float r1 = __shfl(r, g + 1), r2 = __shfl(r, g + 2), r3 = __shfl(r, g + 3);
        const float r4 = __shfl(r, g + 4), r5 = __shfl(r, g + 5), r6 = __shfl(r, g + 6), r7 = __shfl(r, g + 7);
        if (k_me == 0 && row_ok) {
          if (m < 8) {
            for (int q = 0; q < m; ++q) sc += a[q];
          } else {
            sc = ((r + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
            for (int q = n8; q < m; ++q) sc += a[q];
          }
          score[i_me] = sc;
        }
      } else {
        // N > 130: one row at a time over the whole wave (numpy's split at n/2)
#pragma unroll 1
        for (int u = 0; u < U; ++u) {
          const int i = wave + nwaves * (u0 + u);
          if (i >= n || !alive[i]) continue;
          const float v = wave_pairwise_f32(gw + u * GS, m);
          if (lane == 0) score[i] = v;
        }
      }
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (wave == 0) {
      // np.argmin: first minimum; a NaN is the minimum (first NaN wins).
      // One 64-bit key per row, (class 0 NaN / 1 number / 2 dead, value as
      // order-preserving bits, index), so the wave minimum is two shuffles
      // and one compare per step; -0 is taken as +0 (equal scores: the
      // first index)
      static_assert(kMaxClients <= 65536, "16-bit index field");
      uint64_t best = ~0ull;
      for (int i = lane; i < n; i += 64) {
        const float v = score[i];
        const uint64_t cls = !alive[i] ? 2u : (v != v ? 0u : 1u);
        uint32_t ob = 0;
        if (cls == 1) {
          const uint32_t b = __builtin_bit_cast(uint32_t, v + 0.0f);
          ob = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
        }
        const uint64_t k = (cls << 48) | (static_cast<uint64_t>(ob) << 16) | static_cast<uint64_t>(i);
        best = k < best ? k : best;
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t hi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(best >> 32), off));
        const uint32_t lo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(best), off));
        const uint64_t o = (static_cast<uint64_t>(hi) << 32) | lo;
        best = o < best ? o : best;
      }
      const int bc = static_cast<int>(best >> 48);
      const int bi = static_cast<int>(best & 0xffffu);
      if (lane == 0) {
        const int pick = bc < 2 ? bi : -1;
        order[t] = pick;
        if (pick >= 0) alive[pick] = 0;
        if (pick < 0 && status) *status = 1;
      }
    }
    if (t == 0 && scores0) {
      for (int i = tid; i < n; i += blockDim.x) scores0[i] = score[i];
    }
    __syncthreads();
  }
}

// numpy's pairwise fp32 sum over one wave for any n the split depth reaches:
// each split leaves pieces of at most n/2 + 8 elements, so DEPTH levels cover
// n <= 128 * 2^DEPTH - 16 (DEPTH = 7: n <= 16368).  Out of line, one copy per
// level.
template <int DEPTH>
__device__ __attribute__((noinline)) float wave_pairwise_deep_f32(const float* a, int n) {
  if constexpr (DEPTH == 0) {
    return wave_pw_block_f32(a, n);
  } else {
    if (n <= 128) return wave_pw_block_f32(a, n);
    int q = n / 2;
    q -= q % 8;
    const float lo = wave_pairwise_deep_f32<DEPTH - 1>(a, q);
    return lo + wave_pairwise_deep_f32<DEPTH - 1>(a + q, n - q);
  }
}

// Krum rounds for kMaxClients < N <= kKrumMaxClients (no client-count ceiling
// the shipped configurations reach; the reference has none,
// robust_estimator.py:234-249).  One workgroup of 16 waves; alive flags and
// scores in dynamic LDS; a wave takes one alive row at a time, compacts its
// first m alive sorted distances into its own slice of the global scratch
// (16 x n floats, L2-resident) and sums them in numpy's pairwise order.
constexpr int kKrumMaxClients = 8192;
__global__ void __launch_bounds__(1024) krum_rounds_huge_kernel(const float* __restrict__ Sg,
                                                                const int* __restrict__ Jg, int n, int f, int rounds,
                                                                int* __restrict__ order, float* __restrict__ scores0,
                                                                float* __restrict__ scratch) {
  extern __shared__ __attribute__((aligned(16))) char kh_smem[];
  float* score = reinterpret_cast<float*>(kh_smem);
  unsigned char* alive = reinterpret_cast<unsigned char*>(score + n);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nwaves = blockDim.x >> 6;
  float* gw = scratch + static_cast<int64_t>(wave) * n;
  for (int i = tid; i < n; i += blockDim.x) alive[i] = 1;
  __syncthreads();
  for (int t = 0; t < rounds; ++t) {
    const int nr = n - t;
    const int m = slice_count(nr - f - 2, nr - 1);
#pragma unroll 1
    for (int i = wave; i < n; i += nwaves) {
      if (!alive[i]) continue;   // wave-uniform
      int c = 0;
      for (int p0 = 0; p0 < n - 1 && c < m; p0 += 64) {
        const int p = p0 + lane;
        const int64_t e = static_cast<int64_t>(i) * n + p;
        const bool ok = p < n - 1 && alive[checked_row(Jg[p < n - 1 ? e : 0], n)];
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(ok);
        const int pre = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(bal >> 32),
                                                  __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(bal), 0));
        if (ok && c + pre < m) gw[c + pre] = Sg[e];
        c += __builtin_popcountll(bal);
      }
      __threadfence_block();
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      const float v = wave_pairwise_deep_f32<7>(gw, m);
      if (lane == 0) score[i] = v;
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (wave == 0) {
      // np.argmin as krum_rounds_kernel: first minimum, a NaN is the minimum
      int bc = 2, bi = 0x7fffffff;
      float bv = 0.f;
      for (int i = lane; i < n; i += 64) {
        const float v = score[i];
        const int c = !alive[i] ? 2 : (v != v ? 0 : 1);
        if (c < bc || (c == bc && c == 1 && v < bv)) {
          bc = c;
          bv = v;
          bi = i;
        }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const int oc = __shfl_xor(bc, off);
        const float ov = __shfl_xor(bv, off);
        const int oi = __shfl_xor(bi, off);
        const bool better = oc < bc || (oc == bc && ((oc == 1 && ov < bv) || ((oc != 1 || ov == bv) && oi < bi)));
        if (better) {
          bc = oc;
          bv = ov;
          bi = oi;
        }
      }
      if (lane == 0) {
        const int best = bc < 2 ? bi : -1;
        order[t] = best;
        if (best >= 0) alive[best] = 0;
      }
    }
    if (t == 0 && scores0) {
      for (int i = tid; i < n; i += blockDim.x) scores0[i] = score[i];
    }
    __syncthreads();
  }
}

// bytes of the rounds' compaction scratch (N > kMaxClients only)
static size_t krum_scratch_bytes(int n) { return n > kMaxClients ? static_cast<size_t>(16) * n * 4 + 256 : 0; }

unsigned int krum_row_faults(bool reset) { return tu_row_faults(reset); }

// out[r, :] = X[order[r], :] (the chosen clients' rows); the index is checked
// against the n rows of X
__global__ void gather_rows_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                   const int* __restrict__ order, int nrows, float* __restrict__ out, int64_t ldo) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int r = blockIdx.y;
  if (j >= d || r >= nrows) return;
  const int src = checked_row(order[r], n);
  out[r * ldo + j] = X[static_cast<int64_t>(src) * ldx + j];
}

size_t krum_workspace_bytes(int n, int64_t d);
size_t gram_workspace_bytes(int n, int64_t d);
int launch_gram(const float* X, int n, int64_t d, int64_t ldx, double* G, void* ws, size_t ws_bytes, hipStream_t s);

// workspace layout: [flag (256 B)][G fp64 n*n][acc fp64 n*n][cls int n*n][D n*n][S n*n][J n*n]
// [rounds scratch (N > kMaxClients)][gram slab]
size_t krum_workspace_bytes(int n, int64_t d) {
  const size_t nn = static_cast<size_t>(n) * n;
  return 256 + nn * 8 * 2 + nn * 4 * 4 + krum_scratch_bytes(n) + gram_workspace_bytes(n, d);
}

static int launch_rowsort_and_rounds(const float* D, int n, int f, int rounds, int* order, float* scores0,
                                     const int* nonfinite, const double* acc, const int* cls, hipStream_t s);

// X (optional): the data G came from; with it, a non-finite G switches the
// distances to the exact per-pair route (krum_direct_kernel), nonfinite / acc
// its flag and n x n fp64 accumulator
static int launch_krum_rounds(const double* G, int n, int f, int rounds, int* order, float* scores0, char* ws,
                              const float* X, int64_t d, int64_t ldx, int* nonfinite, double* acc, int* cls,
                              hipStream_t s, int nx = 0, int bs = 1) {
  const size_t nn = static_cast<size_t>(n) * n;
  float* D = reinterpret_cast<float*>(ws);
  (void)nn;
  // narrow layers (d <= kExactMaxD) always take the exact route: with few
  // coordinates the nearest pairs sit far below the rows' norms, where the
  // Gram's G_ii + G_jj - 2 G_ij loses the bits the reference's fp32 norm of
  // the difference keeps (one slice per tile pair: no atomics, deterministic)
  const bool narrow = X != nullptr && d <= kExactMaxD;
  if (X != nullptr) SRA_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(nonfinite), narrow ? 1 : 0, 1, s));
  hipLaunchKernelGGL(krum_dist_kernel, dim3(cdiv(n * n, 256)), dim3(256), 0, s, G, n, D, X ? nonfinite : nullptr,
                     X ? acc : nullptr, X ? cls : nullptr);
  int rc = launch_status("krum_dist_kernel");
  if (rc) return rc;
  if (X != nullptr && n > 1) {
    const int nt = static_cast<int>(cdiv(n, kDirTile));
    const int64_t kb = cdiv(d, kDirK);
    const int slices = narrow ? 1 : static_cast<int>(kb < 256 ? kb : 256);
    hipLaunchKernelGGL(krum_direct_kernel, dim3(slices, nt * (nt + 1) / 2), dim3(256), 0, s, X, n, d, ldx,
                       bs == 1 ? n : nx, bs, nonfinite, acc, cls, slices);
    rc = launch_status("krum_direct_kernel");
    if (rc) return rc;
  }
  return launch_rowsort_and_rounds(D, n, f, rounds, order, scores0, X ? nonfinite : nullptr, X ? acc : nullptr,
                                   X ? cls : nullptr, s);
}

// Row sorts and the selection rounds, from D (or, with *nonfinite set, from the
// exact per-pair acc / cls); D heads [D n*n][S n*n][J n*n][rounds scratch].
static int launch_rowsort_and_rounds(const float* D, int n, int f, int rounds, int* order, float* scores0,
                                     const int* nonfinite, const double* acc, const int* cls, hipStream_t s) {
  const size_t nn = static_cast<size_t>(n) * n;
  float* S = const_cast<float*>(D) + nn;
  int* J = reinterpret_cast<int*>(S + nn);
  int rc = SRA_OK;
  if (n > 1) {
    int pn = 1;
    while (pn < n - 1) pn <<= 1;
    static const hipError_t attr_s =
        hipFuncSetAttribute(reinterpret_cast<const void*>(krum_rowsort_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 8 * kKrumMaxClients);
    SRA_REQUIRE(attr_s == hipSuccess || pn * 8 <= 65536, SRA_ERR_UNSUPPORTED,
                "krum_rowsort_kernel: cannot reserve %d bytes of dynamic LDS", pn * 8);
    hipLaunchKernelGGL(krum_rowsort_kernel, dim3(n), dim3(256), pn * 8, s, D, n, S, J, nonfinite, acc, cls);
    rc = launch_status("krum_rowsort_kernel");
    if (rc) return rc;
  }
  if (n > kMaxClients) {
    float* scratch = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(J + nn) + 255) & ~uintptr_t(255));
    const int lds = n * 5 + 16;   // scores + alive flags
    hipLaunchKernelGGL(krum_rounds_huge_kernel, dim3(1), dim3(1024), lds, s, S, J, n, f, rounds, order, scores0,
                       scratch);
    return launch_status("krum_rounds_huge_kernel");
  }
  if (n <= 128) {
    const int lds = 16 * 8 * kKrumGStaged * 4 + n * n * 5;   // compacted rows + S fp32 + J bytes
    static const hipError_t attr =
        hipFuncSetAttribute(reinterpret_cast<const void*>(krum_rounds_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 16 * 8 * kKrumGStaged * 4 + 128 * 128 * 5);
    if (attr == hipSuccess) {
      hipLaunchKernelGGL(krum_rounds_kernel<true>, dim3(1), dim3(1024), lds, s, S, J, n, f, rounds, order, scores0,
                         nullptr);
      return launch_status("krum_rounds_kernel");
    }
  }
  if (n > kKrumGGlobal + 2) {   // compacted rows longer than 256
    constexpr int lds_big = 16 * 2 * kKrumGBig * 4;
    static const hipError_t attr_b =
        hipFuncSetAttribute(reinterpret_cast<const void*>(krum_rounds_kernel<false, kKrumGBig, 2>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds_big);
    SRA_REQUIRE(attr_b == hipSuccess, SRA_ERR_UNSUPPORTED,
                "krum_rounds_kernel: cannot reserve %d bytes of dynamic LDS (%s)", lds_big, hipGetErrorString(attr_b));
    hipLaunchKernelGGL((krum_rounds_kernel<false, kKrumGBig, 2>), dim3(1), dim3(1024), lds_big, s, S, J, n, f, rounds,
                       order, scores0, nullptr);
    return launch_status("krum_rounds_kernel");
  }
  static const hipError_t attr_g =
      hipFuncSetAttribute(reinterpret_cast<const void*>(krum_rounds_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 16 * 8 * kKrumGGlobal * 4);
  SRA_REQUIRE(attr_g == hipSuccess, SRA_ERR_UNSUPPORTED,
              "krum_rounds_kernel: cannot reserve %d bytes of dynamic LDS (%s)", 16 * 8 * kKrumGGlobal * 4,
              hipGetErrorString(attr_g));
  hipLaunchKernelGGL(krum_rounds_kernel<false>, dim3(1), dim3(1024), 16 * 8 * kKrumGGlobal * 4, s, S, J, n, f, rounds,
                     order, scores0, nullptr);
  return launch_status("krum_rounds_kernel");
}

// [D n*n][S n*n][J n*n][rounds scratch]
size_t krum_from_gram_workspace_bytes(int n) { return static_cast<size_t>(n) * n * 12 + krum_scratch_bytes(n); }

int launch_krum_rounds_from_gram(const double* G, int n, int f, int rounds, int* order, float* scores0,
                                 char* ws, hipStream_t s) {
  return launch_krum_rounds(G, n, f, rounds, order, scores0, ws, nullptr, 0, 0, nullptr, nullptr, nullptr, s);
}

int launch_krum(const float* X, int n, int64_t d, int64_t ldx, int f, int rounds, int* order, float* scores0,
                void* ws, size_t ws_bytes, hipStream_t s) {
  SRA_REQUIRE(n >= 1 && n <= kKrumMaxClients, SRA_ERR_UNSUPPORTED, "Krum supports 1 <= N <= %d (got %d)",
              kKrumMaxClients, n);
  SRA_REQUIRE(rounds >= 1 && rounds <= n, SRA_ERR_ARG, "rounds must be in [1, N] (got %d)", rounds);
  SRA_REQUIRE(ws != nullptr && ws_bytes >= krum_workspace_bytes(n, d), SRA_ERR_WORKSPACE,
              "Krum workspace too small: need %zu bytes", krum_workspace_bytes(n, d));
  const size_t nn = static_cast<size_t>(n) * n;
  char* base = static_cast<char*>(ws);
  int* nonfinite = reinterpret_cast<int*>(base);
  double* G = reinterpret_cast<double*>(base + 256);
  double* acc = G + nn;
  int* cls = reinterpret_cast<int*>(acc + nn);
  char* rest = reinterpret_cast<char*>(cls + nn);
  char* slab = rest + nn * 4 * 3 + krum_scratch_bytes(n);
  int rc = launch_gram(X, n, d, ldx, G, slab, gram_workspace_bytes(n, d), s);
  if (rc) return rc;
  return launch_krum_rounds(G, n, f, rounds, order, scores0, rest, X, d, ldx, nonfinite, acc, cls, s);
}

// mom_krum (src/robust_estimator.py:250-256) without the bucket matrix: the
// Gram of the bucket means straight from the clients (gram_bucket.hip), Krum
// over the nb = ceil(n / bs) buckets (the exact route, when flagged, forms the
// means on the fly), then the chosen bucket's mean row.
int launch_gram_buckets(const float* X, int n, int bs, int64_t d, int64_t ldx, double* G, float* slab,
                        hipStream_t s);

__global__ void __launch_bounds__(256) bucket_row_kernel(const float* __restrict__ X, int n, int64_t d, int64_t ldx,
                                                         int bs, int nb, const int* __restrict__ order,
                                                         float* __restrict__ out) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= d) return;
  out[k] = row_value(X, ldx, n, bs, checked_row(order[0], nb), k);
}

int launch_mom_krum(const float* X, int n, int64_t d, int64_t ldx, int f, int bs, int* order, float* out, void* ws,
                    size_t ws_bytes, hipStream_t s) {
  SRA_REQUIRE(n >= 1 && bs >= 1 && bs <= 4, SRA_ERR_UNSUPPORTED, "fused mom_krum: 1 <= bucket size <= 4 (got %d)",
              bs);
  const int nb = static_cast<int>(cdiv(n, bs));
  SRA_REQUIRE(nb <= 32 * kBucketGramMaxNB, SRA_ERR_UNSUPPORTED, "fused mom_krum: at most %d buckets (got %d)",
              32 * kBucketGramMaxNB, nb);
  SRA_REQUIRE(ws != nullptr && ws_bytes >= krum_workspace_bytes(nb, d), SRA_ERR_WORKSPACE,
              "mom_krum workspace too small: need %zu bytes", krum_workspace_bytes(nb, d));
  const size_t nn = static_cast<size_t>(nb) * nb;
  char* base = static_cast<char*>(ws);
  int* nonfinite = reinterpret_cast<int*>(base);
  double* G = reinterpret_cast<double*>(base + 256);
  double* acc = G + nn;
  int* cls = reinterpret_cast<int*>(acc + nn);
  char* rest = reinterpret_cast<char*>(cls + nn);
  float* slab = reinterpret_cast<float*>(rest + nn * 4 * 3 + krum_scratch_bytes(nb));
  int rc = launch_gram_buckets(X, n, bs, d, ldx, G, slab, s);
  if (rc) return rc;
  rc = launch_krum_rounds(G, nb, f, 1, order, nullptr, rest, X, d, ldx, nonfinite, acc, cls, s, n, bs);
  if (rc) return rc;
  hipLaunchKernelGGL(bucket_row_kernel, dim3(cdiv(d, 256)), dim3(256), 0, s, X, n, d, ldx, bs, nb, order, out);
  return launch_status("bucket_row_kernel");
}

// ---------------------------------------------------------------------------
// The exact per-pair route over a column-sharded layer (shard.krum, mom_krum,
// Bulyan-Krum).  ||a - b||^2 over all columns is the sum over the
// shards of ||a_s - b_s||^2, so every rank forms its partial with
// krum_direct_kernel, codes the pair's class into the value (NaN if any term
// is NaN, else +inf if any is inf: fp64 addition of the ranks' partials then
// reproduces the reference's class rule, NaN + x = NaN, inf + finite = inf), one
// reduce sums them on the scoring rank, and launch_krum_from_pairs scores the
// sum with the unsharded route's row sort (NaN last) and rounds.
// ---------------------------------------------------------------------------
__global__ void pair_encode_kernel(double* __restrict__ acc, const int* __restrict__ cls, int n) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= static_cast<int64_t>(n) * n) return;
  const int c = cls[e];
  if (c & 1) acc[e] = __builtin_nan("");
  else if (c & 2) acc[e] = __builtin_inf();
}

// [flag (256 B)][cls int n*n]
size_t krum_pair_sq_workspace_bytes(int nb) { return 256 + static_cast<size_t>(nb) * nb * 4; }

int launch_krum_pair_sq(const float* X, int nx, int64_t d, int64_t ldx, int bs, double* acc, void* ws,
                        size_t ws_bytes, hipStream_t s) {
  const int nb = static_cast<int>(cdiv(nx, bs));
  SRA_REQUIRE(nb >= 1 && nb <= kKrumMaxClients, SRA_ERR_UNSUPPORTED, "Krum supports 1 <= N <= %d (got %d)",
              kKrumMaxClients, nb);
  SRA_REQUIRE(ws != nullptr && ws_bytes >= krum_pair_sq_workspace_bytes(nb), SRA_ERR_WORKSPACE,
              "pair workspace too small: need %zu bytes", krum_pair_sq_workspace_bytes(nb));
  const size_t nn = static_cast<size_t>(nb) * nb;
  int* flag = static_cast<int*>(ws);
  int* cls = reinterpret_cast<int*>(static_cast<char*>(ws) + 256);
  SRA_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flag), 1, 1, s));
  SRA_HIP(hipMemsetAsync(acc, 0, nn * 8, s));
  SRA_HIP(hipMemsetAsync(cls, 0, nn * 4, s));
  if (nb > 1) {
    const int nt = static_cast<int>(cdiv(nb, kDirTile));
    const int64_t kb = cdiv(d, kDirK);
    const int slices = d <= kExactMaxD ? 1 : static_cast<int>(kb < 256 ? kb : 256);
    hipLaunchKernelGGL(krum_direct_kernel, dim3(slices, nt * (nt + 1) / 2), dim3(256), 0, s, X, nb, d, ldx,
                       bs == 1 ? nb : nx, bs, flag, acc, cls, slices);
    int rc = launch_status("krum_direct_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(pair_encode_kernel, dim3(cdiv(static_cast<int64_t>(nn), 256)), dim3(256), 0, s, acc, cls, nb);
  return launch_status("pair_encode_kernel");
}

// [flag (256 B)][D n*n][S n*n][J n*n][rounds scratch]
size_t krum_from_pairs_workspace_bytes(int n) { return 256 + krum_from_gram_workspace_bytes(n); }

int launch_krum_from_pairs(const double* acc, int n, int f, int rounds, int* order, float* scores0, void* ws,
                           hipStream_t s) {
  int* flag = static_cast<int*>(ws);
  SRA_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flag), 1, 1, s));
  return launch_rowsort_and_rounds(reinterpret_cast<float*>(static_cast<char*>(ws) + 256), n, f, rounds, order,
                                   scores0, flag, acc, nullptr, s);
}

}  // namespace sra

using namespace sra;

extern "C" int sra_krum_pair_sq_workspace_bytes(int64_t n, int32_t bucket_size, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(bucket_size >= 1 && n >= 1 && cdiv(n, bucket_size) <= kKrumMaxClients, SRA_ERR_UNSUPPORTED,
              "Krum supports 1 <= ceil(N / bucket size) <= %d", kKrumMaxClients);
  *bytes = krum_pair_sq_workspace_bytes(static_cast<int>(cdiv(n, bucket_size)));
  return SRA_OK;
}

extern "C" int sra_krum_pair_sq_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t bucket_size,
                                    double* acc, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(X != nullptr && acc != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= (int64_t(1) << 30) && d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad shape");
  SRA_REQUIRE(bucket_size >= 1, SRA_ERR_ARG, "bucket size must be >= 1 (got %d)", bucket_size);
  return launch_krum_pair_sq(X, static_cast<int>(n), d, ldx, bucket_size, acc, ws, ws_bytes,
                             static_cast<hipStream_t>(stream));
}

extern "C" int sra_krum_from_pairs_workspace_bytes(int64_t n, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && n <= kKrumMaxClients, SRA_ERR_UNSUPPORTED, "Krum supports 1 <= N <= %d", kKrumMaxClients);
  *bytes = krum_from_pairs_workspace_bytes(static_cast<int>(n));
  return SRA_OK;
}

extern "C" int sra_krum_from_pairs(const double* acc, int64_t n, int32_t f, int32_t rounds, int32_t* order,
                                   float* scores, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(acc != nullptr && order != nullptr && ws != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= kKrumMaxClients, SRA_ERR_UNSUPPORTED, "Krum supports 1 <= N <= %d", kKrumMaxClients);
  SRA_REQUIRE(rounds >= 1 && rounds <= n, SRA_ERR_ARG, "rounds must be in [1, N]");
  SRA_REQUIRE(ws_bytes >= krum_from_pairs_workspace_bytes(static_cast<int>(n)), SRA_ERR_WORKSPACE,
              "workspace too small: need %zu bytes", krum_from_pairs_workspace_bytes(static_cast<int>(n)));
  return launch_krum_from_pairs(acc, static_cast<int>(n), f, rounds, order, scores, ws,
                                static_cast<hipStream_t>(stream));
}

extern "C" int sra_mom_krum_workspace_bytes(int64_t n, int64_t d, int32_t bucket_size, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && d >= 1 && bucket_size >= 1 && bucket_size <= 4 &&
                  cdiv(n, bucket_size) <= 32 * kBucketGramMaxNB, SRA_ERR_UNSUPPORTED,
              "fused mom_krum: 1 <= bucket size <= 4, at most %d buckets", 32 * kBucketGramMaxNB);
  *bytes = krum_workspace_bytes(static_cast<int>(cdiv(n, bucket_size)), d);
  return SRA_OK;
}

extern "C" int sra_mom_krum_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t bucket_size,
                                int32_t* order, float* out, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(X != nullptr && order != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= (int64_t(1) << 30) && d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad shape");
  return launch_mom_krum(X, static_cast<int>(n), d, ldx, f, bucket_size, order, out, ws, ws_bytes,
                         static_cast<hipStream_t>(stream));
}

extern "C" int sra_krum_workspace_bytes(int64_t n, int64_t d, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && n <= kKrumMaxClients && d >= 1, SRA_ERR_UNSUPPORTED, "Krum supports 1 <= N <= %d",
              kKrumMaxClients);
  *bytes = krum_workspace_bytes(static_cast<int>(n), d);
  return SRA_OK;
}

extern "C" int sra_krum_from_gram_workspace_bytes(int64_t n, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(n >= 1 && n <= kKrumMaxClients, SRA_ERR_UNSUPPORTED, "Krum supports 1 <= N <= %d", kKrumMaxClients);
  *bytes = krum_from_gram_workspace_bytes(static_cast<int>(n));
  return SRA_OK;
}

extern "C" int sra_krum_select_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t rounds,
                                   int32_t* order, float* scores, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(X != nullptr && order != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx (%lld/%lld)", (long long)d, (long long)ldx);
  return launch_krum(X, static_cast<int>(n), d, ldx, f, rounds, order, scores, ws, ws_bytes,
                     static_cast<hipStream_t>(stream));
}

extern "C" int sra_krum_from_gram(const double* G, int64_t n, int32_t f, int32_t rounds, int32_t* order,
                                  float* scores, void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(G != nullptr && order != nullptr && ws != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= kKrumMaxClients, SRA_ERR_UNSUPPORTED, "Krum supports 1 <= N <= %d", kKrumMaxClients);
  SRA_REQUIRE(rounds >= 1 && rounds <= n, SRA_ERR_ARG, "rounds must be in [1, N]");
  SRA_REQUIRE(ws_bytes >= krum_from_gram_workspace_bytes(static_cast<int>(n)), SRA_ERR_WORKSPACE,
              "workspace too small: need %zu bytes", krum_from_gram_workspace_bytes(static_cast<int>(n)));
  return launch_krum_rounds_from_gram(G, static_cast<int>(n), f, rounds, order, scores, static_cast<char*>(ws),
                                      static_cast<hipStream_t>(stream));
}

extern "C" int sra_gather_rows_f32(const float* X, int64_t n, int64_t d, int64_t ldx, const int32_t* rows,
                                   int32_t nrows, float* out, int64_t ldo, void* stream) {
  SRA_REQUIRE(X != nullptr && rows != nullptr && out != nullptr, SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(n >= 1 && n <= (int64_t(1) << 30) && nrows >= 1 && d >= 1 && ldo >= d && ldx >= d, SRA_ERR_SHAPE,
              "bad gather shape");
  hipLaunchKernelGGL(gather_rows_kernel, dim3(cdiv(d, 256), nrows), dim3(256), 0, static_cast<hipStream_t>(stream),
                     X, static_cast<int>(n), d, ldx, rows, nrows, out, ldo);
  return launch_status("gather_rows_kernel");
}
