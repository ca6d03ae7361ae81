// k8 — the attack-side callers of the aggregation path (src/attack.py;
// SURVEY.md §8(f).2).  They run inside the reference's round loop
// (simulate.py:218-229) on the same per-client updates the aggregators read.
//
//   attack_krum (attack.py:202-262), per layer: the malicious rows become
//     -lambda * sign(sum of the benign rows), lambda = 1, 1/2, 1/4, ... the first
//     value for which krum(f=1) over ALL clients picks a malicious row, or the
//     first one below lower_bound.  The reference re-runs the O(m^2 d) krum for
//     every lambda (up to 28 times per layer).  Here the d-dependent work runs once:
//       sign_sum    s_k = sign(sum over benign c, in order, of (double) x_ck)
//       Gram        benign-benign distances exactly as krum (k2 + k3 rounding)
//       sa_norms    A_i = sum_k s_k x_ik, B_i = sum_k x_ik^2 (fp64), S = |s|^2
//     so ||-lambda s - x_i||^2 = lambda^2 S + 2 lambda A_i + B_i and every
//     lambda is scored in client space.  All candidate lambdas are scored at
//     once (one workgroup each); the first successful one wins, as in the loop.
//     The reference's min_dis / max_dis loop (:217-235) does not affect the
//     result and is not reproduced.
//   attack_trimmedmean (attack.py:157-198): one uniform draw from Python's
//     `random` module per element, between the benign extreme and b times it.
//     The Mersenne Twister stream is reproduced on the device (mt19937_kernel:
//     same state in, same words out, the module's state advanced identically),
//     so the malicious rows are bit-identical to the reference's.
//   attack_xie (attack.py:362-372): -weight * (sum of the benign chosen rows,
//     sequential, input precision) / len(choices).
#include "sra_common.hpp"

namespace sra {

constexpr int kAtkBS = 256;
constexpr int kAtkTile = 4096;        // columns per fp64 partial (sa_norms)
constexpr int kAtkMaxClients = 2048;   // distance lists in LDS: 3 x 16 KiB fp64 + 8 KiB fp32

size_t gram_workspace_bytes(int n, int64_t d);
int launch_gram(const float* X, int n, int64_t d, int64_t ldx, double* G, void* ws, size_t ws_bytes, hipStream_t s);

// ---------------------------------------------------------------------------
// attack_krum
// ---------------------------------------------------------------------------
__device__ __forceinline__ double np_sign(double v) {
  return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : (v == 0.0 ? 0.0 : v));   // NaN stays NaN
}

// s_k = sign(0.0 + x_b0k + x_b1k + ...) in fp64, benign rows in order
// (average_sign, attack.py:211-216)
__global__ void __launch_bounds__(kAtkBS) sign_sum_kernel(const float* __restrict__ X, int64_t d, int64_t ldx,
                                                          const int* __restrict__ rows, int nrows,
                                                          float* __restrict__ s) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kAtkBS + threadIdx.x;
  if (k >= d) return;
  double acc = 0.0;
  for (int r = 0; r < nrows; ++r) acc += static_cast<double>(X[static_cast<int64_t>(rows[r]) * ldx + k]);
  s[k] = static_cast<float>(np_sign(acc));
}

// per (tile, benign position y): partial sums of s_k x_yk and x_yk^2; y == nrows
// sums s_k^2.  Fixed-order reductions (deterministic).
__global__ void __launch_bounds__(kAtkBS) sa_partial_kernel(const float* __restrict__ X, int64_t d, int64_t ldx,
                                                            const int* __restrict__ rows, int nrows,
                                                            const float* __restrict__ s, double* __restrict__ part) {
  __shared__ double red[2][kAtkBS / 64];
  const int y = blockIdx.y;
  const int64_t k0 = static_cast<int64_t>(blockIdx.x) * kAtkTile;
  const int64_t k1 = k0 + kAtkTile < d ? k0 + kAtkTile : d;
  double a = 0.0, b = 0.0;
  if (y < nrows) {
    const float* x = X + static_cast<int64_t>(rows[y]) * ldx;
    for (int64_t k = k0 + threadIdx.x; k < k1; k += kAtkBS) {
      const double v = static_cast<double>(x[k]);
      a = fma(static_cast<double>(s[k]), v, a);
      b = fma(v, v, b);
    }
  } else {
    for (int64_t k = k0 + threadIdx.x; k < k1; k += kAtkBS) {
      const double v = static_cast<double>(s[k]);
      a = fma(v, v, a);
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = a;
    red[1][wave] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ta = 0.0, tb = 0.0;
    for (int w = 0; w < kAtkBS / 64; ++w) {
      ta += red[0][w];
      tb += red[1][w];
    }
    double* o = part + (static_cast<int64_t>(blockIdx.x) * (nrows + 1) + y) * 2;
    o[0] = ta;
    o[1] = tb;
  }
}

// AB[y] = (A_y, B_y) for benign position y; AB[nrows] = (S, 0)
__global__ void sa_reduce_kernel(const double* __restrict__ part, int ntiles, int nrows, double* __restrict__ AB) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y > nrows) return;
  double a = 0.0, b = 0.0;
  for (int t = 0; t < ntiles; ++t) {
    a += part[(static_cast<int64_t>(t) * (nrows + 1) + y) * 2];
    b += part[(static_cast<int64_t>(t) * (nrows + 1) + y) * 2 + 1];
  }
  AB[2 * y] = a;
  AB[2 * y + 1] = b;
}

// Benign row i's distances to the other benign rows, fp32 as krum
// (fp32(sqrt(max(G_ii + G_jj - 2 G_ij, 0)))), sorted ascending (NaN last):
// one workgroup per benign row, bitonic in LDS.
__global__ void __launch_bounds__(kAtkBS) benign_rowsort_kernel(const double* __restrict__ G, int m,
                                                                const int* __restrict__ rows, int nrows,
                                                                float* __restrict__ Sb) {
  __shared__ float kv[kAtkMaxClients];
  const int i = blockIdx.x;
  const int gi = rows[i];
  const int cnt = nrows - 1;
  int pn = 1;
  while (pn < cnt) pn <<= 1;
  for (int p = threadIdx.x; p < pn; p += blockDim.x) {
    float v = __builtin_inff();
    if (p < cnt) {
      const int gj = rows[p < i ? p : p + 1];
      const double sq = G[static_cast<int64_t>(gi) * m + gi] + G[static_cast<int64_t>(gj) * m + gj] -
                        2.0 * G[static_cast<int64_t>(gi) * m + gj];
      v = static_cast<float>(sqrt(sq > 0.0 ? sq : 0.0));
    }
    kv[p] = v;
  }
  __syncthreads();
  for (int k = 2; k <= pn; k <<= 1) {
    for (int st = k >> 1; st > 0; st >>= 1) {
      for (int h = threadIdx.x; h < pn / 2; h += blockDim.x) {
        const int a = (h / st) * (2 * st) + (h % st);
        const int b = a + st;
        const bool up = (a & k) == 0;
        const float va = kv[a], vb = kv[b];
        const bool a_gt = (va != va) ? (vb == vb) : (vb == vb && va > vb);
        if (a_gt == up) {
          kv[a] = vb;
          kv[b] = va;
        }
      }
      __syncthreads();
    }
  }
  for (int p = threadIdx.x; p < cnt; p += blockDim.x) Sb[static_cast<int64_t>(i) * kAtkMaxClients + p] = kv[p];
}

__device__ __forceinline__ int slice_len(int size_, int len) {
  if (size_ >= 0) return size_ < len ? size_ : len;
  const int c = len + size_;
  return c > 0 ? c : 0;
}

// One workgroup per candidate lambda_k = 2^-k: krum(f=1) scores of all m
// clients with the malicious rows at -lambda_k s (robust_estimator.py:234-249).
// A client's distance list mixes fp32 benign-benign norms with fp64 norms
// against the fp64 malicious rows, so numpy holds it as float64 and sums the
// smallest m-3 with its pairwise fp64 order.  chosen[k] = np.argmin (first
// minimum; a NaN wins).
__global__ void __launch_bounds__(kAtkBS) attack_krum_search_kernel(const float* __restrict__ Sb,
                                                                    const double* __restrict__ AB, int nrows,
                                                                    const int* __restrict__ mal_mask, int m,
                                                                    int* __restrict__ chosen) {
  __shared__ double dm[kAtkMaxClients];      // distance of benign position i to a malicious row
  __shared__ double ds[kAtkMaxClients];      // the same, sorted (a malicious row's list)
  __shared__ double score[kAtkMaxClients];   // per benign position
  __shared__ double smal;
  const int tid = threadIdx.x;
  const double lam = __builtin_amdgcn_ldexp(1.0, -static_cast<int>(blockIdx.x));
  const int c = m - nrows;
  const double S = AB[2 * nrows];
  int pn = 1;
  while (pn < nrows) pn <<= 1;
  for (int i = tid; i < pn; i += kAtkBS) {
    double v = __builtin_inf();
    if (i < nrows) {
      const double sq = lam * lam * S + 2.0 * lam * AB[2 * i] + AB[2 * i + 1];
      v = sqrt(sq > 0.0 ? sq : 0.0);
      dm[i] = v;
    }
    ds[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= pn; k <<= 1) {
    for (int st = k >> 1; st > 0; st >>= 1) {
      for (int h = tid; h < pn / 2; h += kAtkBS) {
        const int a = (h / st) * (2 * st) + (h % st);
        const int b = a + st;
        const bool up = (a & k) == 0;
        const double va = ds[a], vb = ds[b];
        const bool a_gt = (va != va) ? (vb == vb) : (vb == vb && va > vb);
        if (a_gt == up) {
          ds[a] = vb;
          ds[b] = va;
        }
      }
      __syncthreads();
    }
  }
  const int size_ = slice_len(m - 1 - 2, m - 1);
  // a malicious row: (c-1) exact zeros, then the sorted benign distances
  // numpy's pairwise fp64 sum; lists above 512 need the deeper split
  auto pw = [&](int cnt, auto&& g) -> double { return cnt <= 512 ? np_pw64(0, cnt, g) : np_pw64_rec<5>(0, cnt, g); };
  if (tid == 0) smal = pw(size_, [&](int q) { return q < c - 1 ? 0.0 : ds[q - (c - 1)]; });
  // a benign row: its sorted benign list merged with c copies of dm[i] (any
  // split point inside a run of equal values yields the same sequence)
  for (int i = tid; i < nrows; i += kAtkBS) {
    const float* sb = Sb + static_cast<int64_t>(i) * kAtkMaxClients;
    const double dmi = dm[i];
    int lo = 0, hi = nrows - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (static_cast<double>(sb[mid]) < dmi) lo = mid + 1;
      else hi = mid;
    }
    const int p = lo;
    score[i] = pw(size_, [&](int q) {
      return q < p ? static_cast<double>(sb[q]) : (q < p + c ? dmi : static_cast<double>(sb[q - c]));
    });
  }
  __syncthreads();
  if (tid == 0) {
    int best = -1, bpos = 0;
    double bv = 0.0;
    for (int j = 0; j < m; ++j) {
      const double v = mal_mask[j] ? smal : score[bpos++];
      if (best < 0) {
        best = j;
        bv = v;
        if (v != v) break;
        continue;
      }
      if (v != v) {
        best = j;
        break;
      }
      if (v < bv) {
        best = j;
        bv = v;
      }
    }
    chosen[blockIdx.x] = best;
  }
}

// first candidate whose pick is malicious, else the last one (below lower_bound)
__global__ void attack_krum_pick_kernel(const int* __restrict__ chosen, int K, const int* __restrict__ mal_mask,
                                        double* __restrict__ lam_out, int* __restrict__ chosen_out) {
  int k = K - 1;
  for (int q = 0; q < K; ++q) {
    if (mal_mask[chosen[q]]) {
      k = q;
      break;
    }
  }
  lam_out[0] = __builtin_amdgcn_ldexp(1.0, -k);
  chosen_out[0] = chosen[k];
}

// the malicious layer value -lambda * s (fp64, attack.py:259-260)
__global__ void __launch_bounds__(kAtkBS) attack_krum_row_kernel(const float* __restrict__ s, int64_t d,
                                                                 const double* __restrict__ lam,
                                                                 double* __restrict__ out) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kAtkBS + threadIdx.x;
  if (k >= d) return;
  out[k] = -lam[0] * static_cast<double>(s[k]);
}

// candidates lambda = 2^-k for k = 0 .. K-1: the loop stops at the first
// lambda below lower_bound (after scoring it)
int attack_krum_candidates(double lower_bound) {
  int k = 0;
  while (k < 1100 && std::ldexp(1.0, -k) >= lower_bound) ++k;
  return k + 1;
}

constexpr size_t al256(size_t b) { return (b + 255) & ~static_cast<size_t>(255); }

// workspace: [G m*m f64][gram slab][Sb m*256 f32][s d f32][part tiles*(m+1)*2 f64][AB (m+1)*2 f64][chosen K]
size_t attack_krum_workspace_bytes(int m, int64_t d, int K) {
  const size_t ntiles = static_cast<size_t>(cdiv(d, kAtkTile));
  return 256 + al256(static_cast<size_t>(m) * m * 8) + al256(gram_workspace_bytes(m, d)) +
         al256(static_cast<size_t>(m) * kAtkMaxClients * 4) + al256(static_cast<size_t>(d) * 4) +
         al256(ntiles * (m + 1) * 16) + al256(static_cast<size_t>(m + 1) * 16) + al256(static_cast<size_t>(K) * 4);
}

// ---------------------------------------------------------------------------
// Python's random (MT19937 of Modules/_randommodule.c) on the device
// ---------------------------------------------------------------------------
constexpr int kMtN = 624, kMtM = 397, kMtH = kMtN - kMtM;   // kMtH = 227

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t next, uint32_t far) {
  const uint32_t y = (cur & 0x80000000u) | (next & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// st = [624 state words][position], as random.getstate()[1].  Writes the
// nwords tempered outputs that nwords calls of genrand_uint32 return, and the
// advanced state.  One workgroup.  A twist is three data-parallel phases:
// words [0, 227) read only old words; [227, 454) also read the new words
// [0, 227); [454, 624) read new words [227, 397) (word 623 wraps to the new
// word 0).  Every phase reads its operands before a barrier and writes after it.
__global__ void __launch_bounds__(kAtkBS) mt19937_kernel(const uint32_t* __restrict__ st_in, int64_t nwords,
                                                         uint32_t* __restrict__ out, uint32_t* __restrict__ st_out) {
  __shared__ uint32_t mt[kMtN];
  const int tid = threadIdx.x;
  for (int i = tid; i < kMtN; i += kAtkBS) mt[i] = st_in[i];
  int pos = static_cast<int>(st_in[kMtN]);
  __syncthreads();
  // the rest of the current block
  const int64_t avail = pos < kMtN ? kMtN - pos : 0;
  int64_t done = avail < nwords ? avail : nwords;
  for (int64_t i = tid; i < done; i += kAtkBS) out[i] = mt_temper(mt[pos + i]);
  pos += static_cast<int>(done);
  while (done < nwords) {
#pragma unroll 1
    for (int ph = 0; ph < 3; ++ph) {
      const int kk = ph * kMtH + tid;
      const bool act = tid < kMtH && kk < kMtN;
      uint32_t v = 0;
      if (act) v = mt_mix(mt[kk], mt[kk + 1 < kMtN ? kk + 1 : 0], ph == 0 ? mt[kk + kMtM] : mt[kk - kMtH]);
      __syncthreads();
      if (act) mt[kk] = v;
      __syncthreads();
    }
    const int64_t take = nwords - done < kMtN ? nwords - done : kMtN;
    for (int64_t i = tid; i < take; i += kAtkBS) out[done + i] = mt_temper(mt[i]);
    done += take;
    pos = static_cast<int>(take);
  }
  for (int i = tid; i < kMtN; i += kAtkBS) st_out[i] = mt[i];
  if (tid == 0) st_out[kMtN] = static_cast<uint32_t>(pos);
}

// attack_trimmedmean per element, in the reference's nditer order (layers in
// order, C order within a layer; attack.py:170-197):
//   sign  = sign(0.0 + sum of the benign x, in order)           (fp64)
//   t_c   = p - x_c (fp32); bmax / bmin = np.amax / np.amin over benign c
//   r     = random() from words 2e, 2e+1 ((w0 >> 5) * 2^26 + (w1 >> 6)) / 2^53
//   (a,b) = sign < 0 ? (bmin > 0 ? (bmin/B, bmin) : (bmin*B, bmin))
//                    : (bmax > 0 ? (bmax, bmax*B) : (bmax, bmax/B))
//   v     = a + (b - a) * r, all in float32: NumPy >= 2 casts the Python
//           floats B and r to float32 against float32 operands (NEP 50)
//   out   = -(double) v + (double) p                               (fp64)
__global__ void __launch_bounds__(kAtkBS) attack_trimmedmean_kernel(const float* __restrict__ X, int64_t D,
                                                                    int64_t ldx, const int* __restrict__ rows,
                                                                    int nrows, const float* __restrict__ params,
                                                                    const uint32_t* __restrict__ words, float B,
                                                                    double* __restrict__ out) {
#pragma clang fp contract(off)   // numpy rounds every product and sum separately
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kAtkBS + threadIdx.x;
  if (e >= D) return;
  const float p = params[e];
  double acc = 0.0;
  float bmax = 0.f, bmin = 0.f;
  for (int r = 0; r < nrows; ++r) {
    const float x = X[static_cast<int64_t>(rows[r]) * ldx + e];
    acc += static_cast<double>(x);
    const float t = p - x;
    if (r == 0) {
      bmax = t;
      bmin = t;
    } else {
      // np.amax / np.amin propagate NaN
      bmax = (t > bmax || t != t) && bmax == bmax ? t : bmax;
      bmin = (t < bmin || t != t) && bmin == bmin ? t : bmin;
    }
  }
  const uint32_t w0 = words[2 * e], w1 = words[2 * e + 1];
  const double r = (static_cast<double>(w0 >> 5) * 67108864.0 + static_cast<double>(w1 >> 6)) *
                   (1.0 / 9007199254740992.0);
  float a, b;
  if (acc < 0.0) {
    a = bmin > 0.f ? bmin / B : bmin * B;
    b = bmin;
  } else {
    a = bmax;
    b = bmax > 0.f ? bmax * B : bmax / B;
  }
  const float v = a + (b - a) * static_cast<float>(r);
  out[e] = -static_cast<double>(v) + static_cast<double>(p);
}

// attack_xie: out = (w * sum_r X[rows[r]]) / cnt in the input precision
// (tmp = zeros_like; tmp += row ...; (-weight) * tmp / len(choices))
template <typename T>
__global__ void __launch_bounds__(kAtkBS) rowlist_scaled_sum_kernel(const T* __restrict__ X, int64_t d, int64_t ldx,
                                                                    const int* __restrict__ rows, int nrows, T w,
                                                                    T cnt, T* __restrict__ out) {
#pragma clang fp contract(off)
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kAtkBS + threadIdx.x;
  if (k >= d) return;
  T acc = T(0);
  for (int r = 0; r < nrows; ++r) acc += X[static_cast<int64_t>(rows[r]) * ldx + k];
  out[k] = (w * acc) / cnt;
}

}  // namespace sra

using namespace sra;

extern "C" int sra_attack_krum_workspace_bytes(int64_t m, int64_t d, double lower_bound, size_t* bytes) {
  SRA_REQUIRE(bytes != nullptr, SRA_ERR_ARG, "null bytes pointer");
  SRA_REQUIRE(m >= 2 && m <= kAtkMaxClients && d >= 1, SRA_ERR_UNSUPPORTED, "attack_krum supports 2 <= m <= %d",
              kAtkMaxClients);
  SRA_REQUIRE(lower_bound > 0.0, SRA_ERR_ARG, "lower_bound must be > 0 (the reference loop never ends otherwise)");
  *bytes = attack_krum_workspace_bytes(static_cast<int>(m), d, attack_krum_candidates(lower_bound));
  return SRA_OK;
}

// dir == nullptr: attack_krum's direction, the sign of the benign sum
// (attack.py:211-216); else the caller's (bulyan_attack_krum's attack_vec,
// attack.py:278-282).  The malicious rows are -lambda * dir.
static int attack_krum_impl(const float* X, int64_t m, int64_t d, int64_t ldx, const int32_t* mal_mask,
                            const int32_t* benign_rows, int32_t nbenign, const float* dir, double lower_bound,
                            double* mal_row, double* lam_out, int32_t* chosen_out, void* ws, size_t ws_bytes,
                            void* stream) {
  SRA_REQUIRE(X != nullptr && mal_mask != nullptr && benign_rows != nullptr && mal_row != nullptr &&
                  lam_out != nullptr && chosen_out != nullptr && ws != nullptr,
              SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(m >= 2 && m <= kAtkMaxClients, SRA_ERR_UNSUPPORTED, "attack_krum supports 2 <= m <= %d",
              kAtkMaxClients);
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx (%lld/%lld)", (long long)d, (long long)ldx);
  SRA_REQUIRE(nbenign >= 1 && nbenign < m, SRA_ERR_ARG, "attack_krum needs >= 1 benign and >= 1 malicious client");
  SRA_REQUIRE(lower_bound > 0.0, SRA_ERR_ARG, "lower_bound must be > 0");
  const int K = attack_krum_candidates(lower_bound);
  const int mi = static_cast<int>(m), nb = nbenign;
  const size_t need = attack_krum_workspace_bytes(mi, d, K);
  SRA_REQUIRE(ws_bytes >= need, SRA_ERR_WORKSPACE, "attack_krum workspace too small: need %zu bytes", need);
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* p = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~static_cast<uintptr_t>(255));
  double* G = reinterpret_cast<double*>(p);
  p += al256(static_cast<size_t>(mi) * mi * 8);
  char* slab = p;
  const size_t slab_bytes = gram_workspace_bytes(mi, d);
  p += al256(slab_bytes);
  float* Sb = reinterpret_cast<float*>(p);
  p += al256(static_cast<size_t>(mi) * kAtkMaxClients * 4);
  float* sg = reinterpret_cast<float*>(p);
  p += al256(static_cast<size_t>(d) * 4);
  const int64_t ntiles = cdiv(d, kAtkTile);
  double* part = reinterpret_cast<double*>(p);
  p += al256(static_cast<size_t>(ntiles) * (mi + 1) * 16);
  double* AB = reinterpret_cast<double*>(p);
  p += al256(static_cast<size_t>(mi + 1) * 16);
  int* chosen = reinterpret_cast<int*>(p);

  int rc;
  if (dir == nullptr) {
    hipLaunchKernelGGL(sign_sum_kernel, dim3(cdiv(d, kAtkBS)), dim3(kAtkBS), 0, s, X, d, ldx, benign_rows, nb, sg);
    rc = launch_status("sign_sum_kernel");
    if (rc) return rc;
  } else {
    SRA_HIP(hipMemcpyAsync(sg, dir, sizeof(float) * static_cast<size_t>(d), hipMemcpyDeviceToDevice, s));
  }
  rc = launch_gram(X, mi, d, ldx, G, slab, slab_bytes, s);
  if (rc) return rc;
  hipLaunchKernelGGL(sa_partial_kernel, dim3(ntiles, nb + 1), dim3(kAtkBS), 0, s, X, d, ldx, benign_rows, nb, sg,
                     part);
  rc = launch_status("sa_partial_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(sa_reduce_kernel, dim3(cdiv(nb + 1, 256)), dim3(256), 0, s, part, static_cast<int>(ntiles), nb,
                     AB);
  rc = launch_status("sa_reduce_kernel");
  if (rc) return rc;
  if (nb > 1) {
    hipLaunchKernelGGL(benign_rowsort_kernel, dim3(nb), dim3(kAtkBS), 0, s, G, mi, benign_rows, nb, Sb);
    rc = launch_status("benign_rowsort_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(attack_krum_search_kernel, dim3(K), dim3(kAtkBS), 0, s, Sb, AB, nb, mal_mask, mi, chosen);
  rc = launch_status("attack_krum_search_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(attack_krum_pick_kernel, dim3(1), dim3(1), 0, s, chosen, K, mal_mask, lam_out, chosen_out);
  rc = launch_status("attack_krum_pick_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(attack_krum_row_kernel, dim3(cdiv(d, kAtkBS)), dim3(kAtkBS), 0, s, sg, d, lam_out, mal_row);
  return launch_status("attack_krum_row_kernel");
}

extern "C" int sra_attack_krum_f32(const float* X, int64_t m, int64_t d, int64_t ldx, const int32_t* mal_mask,
                                   const int32_t* benign_rows, int32_t nbenign, double lower_bound, double* mal_row,
                                   double* lam_out, int32_t* chosen_out, void* ws, size_t ws_bytes, void* stream) {
  return attack_krum_impl(X, m, d, ldx, mal_mask, benign_rows, nbenign, nullptr, lower_bound, mal_row, lam_out,
                          chosen_out, ws, ws_bytes, stream);
}

extern "C" int sra_attack_krum_dir_f32(const float* X, int64_t m, int64_t d, int64_t ldx, const int32_t* mal_mask,
                                       const int32_t* benign_rows, int32_t nbenign, const float* dir,
                                       double lower_bound, double* mal_row, double* lam_out, int32_t* chosen_out,
                                       void* ws, size_t ws_bytes, void* stream) {
  SRA_REQUIRE(dir != nullptr, SRA_ERR_ARG, "null direction");
  return attack_krum_impl(X, m, d, ldx, mal_mask, benign_rows, nbenign, dir, lower_bound, mal_row, lam_out,
                          chosen_out, ws, ws_bytes, stream);
}

extern "C" int sra_mt19937_words(const uint32_t* state_in, int64_t nwords, uint32_t* words, uint32_t* state_out,
                                 void* stream) {
  SRA_REQUIRE(state_in != nullptr && state_out != nullptr && (nwords == 0 || words != nullptr), SRA_ERR_ARG,
              "null pointer");
  SRA_REQUIRE(nwords >= 0, SRA_ERR_ARG, "nwords must be >= 0");
  hipLaunchKernelGGL(mt19937_kernel, dim3(1), dim3(kAtkBS), 0, static_cast<hipStream_t>(stream), state_in, nwords,
                     words, state_out);
  return launch_status("mt19937_kernel");
}

extern "C" int sra_attack_trimmedmean_f32(const float* X, int64_t D, int64_t ldx, const int32_t* benign_rows,
                                          int32_t nbenign, const float* params, const uint32_t* words, double b,
                                          double* mal_row, void* stream) {
  SRA_REQUIRE(X != nullptr && benign_rows != nullptr && params != nullptr && words != nullptr && mal_row != nullptr,
              SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(D >= 1 && ldx >= D, SRA_ERR_SHAPE, "bad D/ldx");
  SRA_REQUIRE(nbenign >= 1, SRA_ERR_ARG, "attack_trimmedmean needs >= 1 benign client (np.amax of an empty set)");
  hipLaunchKernelGGL(attack_trimmedmean_kernel, dim3(cdiv(D, kAtkBS)), dim3(kAtkBS), 0,
                     static_cast<hipStream_t>(stream), X, D, ldx, benign_rows, nbenign, params, words,
                     static_cast<float>(b), mal_row);
  return launch_status("attack_trimmedmean_kernel");
}

template <typename T>
static int attack_xie_impl(const T* X, int64_t d, int64_t ldx, const int32_t* rows, int32_t nrows, double weight,
                           int64_t nchoices, T* out, void* stream) {
  SRA_REQUIRE(X != nullptr && out != nullptr && (nrows == 0 || rows != nullptr), SRA_ERR_ARG, "null pointer");
  SRA_REQUIRE(d >= 1 && ldx >= d, SRA_ERR_SHAPE, "bad d/ldx");
  SRA_REQUIRE(nrows >= 0 && nchoices >= 1, SRA_ERR_ARG, "need len(choices) >= 1");
  hipLaunchKernelGGL((rowlist_scaled_sum_kernel<T>), dim3(cdiv(d, kAtkBS)), dim3(kAtkBS), 0,
                     static_cast<hipStream_t>(stream), X, d, ldx, rows, nrows, static_cast<T>(-weight),
                     static_cast<T>(nchoices), out);
  return launch_status("rowlist_scaled_sum_kernel");
}

extern "C" int sra_attack_xie_f32(const float* X, int64_t d, int64_t ldx, const int32_t* rows, int32_t nrows,
                                  double weight, int64_t nchoices, float* out, void* stream) {
  return attack_xie_impl<float>(X, d, ldx, rows, nrows, weight, nchoices, out, stream);
}

extern "C" int sra_attack_xie_f64(const double* X, int64_t d, int64_t ldx, const int32_t* rows, int32_t nrows,
                                  double weight, int64_t nchoices, double* out, void* stream) {
  return attack_xie_impl<double>(X, d, ldx, rows, nrows, weight, nchoices, out, stream);
}
