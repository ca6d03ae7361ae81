// k6, round 5 — the spectral filters' one-wave solver (filterL2 and its MoM
// form; replaces the four-wave lanczos_solve_kernel).
//
// Reference: src/robust_estimator.py:144-175 (filterL2_: 2*int(eps*n)
// iterations of: weighted mean and covariance, top eigenpair by eigh, early
// exit if lambda^2 <= expansion * sigma^2, tau = ((x - mu).v)^2, c *= 1 -
// tau / tau_max, drop the argmax, c /= |c|_1) and :177-208 (the itv chunks).
//
// Client space as before: with w = c / sum(c), the weighted
// covariance's nonzero spectrum is that of M = W^1/2 C W^1/2, C the Gram of
// the rows centred at the weighted mean, and tau_i = (C W^1/2 u)_i^2 / lambda
// for M's top eigenpair (lambda, u).  What is new:
//
//  * ONE wave per chunk, four per CU (one per SIMD).  C is held in the
//    circulant-half form of wave_sym.hpp (lane l: rows 2l and 2l + 1, the 65
//    diagonals k = 0 .. 64; WKV of them in VGPRs, the rest in LDS), so a
//    matvec is 130 + 126 fp64 fmas and 126 DPP moves per lane, and every
//    reduction of the Lanczos step, the checks and the filter decision is a
//    DPP / readlane wave reduction: no workgroup barrier anywhere (the
//    four-wave solver paid two block reductions per Lanczos step, two
//    workgroups per CU).
//  * C is recentred in place every iteration instead of being rebuilt from
//    the chunk Gram G: with g = C w and s = w'g, C <- C - g 1' - 1 g' + s 1 1'
//    is (I - 1 w')C(I - w 1'), the Gram centred at the new weighted mean,
//    because (I - 1 w')(I - 1 w_old') = I - 1 w' when w'1 = 1.  G is read
//    once per chunk (the four-wave solver re-read its 128 KiB every
//    iteration: 78.6 GB per C4 call), and the entries stay centred at the
//    current weights, so forming them never cancels the offset of the
//    unweighted mean.  M is applied as W^1/2 C W^1/2 x (two scalings per
//    lane around the matvec).
//  * Lanczos basis vectors go to a per-wave global scratch (1 KiB per step,
//    off the step's critical path; read back once per iteration for the
//    Ritz vector).
//
// The Lanczos schedule is the four-wave solver's (plain three-term Lanczos,
// checks at residual-decay-extrapolated steps, acceptance at 2.5e-16 lambda,
// a ghost retries once with dense checks, then a re-orthogonalising attempt
// in the same kernel; a chunk that still fails is listed for
// filter_solve_kernel).  The check (top eigenpair of T_m) is fast_check's
// algorithm in one wave: Laguerre from the Gershgorin bound, multisection
// over 64 Sturm points per round, the two eigenvector recurrences of
// (T - theta) f = 0 interleaved in one instruction stream, the twist.
#include "filter_common.hpp"
#include "sra_common.hpp"
#include "wave_sym.hpp"

namespace sra {

constexpr int WKV = 36;                       // C's diagonals in VGPRs (the rest in LDS: four waves per CU fill it)
constexpr int WKL = wsym::NK - WKV;           // ... in LDS
constexpr int kExStride = 72;                 // check: exponents per block of 4 chain steps, per chain
constexpr int kWScr = 4 * MMAX + 2 * kExStride;   // operand (256) + group shifts (384) | check scratch
static_assert(kWScr >= wsym::kZd + wsym::kTb, "the check scratch overlays the matvec scratch");
constexpr int kWTrw = 2 * MMAX + 32;          // T record: (alpha_q, beta^2_{q-1}) pairs + prefetch padding
// LDS per wave: C's LDS diagonals, the matvec / check scratch, the T record,
// its reversed copy (the backward chain), the accepted check's eigenvector
constexpr size_t kWaveLds = sizeof(double) * (static_cast<size_t>(WKL) * FNP + kWScr + 2 * kWTrw + MMAX);
static_assert(4 * kWaveLds <= 163840, "four one-wave solvers must fit one CU's LDS");
constexpr int kWaveGrid = 1024;               // 4 waves per CU x 256 CUs; each owns a basis slot
constexpr double kEps = 1.1102230246251565e-16;       // unit roundoff
constexpr double kSqrtEps = 1.0536712127723509e-08;   // sqrt(kEps): the semi-orthogonality bound

// The pairs T2[q] = (alpha_q, beta^2 of (q-1, q)) for q = 1 .. m-1 into f, g()
// after every fourth: the next block's four LDS reads are issued before the
// current block's steps, so a serial chain (~30 cycles a step) does not wait
// on LDS latency (reads reach T2[m + 6], inside the record's padding).
template <typename F, typename G>
__device__ __forceinline__ void tstream(const double2* T2, int m, F&& f, G&& g) {
  double2 c0 = T2[1], c1 = T2[2], c2 = T2[3], c3 = T2[4];
  int q = 1;
  for (; q + 4 <= m; q += 4) {
    const double2 n0 = T2[q + 4], n1 = T2[q + 5], n2 = T2[q + 6], n3 = T2[q + 7];
    f(c0);
    f(c1);
    f(c2);
    f(c3);
    g();
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
  }
  if (q < m) f(c0);
  if (q + 1 < m) f(c1);
  if (q + 2 < m) f(c2);
}

// ---- the check: top Ritz pair of T_m in one wave ---------------------------
// T: LDS record, T[2q] = alpha_q, T[2q+1] = beta^2 of (q-1, q) (T[1] = 0).
// Returns theta (2-ulp bracket midpoint), the last component of the
// normalised eigenvector (the residual is beta_m |z_{m-1}|), and writes z[0, m).
__device__ __forceinline__ void wave_check(const double* T, int m, double theta_lb, double hint, double glo,
                                           double ghi, double* z, double* scr, double* trev, double* theta_out,
                                           double* zlast_out, int* rounds_out, long long* ph = nullptr) {
  m = __builtin_amdgcn_readfirstlane(m);
  long long tp = ph ? clock64() : 0;
  auto stamp = [&](int i) {   // debug builds: cycles per check phase
    if (ph) {
      const long long t = clock64();
      ph[i] += t - tp;
      tp = t;
    }
  };
  const int lane = threadIdx.x & 63;
  double* gq = scr;                  // [MMAX] g | [MMAX] Q  (forward chain)
  double* hr = scr + 2 * MMAX;       // [MMAX] h | [MMAX] R  (backward chain)
  double* ex = scr + 4 * MMAX;       // [kExStride] forward exponents | [kExStride] backward
  const double a0 = T[0];
  double lo = fmax(glo, fmax(theta_lb, a0));
  double hi = ghi;
  if (!(lo < hi)) lo = glo;
  const bool hinted = hint >= 0.0 && theta_lb > -1e299;
  const double hg = lo + 4.0 * hint + 4e-16 * fabs(lo);
  const double2* T2 = reinterpret_cast<const double2*>(T);
  // Sturm count at x: the number of eigenvalues below x (>= m: x is above all)
  auto count = [&](double x) -> int {
    double p2 = 1.0, p1 = a0 - x;
    unsigned cnt = static_cast<unsigned>(__builtin_bit_cast(unsigned long long, p1) >> 63);
    auto step = [&](double2 t) __attribute__((always_inline)) {
      const double pk = fma(t.x - x, p1, -(t.y * p2));
      cnt += static_cast<unsigned>((__builtin_bit_cast(unsigned long long, pk) ^
                                    __builtin_bit_cast(unsigned long long, p1)) >> 63);
      p2 = p1;
      p1 = pk;
    };
    tstream(T2, m, step, [&]() __attribute__((always_inline)) {
      const int e = __builtin_amdgcn_frexp_exp(p1);
      p1 = __builtin_amdgcn_ldexp(p1, -e);
      p2 = __builtin_amdgcn_ldexp(p2, -e);
    });
    return static_cast<int>(cnt);
  };
  // one multisection round: 64 Sturm points (one per lane) of the given kind
  // in [lo, hi]; returns true when the bracket is at two ulps (or stalled).
  // kind 0 uniform, 1 geometric above lo up to lo + 4 hint (hinted checks),
  // 2 geometric above lo over the whole bracket (cold), 3 the Laguerre bracket
  // with both ends included (verifies it; false + reset when it misses)
  const double lo0 = lo, hi0 = hi;
  bool laguerre = false;
  auto mround = [&](int kind) -> bool {
    const double rlo = lo, rhi = hi;
    auto point = [&](int p) -> double {
      if (kind == 1) return p < 63 ? rlo + (hg - rlo) * ((p + 1) * (1.0 / 63.0)) : rhi;
      if (kind == 2) return rlo + (rhi - rlo) * __builtin_amdgcn_ldexp(1.0, p - 63);
      if (kind == 3) return rlo + (rhi - rlo) * (p * (1.0 / 63.0));
      return rlo + (rhi - rlo) * ((p + 1) * (1.0 / 65.0));
    };
    const unsigned long long ok = __builtin_amdgcn_ballot_w64(count(point(lane)) >= m);
    const int first = ok ? __builtin_ctzll(ok) : 64;
    if (kind == 3 && (first == 0 || first == 64)) {   // not inside the Laguerre bracket
      lo = lo0;
      hi = hi0;
      laguerre = false;
      return false;
    }
    const double xf = first < 64 ? point(first) : rhi;
    const double xb = first > 0 ? point(first - 1) : rlo;
    const bool stalled = xb == lo && xf == hi;
    lo = xb;
    hi = xf;
    return stalled || hi - lo <= 4.5e-16 * fmax(fabs(lo), fabs(hi));
  };
  int round = 0;
  bool done = false;
  // cold start: two multisection rounds (geometric above the lower bound, then
  // uniform) bracket the top eigenvalue to ~1e-4 of the Gershgorin range, then
  // Laguerre from the bracket's top (above the spectrum: it decreases
  // monotonically to the top eigenvalue, cubically this close), then one
  // round over +-64 ulps verifies it
  if (!hinted && m > 2) {
    done = mround(2);
    ++round;
    if (!done) {
      done = mround(0);
      ++round;
    }
    if (!done) {
      const double llo = lo;
      double x = hi;
      for (int itl = 0; itl < 16; ++itl) {
        double p0 = 1.0, p1 = x - a0, d0 = 0.0, d1 = 1.0, e0 = 0.0, e1 = 0.0;
        auto lstep = [&](double2 t) __attribute__((always_inline)) {
          const double c = x - t.x;
          const double pn = fma(c, p1, -(t.y * p0));
          const double dn = fma(c, d1, p1 - t.y * d0);
          const double en = fma(c, e1, 2.0 * d1 - t.y * e0);
          p0 = p1; p1 = pn;
          d0 = d1; d1 = dn;
          e0 = e1; e1 = en;
        };
        tstream(T2, m, lstep, [&]() __attribute__((always_inline)) {
          const int e = __builtin_amdgcn_frexp_exp(fmax(fabs(p1), fabs(d1)));
          p0 = __builtin_amdgcn_ldexp(p0, -e); p1 = __builtin_amdgcn_ldexp(p1, -e);
          d0 = __builtin_amdgcn_ldexp(d0, -e); d1 = __builtin_amdgcn_ldexp(d1, -e);
          e0 = __builtin_amdgcn_ldexp(e0, -e); e1 = __builtin_amdgcn_ldexp(e1, -e);
        });
        if (!(p1 != 0.0)) break;
        const double G = d1 / p1, H = G * G - e1 / p1;
        const double nn = static_cast<double>(m);
        const double den = G + sqrt(fmax((nn - 1.0) * (nn * H - G * G), 0.0));
        const double xn = x - nn / den;
        if (!(xn < x) || !(xn >= llo)) break;
        const bool fin = x - xn <= 4e-16 * fabs(x);
        x = xn;
        if (fin) break;
      }
      const double u = 64.0 * 2.2204460492503131e-16 * fabs(x);
      if (x - u > lo && x + u < hi) {
        lo = x - u;
        hi = x + u;
        laguerre = true;
      }
    }
  }
  stamp(0);
  for (; !done && round < 48; ++round) {
    const int kind = laguerre ? 3 : (hinted && hg < hi && round == 0 ? 1 : 0);
    const bool was_l = laguerre;
    done = mround(kind);
    if (was_l) laguerre = false;
  }
  const double lm = 0.5 * (lo + hi);
  stamp(1);
  // ---- the two eigenvector recurrences of (T - lm) f = 0 in the division-
  // free minor form (fast_check), forward from the top and backward from the
  // bottom, rescaled by powers of two every four steps.  Round 5: lanes 0-31
  // run the forward chain on T, lanes 32-63 the same code on the reversed
  // record T'2[q] = (alpha_{m-1-q}, beta^2_{m-q}) -- the backward recurrence
  // is the forward one of J T J -- so one instruction stream carries both
  // chains (half the issue slots of running both in every lane)
  {
    const bool fwd = lane < 32;
    double2* Tr2 = reinterpret_cast<double2*>(trev);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int q = lane + 64 * s2;
      if (q < m) Tr2[q] = double2{T[2 * (m - 1 - q)], q > 0 ? T[2 * (m - q) + 1] : 0.0};
      else if (q < m + 8) Tr2[q] = double2{0.0, 0.0};   // the prefetch padding
    }
    wsym::lds_order();
    const double2* S2 = fwd ? T2 : Tr2;
    double* v = fwd ? gq : hr;                        // [MMAX] g | [MMAX] Q, or h | R
    double* exs = fwd ? ex : ex + kExStride;
    // the value of step k lands at k + 1 (forward) / m - 2 - k (backward)
    const int i0 = fwd ? 1 : m - 2, di = fwd ? 1 : -1;
    const bool wr = lane == 0 || lane == 32;          // one writer per chain
    double g1 = 1.0, g0 = 0.0, qv = 1.0;
    int eg = 0, eq = 0;
    if (wr) {
      exs[0] = exs[1] = 0.0;
      v[fwd ? 0 : m - 1] = 1.0;
      v[MMAX + (fwd ? 0 : m - 1)] = 1.0;
    }
    double2 c = S2[0];
    auto step = [&](double2 nx) __attribute__((always_inline)) {
      const double gn = fma(lm - c.x, g1, -(c.y * g0));
      qv *= nx.y;
      g0 = g1;
      g1 = gn;
      c = nx;
    };
    auto rescale_values = [&]() __attribute__((always_inline)) {
      int e = __builtin_amdgcn_frexp_exp(g1);
      g1 = __builtin_amdgcn_ldexp(g1, -e);
      g0 = __builtin_amdgcn_ldexp(g0, -e);
      eg += e;
      e = __builtin_amdgcn_frexp_exp(qv);
      qv = __builtin_amdgcn_ldexp(qv, -e);
      eq += e;
    };
    const int steps = m - 1;
    double2 f0 = S2[1], f1 = S2[2], f2 = S2[3], f3 = S2[4];
    int k = 0;
    for (; k + 4 <= steps; k += 4) {
      const double2 n0 = S2[k + 5], n1 = S2[k + 6], n2 = S2[k + 7], n3 = S2[k + 8];
      double sg[4], sq[4];
      step(f0);
      sg[0] = g1; sq[0] = qv;
      step(f1);
      sg[1] = g1; sq[1] = qv;
      step(f2);
      sg[2] = g1; sq[2] = qv;
      step(f3);
      rescale_values();
      sg[3] = g1; sq[3] = qv;
      if (wr) {
        const int ib = i0 + di * k;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[ib + di * u] = sg[u];
          v[MMAX + ib + di * u] = sq[u];
        }
        const int b = 2 * ((k + 4) >> 2);
        exs[b] = static_cast<double>(eg);
        exs[b + 1] = static_cast<double>(eq);
      }
      f0 = n0; f1 = n1; f2 = n2; f3 = n3;
    }
    if (k < steps) {
      step(f0);
      if (wr) { v[i0 + di * k] = g1; v[MMAX + i0 + di * k] = qv; }
    }
    if (k + 1 < steps) {
      step(f1);
      if (wr) { v[i0 + di * (k + 1)] = g1; v[MMAX + i0 + di * (k + 1)] = qv; }
    }
    if (k + 2 < steps) {
      step(f2);
      if (wr) { v[i0 + di * (k + 2)] = g1; v[MMAX + i0 + di * (k + 2)] = qv; }
    }
  }
  wsym::lds_order();   // every lane reads its neighbours' chain values
  stamp(2);
  auto pexp = [&](const double* exb, int p, int which) -> int { return static_cast<int>(exb[2 * (p >> 2) + which]); };
  const double* exf = ex;
  const double* exb = ex + kExStride;
  // ---- gamma, twist (first index of the smallest |gamma|), z
  double zv[2], gam = 1e308;
  int tw = 0;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int k = lane + 64 * s2;
    zv[s2] = 0.0;
    if (k < m) {
      double g = T[2 * k] - lm;
      if (k > 0)
        g += T[2 * k + 1] * __builtin_amdgcn_ldexp(gq[k - 1] * rcp_nr(gq[k]), pexp(exf, k - 1, 0) - pexp(exf, k, 0));
      if (k + 1 < m)
        g += T[2 * k + 3] *
             __builtin_amdgcn_ldexp(hr[k + 1] * rcp_nr(hr[k]), pexp(exb, m - 2 - k, 0) - pexp(exb, m - 1 - k, 0));
      const double ga = fabs(g);
      if (ga < gam) {
        gam = ga;
        tw = k;
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double og = __shfl_xor(gam, off);
    const int ot = __shfl_xor(tw, off);
    if (og < gam || (og == gam && ot < tw)) {
      gam = og;
      tw = ot;
    }
  }
  tw = __builtin_amdgcn_readfirstlane(tw);
  const double igr = rcp_nr(gq[tw]), ihr = rcp_nr(hr[tw]);
  const double qr = gq[MMAX + tw], rr = hr[MMAX + tw];
  const int egr = pexp(exf, tw, 0), eqr = pexp(exf, tw, 1);
  const int ehr = pexp(exb, m - 1 - tw, 0), err = pexp(exb, m - 1 - tw, 1);
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int k = lane + 64 * s2;
    if (k < m) {
      if (k <= tw) {   // (g_k / g_r) sqrt(Q_r / Q_k)
        int e2 = eqr - pexp(exf, k, 1);
        double qratio = qr * rcp_nr(gq[MMAX + k]);
        if (e2 & 1) { qratio *= 2.0; e2 -= 1; }
        zv[s2] = __builtin_amdgcn_ldexp(gq[k] * igr * sqrt(qratio), pexp(exf, k, 0) - egr + e2 / 2);
      } else {         // (h_k / h_r) sqrt(R_r / R_k)
        int e2 = err - pexp(exb, m - 1 - k, 1);
        double rratio = rr * rcp_nr(hr[MMAX + k]);
        if (e2 & 1) { rratio *= 2.0; e2 -= 1; }
        zv[s2] = __builtin_amdgcn_ldexp(hr[k] * ihr * sqrt(rratio), pexp(exb, m - 1 - k, 0) - ehr + e2 / 2);
      }
    }
  }
  const double inv = 1.0 / sqrt(wave_sum(zv[0] * zv[0] + zv[1] * zv[1]));
  if (lane < m) z[lane] = zv[0] * inv;
  if (lane + 64 < m) z[lane + 64] = zv[1] * inv;
  wsym::lds_order();
  stamp(3);
  *zlast_out = rl_any(zv, m - 1) * inv;
  *theta_out = lm;
  *rounds_out = round + 1;
}

// ---- C <- C - g 1' - 1 g' + s 1 1' on the packed form ----------------------
// zd holds g doubled; ri_s = s - g_row.  Entry (m, m + k): (C + ri) - g_{m+k}
template <int KV>
__device__ __forceinline__ void recentre(wsym::Packed<KV>& P, double* cl, const double* zd, double ri0, double ri1) {
  const int lane = threadIdx.x & 63;
  const double2* xp = reinterpret_cast<const double2*>(zd) + lane;
  wsym::sfor<wsym::NK>([&](auto K) {
    constexpr int k = decltype(K)::value;
    constexpr int j = k / 2;
    double gj0, gj1;
    if constexpr ((k & 1) == 0) {
      const double2 X = xp[j];
      gj0 = X.x;
      gj1 = X.y;
    } else {
      gj0 = xp[j].y;
      gj1 = xp[j + 1].x;
    }
    if constexpr (k < KV) {
      P.cv[k][0] = (P.cv[k][0] + ri0) - gj0;
      P.cv[k][1] = (P.cv[k][1] + ri1) - gj1;
    } else {
      double2* c = reinterpret_cast<double2*>(cl + (k - KV) * FNP) + lane;
      const double2 v = *c;
      *c = double2{(v.x + ri0) - gj0, (v.y + ri1) - gj1};
    }
  });
}

// first index of the largest value over the wave (value, index) pairs
__device__ __forceinline__ int wave_argmax_first(double v, int i, double* vbest) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ov = __shfl_xor(v, off);
    const int oi = __shfl_xor(i, off);
    if (ov > v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
  *vbest = readlane_f64(v, 0);
  return __builtin_amdgcn_readfirstlane(i);
}

// ---- eight wave sums at once ------------------------------------------------
// h[i] = sum over the wave of p[i], wave-uniform.  A reduce-scatter halves the
// values per lane at every level -- v_permlane32_swap (lane ^ 32), then
// v_permlane16_swap (rows 0/2 vs 1/3), then DPP row_ror:8 (lane ^ 8) -- so
// the last three levels are one value's DPP sum over eight lanes, and value
// i ends in lanes 8i .. 8i + 7 (13 cross-lane moves and adds per value pair
// instead of wave_sum's 8 DPP moves + 8 readlanes per value).
__device__ __forceinline__ void swap_rows(double& a, double& b, bool wide) {
  const unsigned long long ua = __builtin_bit_cast(unsigned long long, a), ub = __builtin_bit_cast(unsigned long long, b);
  const unsigned al = static_cast<unsigned>(ua), ah = static_cast<unsigned>(ua >> 32);
  const unsigned bl = static_cast<unsigned>(ub), bh = static_cast<unsigned>(ub >> 32);
  unsigned nal, nah, nbl, nbh;
  if (wide) {   // lanes 32-63 of a <-> lanes 0-31 of b
    const auto lo = __builtin_amdgcn_permlane32_swap(al, bl, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(ah, bh, false, false);
    nal = lo[0]; nbl = lo[1]; nah = hi[0]; nbh = hi[1];
  } else {      // odd rows of a <-> even rows of b
    const auto lo = __builtin_amdgcn_permlane16_swap(al, bl, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
    nal = lo[0]; nbl = lo[1]; nah = hi[0]; nbh = hi[1];
  }
  a = __builtin_bit_cast(double, (static_cast<unsigned long long>(nah) << 32) | nal);
  b = __builtin_bit_cast(double, (static_cast<unsigned long long>(nbh) << 32) | nbl);
}

__device__ __forceinline__ void wave_sum8(const double (&p)[8], double (&h)[8]) {
  const int lane = threadIdx.x & 63;
  double q[4], r[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // lanes < 32: value i, lanes >= 32: value i + 4
    double a = p[i], b = p[i + 4];
    swap_rows(a, b, true);
    q[i] = a + b;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {   // even rows: q[i]'s value, odd rows: q[i + 2]'s
    double a = q[i], b = q[i + 2];
    swap_rows(a, b, false);
    r[i] = a + b;
  }
  // lanes 0-7 of a row keep r[0], lanes 8-15 keep r[1]; each takes the other
  // half's copy of the value it keeps
  const bool upper = (lane & 8) != 0;
  const double keep = upper ? r[1] : r[0], send = upper ? r[0] : r[1];
  double v = keep + dpp_f64<0x128>(send);   // row_ror:8
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = readlane_f64(v, 8 * i);
}

// ---- ex_noregret's KL projection, one wave (kl_project_t in filter.hip) ---
// {c : sum c = 1, c <= cap} over the nk kept clients (robust_estimator.py:
// 74-99): candidate i caps the i + 1 largest weights and rescales the rest;
// the feasible candidate with the smallest KL wins (first on ties), the
// reference's loop stops at the first infeasible clip.  Lane l: rows 2l,
// 2l + 1 and the compact entries / candidates l, l + 64.  scr: 512 doubles.
// Returns false when no candidate is feasible (projected_c = None, :99).
__device__ bool wave_kl_project(double& c0, double& c1, bool ai0, bool ai1, int nk, double cap, double* scr,
                                int* capped) {
  const int lane = threadIdx.x & 63;
  double* cc = scr;                                      // [FNP] compact weights
  double* sv = scr + FNP;                                // [FNP] weights in descending order
  double* hl = scr + 2 * FNP;                            // [FNP] sv log(sv / cap)
  int* irank = reinterpret_cast<int*>(scr + 3 * FNP);    // [FNP] descending rank of a compact entry
  const unsigned long long m0 = __builtin_amdgcn_ballot_w64(ai0), m1 = __builtin_amdgcn_ballot_w64(ai1);
  const unsigned long long below = (1ull << lane) - 1ull;
  const int pos0 = __builtin_popcountll(m0 & below) + __builtin_popcountll(m1 & below);
  const int pos1 = pos0 + (ai0 ? 1 : 0);
  wsym::lds_order();
  if (ai0) cc[pos0] = c0;
  if (ai1) cc[pos1] = c1;
  wsym::lds_order();
  // descending rank; ties: later compact index first (flip of a stable ascending argsort)
  const int t0 = lane, t1 = lane + 64;
  const double v0 = t0 < nk ? cc[t0] : 0.0, v1 = t1 < nk ? cc[t1] : 0.0;
  int rk0 = 0, rk1 = 0;
  for (int q = 0; q < nk; ++q) {
    const double cq = cc[q];
    rk0 += (cq > v0 || (cq == v0 && q > t0)) ? 1 : 0;
    rk1 += (cq > v1 || (cq == v1 && q > t1)) ? 1 : 0;
  }
  if (t0 < nk) {
    irank[t0] = rk0;
    sv[rk0] = v0;
    hl[rk0] = v0 * log(v0 / cap);
  }
  if (t1 < nk) {
    irank[t1] = rk1;
    sv[rk1] = v1;
    hl[rk1] = v1 * log(v1 / cap);
  }
  wsym::lds_order();
  double negkl[2] = {-__builtin_inf(), -__builtin_inf()}, scale[2] = {0.0, 0.0};
  int stop = 1 << 30;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int i = lane + 64 * s;
    if (i < nk) {
      const double clip = 1.0 - np_pw64(0, i + 1, [&](int) { return cap; });
      if (clip <= 0.0) {
        stop = stop < i ? stop : i;
      } else if (i + 1 < nk) {
        const double norm = np_pw64(i + 1, nk - i - 1, [&](int q) { return sv[q]; });
        scale[s] = clip / norm;
        if (!(sv[i + 1] * scale[s] > cap)) {
          double head = 0.0;
          for (int q = 0; q <= i; ++q) head += hl[q];
          negkl[s] = -(head - norm * log(scale[s]));
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int o2 = __shfl_xor(stop, off);
    stop = o2 < stop ? o2 : stop;
  }
  stop = __builtin_amdgcn_readfirstlane(stop);
  if (lane >= stop) negkl[0] = -__builtin_inf();
  if (lane + 64 >= stop) negkl[1] = -__builtin_inf();
  const bool take1 = negkl[1] > negkl[0];   // ties: the lower candidate index
  double best;
  const int bi = wave_argmax_first(take1 ? negkl[1] : negkl[0], take1 ? lane + 64 : lane, &best);
  const bool ok = best > -__builtin_inf();
  *capped = ok ? bi + 1 : 0;
  if (ok) {
    const double sb = readlane_f64(bi < 64 ? scale[0] : scale[1], bi & 63);
    if (ai0) c0 = irank[pos0] <= bi ? cap : cc[pos0] * sb;
    if (ai1) c1 = irank[pos1] <= bi ? cap : cc[pos1] * sb;
  }
  wsym::lds_order();   // the scratch is the next check's
  return ok;
}

// out[j] = sum_i kept c_i x_ij / scale over the chunk's coordinates in fp64
// with the clients in order (chunk_mean_kernel's arithmetic, bit-identical);
// unweighted (ex_noregret's None exit): the fp32 mean.  cv / kf: the weights
// and kept flags in LDS.  A lane per coordinate, sixteen per pass in flight.
__device__ __attribute__((noinline)) void chunk_means(const float* Xm, int64_t ldxm, int64_t jx0, int64_t gj0, int itv,
                                                      int64_t d, int n, const double* cv, const double* kf,
                                                      double scale, bool unw, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t gj1 = gj0 + itv < d ? gj0 + itv : d;
  const int kk = static_cast<int>(gj1 - gj0);
  const float* xb = Xm + (gj0 - jx0);
  for (int jb = 0; jb < kk; jb += 16 * 64) {
    double acc[16];
    float acc32[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      acc[t] = 0.0;
      acc32[t] = 0.f;
    }
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
      if (kf[i] == 0.0) continue;   // wave-uniform
      const double ci = cv[i];
      ++cnt;
      const float* xr = xb + static_cast<int64_t>(i) * ldxm;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int jj = jb + 64 * t + lane;
        const float x = jj < kk ? xr[jj] : 0.f;
        if (unw) acc32[t] += x;
        else acc[t] += static_cast<double>(x) * ci;
      }
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int jj = jb + 64 * t + lane;
      if (jj < kk) out[gj0 + jj] = unw ? static_cast<double>(acc32[t] / static_cast<float>(cnt)) : acc[t] / scale;
    }
  }
}

template <int MODE, bool DBG>
__global__ void __launch_bounds__(64, 1) wave_solve_kernel(SolveArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* cl = reinterpret_cast<double*>(smem);   // [WKL][FNP] C's LDS diagonals
  double* scr = cl + WKL * FNP;                   // [kWScr] operand + group shifts | check scratch
  double* zd = scr;
  double* tb = scr + wsym::kZd;
  double* trw = scr + kWScr;                      // [kWTrw] tridiagonal record
  double* trev = trw + kWTrw;                     // [kWTrw] the record reversed (wave_check)
  double* zbuf = trev + kWTrw;                    // [MMAX] eigenvector of T_m of the last check
  const int lane = threadIdx.x;
  const int r0 = 2 * lane, r1 = r0 + 1;
  const int n = A.n;
  double* Vb = A.Vg + static_cast<size_t>(blockIdx.x) * (MMAX + 1) * FNP;
  if (lane < 32) trw[2 * MMAX + lane] = 0.0;   // prefetch padding of the T record

  for (;;) {
    int ch = lane == 0 ? atomicAdd(A.fb_count + 4, 1) : 0;
    ch = __builtin_amdgcn_readfirstlane(ch);
    if (ch >= A.nb) break;
    const bool dbg = DBG && ch == 0;
    // ---- C = G (the chunk Gram, centred at the unweighted mean) into the packed form
    wsym::Packed<WKV> P;
    {
      const double* Gc = A.G + static_cast<size_t>(ch) * FNP * FNP;
      wsym::sfor<wsym::NK>([&](auto K) {
        constexpr int k = decltype(K)::value;
        const double v0 = Gc[r0 * FNP + ((r0 + k) & (FNP - 1))];
        const double v1 = Gc[r1 * FNP + ((r1 + k) & (FNP - 1))];
        if constexpr (k < WKV) {
          P.cv[k][0] = v0;
          P.cv[k][1] = v1;
        } else {
          reinterpret_cast<double2*>(cl + (k - WKV) * FNP)[lane] = double2{v0, v1};
        }
      });
    }
    bool ai0 = r0 < n, ai1 = r1 < n;
    if constexpr (MODE == 1) {   // the kept set of the pre-filter (noregret_pre_kernel)
      const int2 a2 = reinterpret_cast<const int2*>(A.act + static_cast<size_t>(ch) * FNP)[lane];
      ai0 = ai0 && a2.x != 0;
      ai1 = ai1 && a2.y != 0;
    }
    double ci0 = ai0 ? 1.0 : 0.0, ci1 = ai1 ? 1.0 : 0.0;
    const int fdrop = static_cast<int>(ceil(A.eps * n));
    const int n_keep = MODE == 1 ? n - (fdrop < n ? fdrop : n) : n;
    const double step = MODE == 1 ? A.misc[static_cast<size_t>(ch) * kMisc + 1] : 0.0;
    const int iters = MODE == 0 ? 2 * static_cast<int>(A.eps * n) : static_cast<int>(2 * A.eps * n_keep);
    // ex_noregret: projected_c = None (no feasible candidate, :99): the next
    // iteration runs with weights=None (the plain mean and covariance,
    // :65-67) and either exits with that mean (:71-72) or fails at
    // c * (1 - step * tau) (:75, TypeError); at the last iteration the final
    // np.average(weights=None) returns it (:101)
    bool none = false, unweighted = false, have_u = false;
    double u0 = 0.0, u1 = 0.0;   // the last Ritz vector (rows 2 lane, 2 lane + 1)
    int m_hint = MODE == 1 ? 12 : 24;
    double rate_hint = 0.0;
    bool fallback = false;
    int done = 0;
    int* tr = A.trace != nullptr ? A.trace + static_cast<size_t>(ch) * kTraceStride : nullptr;
    const double hh0 = 0.5 + (r0 * 0.6180339887498949 - floor(r0 * 0.6180339887498949));
    const double hh1 = 0.5 + (r1 * 0.6180339887498949 - floor(r1 * 0.6180339887498949));

    for (int it = 0; it < iters; ++it) {
      const long long t_it = dbg ? clock64() : 0;
      if (MODE == 1 && none) {
        ci0 = ai0 ? 1.0 : 0.0;
        ci1 = ai1 ? 1.0 : 0.0;
      }
      // ---- weights, and C recentred at the weighted mean
      const double csum = wave_sum((ai0 ? ci0 : 0.0) + (ai1 ? ci1 : 0.0));
      const int nact = static_cast<int>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(ai0)) +
                                        __builtin_popcountll(__builtin_amdgcn_ballot_w64(ai1)));
      const double w0 = ai0 ? ci0 / csum : 0.0, w1 = ai1 ? ci1 / csum : 0.0;
      const double sw0 = sqrt(w0 > 0.0 ? w0 : 0.0), sw1 = sqrt(w1 > 0.0 ? w1 : 0.0);
      double sgw;
      {
        double g0, g1;
        wsym::put_operand(zd, w0, w1);
        wsym::matvec<WKV>(P, cl, zd, tb, w0, w1, g0, g1);
        sgw = wave_sum(w0 * g0 + w1 * g1);
        wsym::put_operand(zd, g0, g1);
        recentre<WKV>(P, cl, zd, sgw - g0, sgw - g1);
      }

      // ---- top eigenpair of M = W^1/2 C W^1/2 by plain Lanczos
      double lam = 0.0, resid = 0.0;
      int m_conv = 0, nchecks = 0, m_retry = 0;
      bool converged = false;
      double tscale = 0.0;
      long long tcheck = 0, tmv = 0, tstep = 0, tph[4] = {0, 0, 0, 0};
      int trounds = 0;
      // attempt 0: plain Lanczos; 1: after a ghost, again with dense checks;
      // 2: with full re-orthogonalisation against the stored basis
      // ex_noregret (MODE 1) re-orthogonalises from the start: its weights
      // integrate every iteration's eigenvector and its top two eigenvalues
      // close in (gaps ~1e-3 after a few iterations), where plain Lanczos
      // stalled above the accuracy floor
      // block Gram-Schmidt of r~ = (n0, n1) against q_0 .. q_j, eight vectors
      // per block (one wave_sum8 for their coefficients, then their update, so
      // a block is read once per pass); q_j from registers, the others read
      // back from the scratch (a lane reads only the entries it stored:
      // program order suffices).  A second pass when |r|^2 drops below half
      // (DGKS: |r - V h|^2 = |r|^2 - |h|^2); alpha takes the q_j coefficients.
      int ngs = 0;   // debug records: full Gram-Schmidt calls
      auto gs = [&](int j, double q0, double q1, double& n0, double& n1, double& aj) {
        if (DBG) ++ngs;
        const double2* V2 = reinterpret_cast<const double2*>(Vb);
        for (int pass = 0; pass < 2; ++pass) {
          const double nb2 = wave_sum(n0 * n0 + n1 * n1);
          double hn2 = 0.0;
          // the next block's loads are issued before this block's reduction
          // (the basis is in the Infinity Cache: one latency per pass, not per block)
          double2 raw[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) raw[u] = V2[(u < j ? u : 0) * 64 + lane];
          for (int qb = 0; qb <= j; qb += 8) {
            double2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int q = qb + u;
              v[u] = q < j ? raw[u] : (q == j ? double2{q0, q1} : double2{0.0, 0.0});
            }
            if (qb + 8 <= j) {
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int q = qb + 8 + u;
                raw[u] = V2[(q < j ? q : 0) * 64 + lane];
              }
            }
            double p[8], h[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) p[u] = fma(v[u].x, n0, v[u].y * n1);
            wave_sum8(p, h);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              n0 = fma(-h[u], v[u].x, n0);
              n1 = fma(-h[u], v[u].y, n1);
              hn2 = fma(h[u], h[u], hn2);
              aj += qb + u == j ? h[u] : 0.0;
            }
          }
          if (!(pass == 0 && nb2 - hn2 < kDgks * nb2)) break;
        }
      };
      for (int attempt = 0; attempt < 3 && !converged; ++attempt) {
        const bool full = attempt == 2;            // full re-orthogonalisation every step
        const bool pro = MODE == 1 && !full;       // partial (omega recurrence)
        const bool reorth = full || pro;
        const double acc = MODE == 1 ? kResTol : kAccept;
        // ex_noregret damps the top direction gently: the previous Ritz vector
        // (perturbed) is a near-eigenvector of the next M
        const bool warm = MODE == 1 && have_u && attempt == 0;
        double rt0 = sw0 > 0.0 ? (warm ? u0 + 1e-3 * sw0 * hh0 : sw0 * hh0) : 0.0;
        double rt1 = sw1 > 0.0 ? (warm ? u1 + 1e-3 * sw1 * hh1 : sw1 * hh1) : 0.0;
        double qp0 = 0.0, qp1 = 0.0, theta_lb = -1e300, hint = -1.0;
        double res_best = 1e300, lam_best = 0.0;
        tscale = 0.0;
        double gfin_hi = -1e300, gfin_lo = 1e300, a_last = 0.0, b_prev = 0.0;
        const int adv_max = attempt == 1 ? 1 : A.max_adv;
        const int off = MODE == 1 ? -1 : A.first_off;
        const int first = m_hint + off > 4 ? m_hint + off : 4;
        int next_check = attempt == 1 ? (m_retry > 4 ? m_retry : 4) : first;
        int m_a = -1, m_last = 4, m_pre = 4;
        double res_a = 0.0;
        bool ghost = false;
        // PRO state: |r~_j|^2 (computed at the end of step j - 1), and per lane
        // k = lane, lane + 64: omega_{j,k}, omega_{j-1,k}, alpha_k, beta_k, beta_{k+1}
        double nrm_c = pro ? wave_sum(rt0 * rt0 + rt1 * rt1) : 0.0;
        double oc[2] = {lane == 0 ? 1.0 : 0.0, 0.0}, op[2] = {0.0, 0.0};
        double al[2] = {0.0, 0.0}, be[2] = {0.0, 0.0}, be1[2] = {0.0, 0.0};
        bool force = false;
        // omega_{j+1,k} = (beta_{k+1} omega_{j,k+1} + (alpha_k - alpha_j) omega_{j,k}
        //   + beta_k omega_{j,k-1} - beta_j omega_{j-1,k}) / beta_{j+1}, grown by
        // eps (beta_{k+1} + beta_{j+1}) / beta_{j+1}; omega_{j+1,j} = eps sqrt(n) |T| /
        // beta_{j+1}.  Returns max_k<=j |omega_{j+1,k}| and shifts the rows.
        auto omega_step = [&](int j, double aj, double bj, double bn, double tn) -> double {
          // neighbours by DPP wave rotations (no LDS round trip)
          const double u0 = wsym::rol1(oc[0]), u1 = wsym::rol1(oc[1]);
          const double d0 = wsym::ror1(oc[0]), d1 = wsym::ror1(oc[1]);
          const double kp[2] = {lane < 63 ? u0 : u1, lane < 63 ? u1 : 0.0};
          const double km[2] = {lane > 0 ? d0 : 0.0, lane > 0 ? d1 : d0};
          const double ibn = 1.0 / bn;
          const double psi = kEps * sqrt(static_cast<double>(nact)) * tn * ibn;
          double mx = 0.0;
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int k = lane + 64 * s2;
            double w = (be1[s2] * kp[s2] + (al[s2] - aj) * oc[s2] + be[s2] * km[s2] - bj * op[s2]) * ibn;
            w += copysign(kEps * (be1[s2] + bn) * ibn, w);
            w = k < j ? w : (k == j ? psi : (k == j + 1 ? 1.0 : 0.0));
            mx = k <= j ? fmax(mx, fabs(w)) : mx;
            op[s2] = oc[s2];
            oc[s2] = w;
          }
          return wave_max(mx);
        };
        // Step j: y = M r~_j (r~_j = beta_j q_j, deferred normalisation), and
        // beta_j^2 = |r~_j|^2, its square root and reciprocal in the same basic
        // block (the reduction overlaps the matvec), then alpha_j and r~_{j+1};
        // the check of T_j (m = j, residual beta_j |z_{j-1}|) runs after that,
        // so no branch separates the matvec from the reduction, and a check
        // that accepts has spent one step for nothing.
        for (int j = 0;; ++j) {
          const long long ts0 = dbg ? clock64() : 0;
          // beta_j first in program order: its reduction, root and reciprocal
          // depend only on r~_j, so they fill the matvec's latency gaps
          const double nrm2 = pro ? nrm_c : wave_sum(rt0 * rt0 + rt1 * rt1);
          const double bet = sqrt(nrm2);
          const double ib = 1.0 / bet;
          double my0, my1;   // (M r~_j) = W^1/2 C W^1/2 r~_j
          {
            const double z0 = sw0 * rt0, z1 = sw1 * rt1;
            double y0, y1;
            wsym::put_operand(zd, z0, z1);
            wsym::matvec<WKV>(P, cl, zd, tb, z0, z1, y0, y1);
            my0 = sw0 * y0;
            my1 = sw1 * y1;
          }
          // alpha_j beta_j^2 = r~_j . M r~_j: reduced without waiting for 1/beta_j
          const double pa = wave_sum(rt0 * my0 + rt1 * my1);
          const long long ts1 = dbg ? clock64() : 0;
          if (dbg) tmv += ts1 - ts0;
          trw[2 * j + 1] = nrm2;   // every lane stores the same value (no exec-mask branch); T[1] is never used
          tscale = j > 0 ? fmax(tscale, bet) : tscale;
          const bool breakdown = j > 0 && !(bet > 1e-14 * tscale);
          // with re-orthogonalisation T_nact is exact (the Krylov space of the
          // active rows is exhausted)
          const bool exhausted = full && j >= nact;
          const bool do_check = j > 0 && (breakdown || exhausted || j == MMAX || j >= next_check);
          // Gershgorin bounds of T_j: rows 0 .. j-2 final, row j-1 with beta_{j-1} and beta_j
          const double ghi = fmax(gfin_hi, a_last + b_prev), glo = fmin(gfin_lo, a_last - b_prev);
          gfin_hi = j > 0 ? fmax(gfin_hi, a_last + b_prev + bet) : gfin_hi;
          gfin_lo = j > 0 ? fmin(gfin_lo, a_last - b_prev - bet) : gfin_lo;
          b_prev = j > 0 ? bet : b_prev;
          // alpha_j = q_j . M q_j (the basis has MMAX + 1 slots: q_MMAX of the
          // step whose check ends the attempt is stored and never read)
          const double q0 = rt0 * ib, q1 = rt1 * ib;
          reinterpret_cast<double2*>(Vb + j * FNP)[lane] = double2{q0, q1};
          const double mq0 = my0 * ib, mq1 = my1 * ib;
          double aj = pa * ib * ib;
          double n0 = mq0 - aj * q0 - (j > 0 ? bet * qp0 : 0.0);
          double n1 = mq1 - aj * q1 - (j > 0 ? bet * qp1 : 0.0);
          if (full) gs(j, q0, q1, n0, n1, aj);
          if (pro) {
            // partial re-orthogonalisation (Simon): the omega recurrence
            // estimates q_{j+1} . q_k from T alone; when an estimate passes
            // sqrt(eps), r~_{j+1} and r~_{j+2} are orthogonalised against the
            // whole basis and the estimates reset
            bool did = force;
            if (force) gs(j, q0, q1, n0, n1, aj);
            force = false;
            double nn2 = wave_sum(n0 * n0 + n1 * n1);
            if (!did) {
              const double mx = omega_step(j, aj, bet, sqrt(nn2), tscale > fabs(aj) ? tscale : fabs(aj));
              if (mx > kSqrtEps) {
                gs(j, q0, q1, n0, n1, aj);
                nn2 = wave_sum(n0 * n0 + n1 * n1);
                did = force = true;
              }
            }
            const double bn = sqrt(nn2);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              const int k = lane + 64 * s2;
              al[s2] = k == j ? aj : al[s2];
              be[s2] = k == j ? bet : be[s2];
              be1[s2] = k == j ? bn : be1[s2];
              if (did) {
                op[s2] = oc[s2];
                oc[s2] = k <= j ? kEps : (k == j + 1 ? 1.0 : 0.0);
              }
            }
            nrm_c = nn2;
          }
          trw[2 * j] = aj;   // every lane: no exec-mask branch
          if (dbg) tstep += clock64() - ts1;
          if (do_check) {
            const int m = j;
            wsym::lds_order();   // the T record
            ++nchecks;
            const long long tc0 = dbg ? clock64() : 0;
            double lm, zl;
            int rounds = 0;
            wave_check(trw, m, theta_lb, hint, glo, ghi, zbuf, scr, trev, &lm, &zl, &rounds,
                       dbg ? tph : nullptr);
            if (dbg) {
              tcheck += clock64() - tc0;
              trounds += rounds;
            }
            const double res = fabs(bet * zl);
            hint = theta_lb > -1e299 ? fmax(lm - theta_lb, 0.0) : -1.0;
            theta_lb = lm;
            if (res <= acc * fabs(lm) || breakdown || exhausted) {
              converged = true;
              m_conv = m;
              lam = lm;
              resid = res;
              break;
            }
            if (res < res_best) {
              m_pre = m_last;
              res_best = res;
              lam_best = lm;
            }
            ghost = !reorth && res_best < 1e-13 * fabs(lam_best) && res > 4.0 * res_best;
            const bool out_of_steps = j == MMAX;
            if (ghost || out_of_steps) {
              if (lane == 0) atomicAdd(A.fb_count + (ghost ? (attempt == 0 ? 3 : 1) : 2), 1);
              if (!ghost && attempt < 2) {   // out of steps: straight on to the re-orthogonalising attempt
                ghost = true;
                attempt = 1;
              }
              m_retry = m_pre;
              break;
            }
            int adv = 6;   // first interval, before a convergence rate is known (A/B: 4 -> 6 saves ~1 %, 8 loses 10 %)
            double rate = rate_hint;
            if (m_a >= 0 && res_a > res && res > 0.0) rate = rate_hint = log(res / res_a) / (m - m_a);
            if (rate < 0.0 && res > 0.0) {
              const double need = log(acc * fabs(lm) / res) / rate;
              adv = need < 1.0 ? 1 : (need > adv_max ? adv_max : static_cast<int>(ceil(need)));
            }
            m_a = m;
            res_a = res;
            m_last = m;
            next_check = m + adv;
          }
          a_last = aj;
          tscale = fmax(tscale, fabs(aj));
          qp0 = q0;
          qp1 = q1;
          rt0 = n0;
          rt1 = n1;
        }
        if (!ghost) break;
      }
      if (!converged) {
        fallback = true;
        break;
      }
      // ---- Ritz vector u = V z of the accepted check
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // also orders the check's z writes before the reads
      {
        const double* zb = zbuf;   // the accepted check's (the last one)
        const double2* V2 = reinterpret_cast<const double2*>(Vb);
        // eight basis rows in flight per batch (the scratch is in L2 / the
        // Infinity Cache: one load latency per batch, not per row)
        double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
        int qq = 0;
        for (; qq + 8 <= m_conv; qq += 8) {
          double2 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = V2[(qq + u) * 64 + lane];
#pragma unroll
          for (int u = 0; u < 8; u += 2) {
            a0 = fma(zb[qq + u], v[u].x, a0);
            a1 = fma(zb[qq + u], v[u].y, a1);
            b0 = fma(zb[qq + u + 1], v[u + 1].x, b0);
            b1 = fma(zb[qq + u + 1], v[u + 1].y, b1);
          }
        }
        for (; qq + 1 < m_conv; qq += 2) {
          const double za = zb[qq], zb1 = zb[qq + 1];
          const double2 va = V2[qq * 64 + lane], vb = V2[(qq + 1) * 64 + lane];
          a0 = fma(za, va.x, a0);
          a1 = fma(za, va.y, a1);
          b0 = fma(zb1, vb.x, b0);
          b1 = fma(zb1, vb.y, b1);
        }
        if (qq < m_conv) {
          const double za = zb[qq];
          const double2 va = V2[qq * 64 + lane];
          a0 = fma(za, va.x, a0);
          a1 = fma(za, va.y, a1);
        }
        u0 = sw0 > 0.0 ? a0 + b0 : 0.0;
        u1 = sw1 > 0.0 ? a1 + b1 : 0.0;
        if constexpr (MODE == 1) {   // a semi-orthogonal basis (PRO): |V z| = 1 + O(sqrt eps)
          const double iu = 1.0 / sqrt(wave_sum(u0 * u0 + u1 * u1));
          u0 *= iu;
          u1 *= iu;
        }
      }
      have_u = true;
      m_hint = m_conv > 8 ? m_conv : 8;
      if (dbg && it < 256) {
        double* rec = A.dbg + FNP * FNP + static_cast<int64_t>(it) * kDbgRec;
        reinterpret_cast<double2*>(rec)[lane] = double2{ci0, ci1};
        if (lane == 0) {
          rec[FNP] = lam;
          rec[FNP + 1] = m_conv;
          rec[FNP + 2] = resid;
          rec[FNP + 3] = nchecks;
          rec[FNP + 4] = nact;
          rec[FNP + 5] = sgw;
          rec[FNP + 6] = static_cast<double>(tph[0]);   // check phases: Laguerre, multisection,
          rec[FNP + 7] = static_cast<double>(tph[1]);   // eigenvector chains, twist + z
          rec[FNP + 13] = static_cast<double>(tph[2]);
          rec[FNP + 14] = static_cast<double>(tph[3]);
          rec[FNP + 8] = static_cast<double>(clock64() - t_it);
          rec[FNP + 9] = static_cast<double>(tcheck);
          rec[FNP + 10] = static_cast<double>(tmv);
          rec[FNP + 11] = static_cast<double>(tstep);
          rec[FNP + 12] = trounds;
          rec[FNP + 15] = ngs;
        }
      }
      // ---- early exit (robust_estimator.py:163-164 / :71-72)
      if (lam * lam <= A.expansion * A.sigma * A.sigma) {
        unweighted = none;
        break;
      }
      if (MODE == 1 && none) {
        if (lane == 0) *A.status = 2;   // c * (1 - step * tau) with c None: TypeError (:75)
        break;
      }
      // ---- tau_i = (C W^1/2 u)_i^2 / lambda
      double t0, t1;
      {
        const double z0 = sw0 * u0, z1 = sw1 * u1;
        wsym::put_operand(zd, z0, z1);
        wsym::matvec<WKV>(P, cl, zd, tb, z0, z1, t0, t1);
      }
      const double ti0 = t0 * t0 / lam, ti1 = t1 * t1 / lam;
      if constexpr (MODE == 1) {
        // c *= 1 - step tau, then the KL projection onto {sum c = 1, c <= cap}
        // (robust_estimator.py:74-99) over the n_keep kept clients
        const double cap = 1.0 / (1.0 - A.eps) / n_keep;
        if (ai0) ci0 = ci0 * (1.0 - step * ti0);
        if (ai1) ci1 = ci1 * (1.0 - step * ti1);
        int capped = 0;
        if (!wave_kl_project(ci0, ci1, ai0, ai1, n_keep, cap, scr, &capped)) {
          none = true;   // projected_c = None (:99)
          unweighted = it + 1 == iters;
          if (unweighted) {
            ci0 = ai0 ? 1.0 : ci0;
            ci1 = ai1 ? 1.0 : ci1;
          }
        }
        if (tr != nullptr && lane == 0) tr[1 + it] = capped;
      } else {
        // filterL2 (:166-172): c *= 1 - tau / tau_max, the argmax (first
        // index) removed, c /= |c|_1
        double tmax = 0.0;
        const double v0 = ai0 ? ti0 : -__builtin_inf(), v1 = ai1 ? ti1 : -__builtin_inf();
        const bool take1 = v1 > v0;
        const int p = wave_argmax_first(take1 ? v1 : v0, take1 ? r1 : r0, &tmax);
        const double cn0 = (ai0 && r0 != p) ? ci0 * (1.0 - ti0 / tmax) : 0.0;
        const double cn1 = (ai1 && r1 != p) ? ci1 * (1.0 - ti1 / tmax) : 0.0;
        const double l1 = wave_sum(fabs(cn0) + fabs(cn1));
        ci0 = cn0 / l1;
        ci1 = cn1 / l1;
        if (r0 == p) ai0 = false;
        if (r1 == p) ai1 = false;
        if (tr != nullptr && lane == 0) tr[1 + it] = p;
      }
      done = it + 1;
    }

    if (fallback) {
      if (lane == 0) {
        const int k = atomicAdd(A.fb_count, 1);
        A.fb_list[k] = ch;
        A.misc[static_cast<size_t>(ch) * kMisc + 3] = 0.0;   // chunk_mean_kernel writes its means
      }
      continue;
    }
    {
      const double c0 = ai0 ? ci0 : 0.0, c1 = ai1 ? ci1 : 0.0;
      reinterpret_cast<double2*>(A.c + static_cast<size_t>(ch) * FNP)[lane] = double2{c0, c1};
      reinterpret_cast<int2*>(A.act + static_cast<size_t>(ch) * FNP)[lane] = int2{ai0 ? 1 : 0, ai1 ? 1 : 0};
      if (tr != nullptr) {
        tr[1 + FNP + r0] = ai0 ? 1 : 0;
        tr[1 + FNP + r1] = ai1 ? 1 : 0;
        if (lane == 0) tr[0] = done;
      }
      // np.average's scale: numpy's pairwise sum of the kept weights in client order
      double* cv = zd;             // [FNP] weights
      double* kf = tb;             // [FNP] kept flags
      wsym::lds_order();
      reinterpret_cast<double2*>(cv)[lane] = double2{c0, c1};
      reinterpret_cast<double2*>(kf)[lane] = double2{ai0 ? 1.0 : 0.0, ai1 ? 1.0 : 0.0};
      wsym::lds_order();
      double scale = 0.0;
      if (lane == 0) {
        double* kept = tb + FNP;   // [FNP]
        int q2 = 0;
        for (int i = 0; i < n; ++i)
          if (kf[i] != 0.0) kept[q2++] = cv[i];
        scale = np_pw64(0, q2, [&](int zz) { return kept[zz]; });
        A.misc[static_cast<size_t>(ch) * kMisc] = scale;
        A.misc[static_cast<size_t>(ch) * kMisc + 3] = 1.0;   // the means below
        if constexpr (MODE == 1) {
          A.misc[static_cast<size_t>(ch) * kMisc + 2] = unweighted ? 1.0 : 0.0;
          if (unweighted) atomicAdd(A.status + 1, 1);
        }
      }
      scale = readlane_f64(scale, 0);
      wsym::lds_order();
      // ---- the chunk's means (chunk_mean_kernel's arithmetic and order, so
      // bit-identical), out of line: its accumulators do not widen the
      // solver's register allocation
      chunk_means(A.Xm, A.ldxm, A.jx0, (A.chunk0 + ch) * static_cast<int64_t>(A.itv), A.itv, A.d, n, cv, kf, scale,
                  MODE == 1 && unweighted, A.out);
      wsym::lds_order();
    }
  }
}

size_t wave_solve_lds() { return kWaveLds; }
int wave_solve_grid() { return kWaveGrid; }

template <int MODE>
static int launch_wave_solve_t(bool dbg, const SolveArgs& sa, int grid, hipStream_t s) {
  const void* k = dbg ? reinterpret_cast<const void*>(&wave_solve_kernel<MODE, true>)
                      : reinterpret_cast<const void*>(&wave_solve_kernel<MODE, false>);
  SRA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kWaveLds)));
  if (dbg) hipLaunchKernelGGL((wave_solve_kernel<MODE, true>), dim3(grid), dim3(64), kWaveLds, s, sa);
  else hipLaunchKernelGGL((wave_solve_kernel<MODE, false>), dim3(grid), dim3(64), kWaveLds, s, sa);
  return launch_status("wave_solve_kernel");
}

int launch_wave_solve(int mode, bool dbg, const SolveArgs& sa, int grid, hipStream_t s) {
  return mode == 1 ? launch_wave_solve_t<1>(dbg, sa, grid, s) : launch_wave_solve_t<0>(dbg, sa, grid, s);
}

}  // namespace sra
