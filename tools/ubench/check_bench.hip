// Microbenchmark of the spectral-filter solver's convergence check (the top
// Ritz pair of the Lanczos tridiagonal T_m) in isolation: one 256-thread
// workgroup alone on the chip, T from a host Lanczos run (full
// re-orthogonalisation, double) on the weighted-covariance matrix of a
// 128 x 1000 N(0, 0.01^2) chunk -- the C4 bench data.  Times sra::block_check
// (round-2 solver) cold (no previous Ritz value) and warm (previous check 8
// steps earlier), and any candidate check compiled in beside it.
#include "../../secure-robust-federated-learning_amd/csrc/filter.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

namespace {
constexpr int KMAX = 100;

struct Res {
  double theta, zlast;
  long long cycles;
  long long ph[6];
  int rounds;
  double z[sra::MMAX];
};

template <int V>
__global__ void __launch_bounds__(256) check_kernel(const double* al, const double* b2, int m, double theta_lb,
                                                     double hint, Res* res, int reps) {
  __shared__ __attribute__((aligned(16))) double T[sra::TW + 16];
  __shared__ __attribute__((aligned(16))) double z[sra::MMAX];
  __shared__ __attribute__((aligned(16))) double scr[sra::kCheckScr];
  const int tid = threadIdx.x;
  double tscale = 0.0;
  for (int q = tid; q < m; q += 256) {
    T[2 * q] = al[q];
    T[2 * q + 1] = q ? b2[q - 1] : 0.0;
  }
  double glo = 1e300, ghi = -1e300;
  for (int q = 0; q < m; ++q) {
    tscale = fmax(tscale, fmax(fabs(al[q]), q ? sqrt(b2[q - 1]) : 0.0));
    const double r = (q ? sqrt(b2[q - 1]) : 0.0) + (q + 1 < m ? sqrt(b2[q]) : 0.0);
    glo = fmin(glo, al[q] - r);
    ghi = fmax(ghi, al[q] + r);
  }
  __syncthreads();
  double th = 0.0, zl = 0.0;
  long long ph[6] = {0, 0, 0, 0, 0, 0};
  int rounds = 0;
  long long best = 1ll << 60;
  for (int r = 0; r < reps; ++r) {
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) sra::block_check(T, m, theta_lb, hint, tscale, z, scr, &th, &zl, &rounds);
    else sra::fast_check(T, m, theta_lb, hint, glo, ghi, z, scr, &th, &zl, &rounds, ph);
    const long long t1 = __builtin_amdgcn_s_memtime();
    best = t1 - t0 < best ? t1 - t0 : best;
  }
  if (tid == 0) {
    res->theta = th;
    res->zlast = zl;
    res->rounds = rounds;
    res->cycles = best;
    for (int q = 0; q < 6; ++q) res->ph[q] = ph[q] - ph[0];
  }
  for (int q = tid; q < m; q += 256) res->z[q] = z[q];
}

// host Lanczos with full re-orthogonalisation on M (n x n, row-major)
void host_lanczos(const std::vector<double>& M, int n, int steps, std::vector<double>& al, std::vector<double>& b2) {
  std::vector<std::vector<double>> V;
  std::vector<double> q(n), r(n);
  std::mt19937_64 g(7);
  std::normal_distribution<double> nd;
  double nr = 0.0;
  for (int i = 0; i < n; ++i) {
    q[i] = 0.5 + std::fmod(i * 0.6180339887498949, 1.0);
    nr += q[i] * q[i];
  }
  for (double& v : q) v /= std::sqrt(nr);
  double beta = 0.0;
  std::vector<double> qp(n, 0.0);
  for (int j = 0; j < steps; ++j) {
    V.push_back(q);
    for (int i = 0; i < n; ++i) {
      double s = 0.0;
      for (int k = 0; k < n; ++k) s += M[i * n + k] * q[k];
      r[i] = s - beta * qp[i];
    }
    double a = 0.0;
    for (int i = 0; i < n; ++i) a += q[i] * r[i];
    for (int i = 0; i < n; ++i) r[i] -= a * q[i];
    for (int pass = 0; pass < 2; ++pass)
      for (auto& v : V) {
        double h = 0.0;
        for (int i = 0; i < n; ++i) h += v[i] * r[i];
        for (int i = 0; i < n; ++i) r[i] -= h * v[i];
      }
    double nb = 0.0;
    for (int i = 0; i < n; ++i) nb += r[i] * r[i];
    al.push_back(a);
    b2.push_back(nb);
    beta = std::sqrt(nb);
    qp = q;
    for (int i = 0; i < n; ++i) q[i] = r[i] / beta;
  }
}
}  // namespace

int main() {
  const int n = 128, k = 1000;
  std::mt19937_64 gen(1);
  std::normal_distribution<double> nd(0.0, 0.01);
  std::vector<double> X(n * k);
  for (double& v : X) v = static_cast<float>(nd(gen));
  for (int c = 0; c < k; ++c) {
    double mu = 0.0;
    for (int i = 0; i < n; ++i) mu += X[i * k + c];
    mu /= n;
    for (int i = 0; i < n; ++i) X[i * k + c] -= mu;
  }
  std::vector<double> M(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int c = 0; c < k; ++c) s += X[i * k + c] * X[j * k + c];
      M[i * n + j] = s / n;
    }
  std::vector<double> al, b2;
  host_lanczos(M, n, KMAX, al, b2);
  double *dal, *db2;
  Res* dres;
  hipMalloc(&dal, KMAX * 8);
  hipMalloc(&db2, KMAX * 8);
  hipMalloc(&dres, sizeof(Res));
  hipMemcpy(dal, al.data(), KMAX * 8, hipMemcpyHostToDevice);
  hipMemcpy(db2, b2.data(), KMAX * 8, hipMemcpyHostToDevice);
  Res h{}, h1{};
  auto run = [&](int v, int m, double lb, double hint, Res& out) {
    if (v == 0) hipLaunchKernelGGL(check_kernel<0>, dim3(1), dim3(256), 0, 0, dal, db2, m, lb, hint, dres, 5);
    else hipLaunchKernelGGL(check_kernel<1>, dim3(1), dim3(256), 0, 0, dal, db2, m, lb, hint, dres, 5);
    hipMemcpy(&out, dres, sizeof(Res), hipMemcpyDeviceToHost);
  };
  for (int m : {24, 40, 52, 60, 68, 80, 96}) {
    run(0, m, -1e300, -1.0, h);
    const double thc = h.theta;
    run(1, m, -1e300, -1.0, h1);
    double dz = 0.0;
    for (int q = 0; q < m; ++q) dz = std::fmax(dz, std::fabs(std::fabs(h.z[q]) - std::fabs(h1.z[q])));
    printf("m %3d cold: theta %.17g resid %.3e rounds %2d %7lld cyc | fast: dtheta %.1e resid %.3e rounds %2d %7lld cyc"
           "  max|dz| %.1e\n", m, h.theta, std::fabs(h.zlast) * std::sqrt(b2[m - 1]), h.rounds, h.cycles,
           h1.theta - h.theta, std::fabs(h1.zlast) * std::sqrt(b2[m - 1]), h1.rounds, h1.cycles, dz);
    // warm: previous check at m - 8 gives the lower bound and the hint
    run(0, m - 8, -1e300, -1.0, h);
    const double thp = h.theta;
    run(0, m, thp, std::fabs(thc - thp), h);
    run(1, m, thp, std::fabs(thc - thp), h1);
    dz = 0.0;
    for (int q = 0; q < m; ++q) dz = std::fmax(dz, std::fabs(std::fabs(h.z[q]) - std::fabs(h1.z[q])));
    printf("m %3d warm: rounds %2d %7lld cyc | fast: dtheta %.1e rounds %2d %7lld cyc  max|dz| %.1e  phases %lld %lld %lld %lld %lld\n", m, h.rounds,
           h.cycles, h1.theta - h.theta, h1.rounds, h1.cycles, dz, h1.ph[1], h1.ph[2], h1.ph[3], h1.ph[4], h1.ph[5]);
  }
  return 0;
}
