// cpu_sweep.cpp -- TEST / BASELINE INFRASTRUCTURE ONLY (never linked into the product).
//
// The linear BVAR-SV Gibbs sweep of mcmcVAR.m:211-274 restated in C++ AS WRITTEN, for the CPU
// baseline of bench.py ("the build's C++ restatement of the as-written
// algorithm ... one single-threaded process per unit ... linked to the same LAPACK"):
//   CTA.m:57-98      kron-materialised X_j = kron(A(j:N,j), X) ./ lambda (T(N-j+1) x K), X_j'X_j
//                    (dsyrk), chol (dpotrf), Vchol = (iVchol \ I)' (dtrtri), V = Vchol Vchol' (dsyrk),
//                    b = V (iVb + X_j'Y_j) (dgemv, dsymv), PAI(:,j) = b + Vchol z (dtrmv); the
//                    residual (Y - X PAI) A(j:N,:)' by dgemm per equation
//   mcmcVAR.m:236-254  A rows by Cholesky + triangular solves (flat prior)
//   mcmcVAR.m:259-265  logy2, KSC indicators, the log-variance draw (StochVolKSCcorrsqrt, em-matlabbox,
//                    absent: restated as oracle.sv_draw_sequential, the time-ordered block-Cholesky
//                    precision sampler)
//   mcmcVAR.m:268-274  inverse-Wishart draw of PHI
// BLAS / LAPACK: the OpenBLAS that numpy / scipy use (scipy.libs/libscipy_openblas*.so, opened with
// dlopen; LP64 Fortran entry points scipy_d*_), pinned to one thread (parfor: one process per worker).
//
// Usage:
//   cpu_sweep bench <state.bin> <seconds> <seed>      sweeps of one chain for `seconds`, JSON line out
//   cpu_sweep crn <state.bin> <crn.bin> <out.bin>     one sweep on injected common random numbers
// state.bin: int32 N, K, T, dPHI, then doubles Y (T x N), X (T x K), iVdiag, iVb (K x N), sPHI (N x N),
// h0mean (N), h0vcvsqrt (N x N), logy2offset, PAI (K x N), A (N x N), sqrtht (T x N), h (T x N),
// sqrtPHI (N x N); all column-major.  crn.bin: zPAI (K x N), zA (N(N-1)/2), uSV (N x T), zSV
// (N x (T+1)), zPHI (N x (T+dPHI)) (oracle.crn_sizes).  out.bin: PAI, A, sqrtht, h, sqrtPHI, kai (N x T
// as doubles).
#include <dlfcn.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

typedef void (*dgemm_t)(const char*, const char*, const int*, const int*, const int*, const double*, const double*,
                        const int*, const double*, const int*, const double*, double*, const int*);
typedef void (*dsyrk_t)(const char*, const char*, const int*, const int*, const double*, const double*, const int*,
                        const double*, double*, const int*);
typedef void (*dpotrf_t)(const char*, const int*, double*, const int*, int*);
typedef void (*dtrtri_t)(const char*, const char*, const int*, double*, const int*, int*);
typedef void (*dgemv_t)(const char*, const int*, const int*, const double*, const double*, const int*, const double*,
                        const int*, const double*, double*, const int*);
typedef void (*dsymv_t)(const char*, const int*, const double*, const double*, const int*, const double*, const int*,
                        const double*, double*, const int*);
typedef void (*dtrmv_t)(const char*, const char*, const char*, const int*, const double*, const int*, double*,
                        const int*);
typedef void (*dtrsv_t)(const char*, const char*, const char*, const int*, const double*, const int*, double*,
                        const int*);

dgemm_t dgemm;
dsyrk_t dsyrk;
dpotrf_t dpotrf;
dtrtri_t dtrtri;
dgemv_t dgemv;
dsymv_t dsymv;
dtrmv_t dtrmv;
dtrsv_t dtrsv;

void* sym(void* h, const char* name) {
  std::string n1 = std::string("scipy_") + name;
  void* f = dlsym(h, n1.c_str());
  if (!f) f = dlsym(h, name);
  if (!f) {
    std::fprintf(stderr, "cpu_sweep: %s not found in the BLAS library\n", name);
    std::exit(2);
  }
  return f;
}

void load_blas() {
  const char* path = std::getenv("CCMM_CPU_BLAS");
  if (!path) {
    std::fprintf(stderr, "cpu_sweep: CCMM_CPU_BLAS must name the OpenBLAS shared library\n");
    std::exit(2);
  }
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "cpu_sweep: dlopen %s: %s\n", path, dlerror());
    std::exit(2);
  }
  dgemm = (dgemm_t)sym(h, "dgemm_");
  dsyrk = (dsyrk_t)sym(h, "dsyrk_");
  dpotrf = (dpotrf_t)sym(h, "dpotrf_");
  dtrtri = (dtrtri_t)sym(h, "dtrtri_");
  dgemv = (dgemv_t)sym(h, "dgemv_");
  dsymv = (dsymv_t)sym(h, "dsymv_");
  dtrmv = (dtrmv_t)sym(h, "dtrmv_");
  dtrsv = (dtrsv_t)sym(h, "dtrsv_");
  typedef void (*nt_t)(int);
  nt_t nt = (nt_t)dlsym(h, "scipy_openblas_set_num_threads");
  if (!nt) nt = (nt_t)dlsym(h, "openblas_set_num_threads");
  if (nt) nt(1);
}

const double kProb[7] = {0.00730, 0.10556, 0.00002, 0.04395, 0.34001, 0.24566, 0.25750};
const double kMean0[7] = {-10.12999, -3.97281, -8.56686, 2.77786, 0.61942, 1.79518, -1.08819};
const double kVar[7] = {5.79596, 2.61369, 5.17950, 0.16735, 0.64009, 0.34023, 1.26261};

struct Model {
  int N, K, T, dPHI;
  std::vector<double> Y, X, iVdiag, iVb, sPHI, h0mean, h0vcvsqrt;
  double logy2offset;
};
struct State {
  std::vector<double> PAI, A, sqrtht, h, sqrtPHI;
};
struct Crn {  // one sweep's random numbers (oracle.crn_sizes order)
  std::vector<double> zPAI, zA, uSV, zSV, zPHI;
};

#define M2(a, ld, r, c) (a)[(size_t)(c) * (ld) + (r)]

// small dense helpers (N x N, column-major)
void chol_lower(int n, double* a) {  // in place, lower
  int info = 0;
  dpotrf("L", &n, a, &n, &info);
  if (info) throw std::runtime_error("chol");
  for (int c = 0; c < n; ++c)
    for (int r = 0; r < c; ++r) M2(a, n, r, c) = 0.0;
}
void inv_spd(int n, const double* a, double* out) {  // out = a^-1 (Cholesky)
  std::vector<double> L(a, a + (size_t)n * n);
  chol_lower(n, L.data());
  int info = 0;
  dtrtri("L", "N", &n, L.data(), &n, &info);  // L^-1
  // out = L^-T L^-1
  const double one = 1.0, zero = 0.0;
  dgemm("T", "N", &n, &n, &n, &one, L.data(), &n, L.data(), &n, &zero, out, &n);
}

// ---------------------------------------------------------------- CTA.m:57-98 as written
void cta(const Model& m, State& s, const double* z) {
  const int N = m.N, K = m.K, T = m.T;
  const double one = 1.0, zero = 0.0, mone = -1.0;
  const int i1 = 1;
  std::vector<double> E((size_t)T * N), YA((size_t)T * N), Xj((size_t)T * N * K), Yj((size_t)T * N),
      iV((size_t)K * K), Vc((size_t)K * K), V((size_t)K * K), rhs(K), b(K), zc(K);
  for (int j = 0; j < N; ++j) {
    for (int k = 0; k < K; ++k) M2(s.PAI.data(), K, k, j) = 0.0;  // PAI(:,j) = 0 (:63)
    // (Y - X*PAI) * A(j:N,:)'  (:67)
    E = m.Y;
    dgemm("N", "N", &T, &N, &K, &mone, m.X.data(), &T, s.PAI.data(), &K, &one, E.data(), &T);
    const int nr = N - j;
    std::vector<double> Aj((size_t)N * nr);  // A(j:N,:)' : N x nr
    for (int r = 0; r < nr; ++r)
      for (int c = 0; c < N; ++c) M2(Aj.data(), N, c, r) = M2(s.A.data(), N, j + r, c);
    dgemm("N", "N", &T, &nr, &N, &one, E.data(), &T, Aj.data(), &N, &zero, YA.data(), &T);
    const int rows = T * nr;
    // lambda = vec(sqrtht(:,j:N)); Y_j = vec(..) ./ lambda; X_j = kron(A(j:N,j), X) ./ lambda (:66-69)
    for (int r = 0; r < nr; ++r)
      for (int t = 0; t < T; ++t) Yj[(size_t)r * T + t] = YA[(size_t)r * T + t] / M2(s.sqrtht.data(), T, t, j + r);
    for (int k = 0; k < K; ++k)
      for (int r = 0; r < nr; ++r) {
        const double a = M2(s.A.data(), N, j + r, j);
        const double* xk = &M2(m.X.data(), T, 0, k);
        const double* lam = &M2(s.sqrtht.data(), T, 0, j + r);
        double* dst = &M2(Xj.data(), rows, (size_t)r * T, k);
        for (int t = 0; t < T; ++t) dst[t] = a * xk[t] / lam[t];
      }
    // iV_post = iV + X_j'X_j (:73)
    dsyrk("L", "T", &K, &rows, &one, Xj.data(), &rows, &zero, iV.data(), &K);
    for (int k = 0; k < K; ++k) M2(iV.data(), K, k, k) += M2(m.iVdiag.data(), K, k, j);
    // chol(iV_post, 'lower') (:74); Vchol_post = (iVchol_post \ Ik)' (:77); V_post = Vchol Vchol' (:78)
    int info = 0;
    dpotrf("L", &K, iV.data(), &K, &info);
    if (info) throw std::runtime_error("CTA chol (the QR branch of CTA.m:80-92 is not restated here)");
    dtrtri("L", "N", &K, iV.data(), &K, &info);
    for (int c = 0; c < K; ++c)
      for (int r = 0; r < K; ++r) M2(Vc.data(), K, r, c) = (c >= r) ? M2(iV.data(), K, c, r) : 0.0;  // upper
    dsyrk("U", "N", &K, &K, &one, Vc.data(), &K, &zero, V.data(), &K);
    // b_post = V_post (iVb + X_j'Y_j) (:95); PAI(:,j) = b_post + Vchol_post z (:96)
    for (int k = 0; k < K; ++k) rhs[k] = M2(m.iVb.data(), K, k, j);
    dgemv("T", &rows, &K, &one, Xj.data(), &rows, Yj.data(), &i1, &one, rhs.data(), &i1);
    dsymv("U", &K, &one, V.data(), &K, rhs.data(), &i1, &zero, b.data(), &i1);
    for (int k = 0; k < K; ++k) zc[k] = z[(size_t)j * K + k];
    dtrmv("U", "N", "N", &K, Vc.data(), &K, zc.data(), &i1);
    for (int k = 0; k < K; ++k) M2(s.PAI.data(), K, k, j) = b[k] + zc[k];
  }
}

// ---------------------------------------------------------------- one sweep (mcmcVAR.m:228-274)
void sweep(const Model& m, State& s, const Crn& r, std::vector<double>* kai_out) {
  const int N = m.N, K = m.K, T = m.T, dPHI = m.dPHI;
  const double one = 1.0, zero = 0.0, mone = -1.0;
  const int i1 = 1;
  cta(m, s, r.zPAI.data());
  // RESID = Y - X*PAI (:233)
  std::vector<double> RESID = m.Y;
  dgemm("N", "N", &T, &N, &K, &mone, m.X.data(), &T, s.PAI.data(), &K, &one, RESID.data(), &T);
  // A rows (:236-254), flat prior
  std::vector<double> A((size_t)N * N, 0.0);
  for (int i = 0; i < N; ++i) M2(A.data(), N, i, i) = 1.0;
  int off = 0;
  for (int ii = 1; ii < N; ++ii) {
    std::vector<double> Xa((size_t)T * ii), y(T), ZZ((size_t)ii * ii), Zz(ii);
    for (int t = 0; t < T; ++t) {
      const double sh = M2(s.sqrtht.data(), T, t, ii);
      y[t] = M2(RESID.data(), T, t, ii) / sh;
      for (int c = 0; c < ii; ++c) M2(Xa.data(), T, t, c) = M2(RESID.data(), T, t, c) / sh;
    }
    dsyrk("U", "T", &ii, &T, &one, Xa.data(), &T, &zero, ZZ.data(), &ii);
    dgemv("T", &T, &ii, &one, Xa.data(), &T, y.data(), &i1, &zero, Zz.data(), &i1);
    int info = 0;
    dpotrf("U", &ii, ZZ.data(), &ii, &info);  // sqrtiVAlpha_post = chol(iValpha_post) (upper)
    if (info) throw std::runtime_error("A-step chol");
    dtrsv("U", "T", "N", &ii, ZZ.data(), &ii, Zz.data(), &i1);  // tilde = U' \ Zz
    for (int c = 0; c < ii; ++c) Zz[c] += r.zA[off + c];
    dtrsv("U", "N", "N", &ii, ZZ.data(), &ii, Zz.data(), &i1);  // alpha = U \ (tilde + z)
    off += ii;
    for (int c = 0; c < ii; ++c) M2(A.data(), N, ii, c) = -Zz[c];
  }
  s.A = A;
  // logy2 = log((RESID*A').^2 + offset) (:259), as N x T
  std::vector<double> EA((size_t)T * N);
  dgemm("N", "T", &T, &N, &N, &one, RESID.data(), &T, A.data(), &N, &zero, EA.data(), &T);
  std::vector<double> ly((size_t)N * T), obs((size_t)N * T), ir((size_t)N * T);
  if (kai_out) kai_out->assign((size_t)N * T, 0.0);
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < N; ++i) {
      const double e = M2(EA.data(), T, t, i);
      const double y = std::log(e * e + m.logy2offset);
      // KSC 7-component indicators: s = 1 + #{k : u > cdf_k} (oracle.ksc_indicators)
      const double hprev = M2(s.h.data(), T, t, i);
      double ker[7], cs = 0.0, cdf[7];
      for (int k = 0; k < 7; ++k) {
        const double vol = std::sqrt(kVar[k]);
        const double q = (y - hprev - (kMean0[k] - 1.2704)) / vol;
        ker[k] = kProb[k] / vol * std::exp(-0.5 * q * q);
        cs += ker[k];
        cdf[k] = cs;
      }
      const double u = r.uSV[(size_t)t * N + i];
      int sidx = 1;
      for (int k = 0; k < 7; ++k) {
        const double c = (k == 6) ? 1.0 : cdf[k] / cs;
        if (u > c) ++sidx;
      }
      if (kai_out) (*kai_out)[(size_t)t * N + i] = sidx;
      obs[(size_t)t * N + i] = y - (kMean0[sidx - 1] - 1.2704);
      ir[(size_t)t * N + i] = 1.0 / kVar[sidx - 1];
    }
  // precision blocks of x = [h_0; ...; h_T] and the time-ordered block-Cholesky draw
  // (oracle.sv_precision / sv_draw_sequential)
  const int NN = N * N;
  std::vector<double> PHI((size_t)NN), Q((size_t)NN), V0((size_t)NN), V0inv((size_t)NN);
  dgemm("N", "T", &N, &N, &N, &one, s.sqrtPHI.data(), &N, s.sqrtPHI.data(), &N, &zero, PHI.data(), &N);
  inv_spd(N, PHI.data(), Q.data());
  dgemm("N", "T", &N, &N, &N, &one, m.h0vcvsqrt.data(), &N, m.h0vcvsqrt.data(), &N, &zero, V0.data(), &N);
  inv_spd(N, V0.data(), V0inv.data());
  const int T1 = T + 1;
  std::vector<double> Ld((size_t)T1 * NN), Lo((size_t)T1 * NN, 0.0), w((size_t)T1 * N), Dt((size_t)NN), bt(N);
  for (int t = 0; t < T1; ++t) {
    if (t == 0) {
      for (int q = 0; q < NN; ++q) Dt[q] = V0inv[q] + Q[q];
      dgemv("N", &N, &N, &one, V0inv.data(), &N, m.h0mean.data(), &i1, &zero, bt.data(), &i1);
    } else {
      for (int q = 0; q < NN; ++q) Dt[q] = (t == T ? 1.0 : 2.0) * Q[q];
      for (int i = 0; i < N; ++i) {
        M2(Dt.data(), N, i, i) += ir[(size_t)(t - 1) * N + i];
        bt[i] = obs[(size_t)(t - 1) * N + i] * ir[(size_t)(t - 1) * N + i];
      }
      // Lo_t = -(Ld_{t-1} \ Q)' ; D_t -= Lo_t Lo_t' ; b_t -= Lo_t w_{t-1}
      double* lo = &Lo[(size_t)t * NN];
      std::vector<double> X1(Q);
      const double* Lp = &Ld[(size_t)(t - 1) * NN];
      for (int c = 0; c < N; ++c) dtrsv("L", "N", "N", &N, Lp, &N, &X1[(size_t)c * N], &i1);
      for (int a = 0; a < N; ++a)
        for (int c = 0; c < N; ++c) M2(lo, N, a, c) = -M2(X1.data(), N, c, a);
      dsyrk("L", "N", &N, &N, &mone, lo, &N, &one, Dt.data(), &N);
      dgemv("N", &N, &N, &mone, lo, &N, &w[(size_t)(t - 1) * N], &i1, &one, bt.data(), &i1);
    }
    double* ld = &Ld[(size_t)t * NN];
    std::memcpy(ld, Dt.data(), sizeof(double) * NN);
    chol_lower(N, ld);
    std::memcpy(&w[(size_t)t * N], bt.data(), sizeof(double) * N);
    dtrsv("L", "N", "N", &N, ld, &N, &w[(size_t)t * N], &i1);
  }
  std::vector<double> x((size_t)T1 * N), rr(N);
  for (int t = T1 - 1; t >= 0; --t) {
    for (int i = 0; i < N; ++i) rr[i] = w[(size_t)t * N + i] + r.zSV[(size_t)t * N + i];
    if (t + 1 < T1)
      dgemv("T", &N, &N, &mone, &Lo[(size_t)(t + 1) * NN], &N, &x[(size_t)(t + 1) * N], &i1, &one, rr.data(), &i1);
    dtrsv("L", "T", "N", &N, &Ld[(size_t)t * NN], &N, rr.data(), &i1);
    std::memcpy(&x[(size_t)t * N], rr.data(), sizeof(double) * N);
  }
  std::vector<double> eta((size_t)T * N);
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < N; ++i) {
      const double h = x[(size_t)(t + 1) * N + i];
      M2(s.h.data(), T, t, i) = h;
      M2(s.sqrtht.data(), T, t, i) = std::exp(h / 2.0);
      M2(eta.data(), T, t, i) = h - x[(size_t)t * N + i];
    }
  // PHI (:268-274): Lpost = chol(s_PHI + eta'eta, 'lower'), R = chol(Z Z'), sqrtPHI = Lpost / R,
  // PHI = sqrtPHI sqrtPHI', sqrtPHI = chol(PHI, 'lower')
  std::vector<double> S(m.sPHI), ZZ((size_t)NN), sq((size_t)NN);
  dsyrk("L", "T", &N, &T, &one, eta.data(), &T, &one, S.data(), &N);
  chol_lower(N, S.data());
  const int TZ = T + dPHI;
  dsyrk("U", "N", &N, &TZ, &one, r.zPHI.data(), &N, &zero, ZZ.data(), &N);
  int info = 0;
  dpotrf("U", &N, ZZ.data(), &N, &info);
  for (int c = 0; c < N; ++c)
    for (int rr2 = c + 1; rr2 < N; ++rr2) M2(ZZ.data(), N, rr2, c) = 0.0;
  // sq = Lpost * R^-1: solve sq R = Lpost row by row (R upper): sq' = R' \ Lpost'
  std::vector<double> LpT((size_t)NN);
  for (int a = 0; a < N; ++a)
    for (int c = 0; c < N; ++c) M2(LpT.data(), N, c, a) = M2(S.data(), N, a, c);
  for (int c = 0; c < N; ++c) dtrsv("U", "T", "N", &N, ZZ.data(), &N, &LpT[(size_t)c * N], &i1);
  for (int a = 0; a < N; ++a)
    for (int c = 0; c < N; ++c) M2(sq.data(), N, a, c) = M2(LpT.data(), N, c, a);
  dgemm("N", "T", &N, &N, &N, &one, sq.data(), &N, sq.data(), &N, &zero, PHI.data(), &N);
  chol_lower(N, PHI.data());
  s.sqrtPHI = PHI;
}

template <class T_>
void rd(FILE* f, T_* p, size_t n) {
  if (std::fread(p, sizeof(T_), n, f) != n) {
    std::fprintf(stderr, "cpu_sweep: short read\n");
    std::exit(2);
  }
}

void read_state(const char* path, Model& m, State& s) {
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    std::perror(path);
    std::exit(2);
  }
  int32_t hdr[4];
  rd(f, hdr, 4);
  m.N = hdr[0];
  m.K = hdr[1];
  m.T = hdr[2];
  m.dPHI = hdr[3];
  const size_t N = m.N, K = m.K, T = m.T;
  auto vec = [&](std::vector<double>& v, size_t n) {
    v.resize(n);
    rd(f, v.data(), n);
  };
  vec(m.Y, T * N);
  vec(m.X, T * K);
  vec(m.iVdiag, K * N);
  vec(m.iVb, K * N);
  vec(m.sPHI, N * N);
  vec(m.h0mean, N);
  vec(m.h0vcvsqrt, N * N);
  rd(f, &m.logy2offset, 1);
  vec(s.PAI, K * N);
  vec(s.A, N * N);
  vec(s.sqrtht, T * N);
  vec(s.h, T * N);
  vec(s.sqrtPHI, N * N);
  std::fclose(f);
}

void draw(const Model& m, std::mt19937_64& g, Crn& r) {
  std::normal_distribution<double> nd;
  std::uniform_real_distribution<double> ud;
  const size_t N = m.N, K = m.K, T = m.T;
  auto fill = [&](std::vector<double>& v, size_t n, bool uni) {
    v.resize(n);
    for (auto& x : v) x = uni ? ud(g) : nd(g);
  };
  fill(r.zPAI, K * N, false);
  fill(r.zA, N * (N - 1) / 2, false);
  fill(r.uSV, N * T, true);
  fill(r.zSV, N * (T + 1), false);
  fill(r.zPHI, N * (T + m.dPHI), false);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: cpu_sweep bench <state.bin> <seconds> <seed> | crn <state.bin> <crn.bin> <out.bin>\n");
    return 2;
  }
  load_blas();
  Model m;
  State s;
  read_state(argv[2], m, s);
  const std::string mode = argv[1];
  try {
    if (mode == "bench") {
      const double budget = std::atof(argv[3]);
      std::mt19937_64 g(std::strtoull(argv[4], nullptr, 10));
      Crn r;
      long n = 0;
      const auto t0 = std::chrono::steady_clock::now();
      double el = 0.0;
      do {
        draw(m, g, r);
        sweep(m, s, r, nullptr);
        ++n;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      } while (el < budget);
      std::printf("{\"sweeps\": %ld, \"seconds\": %.6f}\n", n, el);
    } else if (mode == "crn") {
      if (argc < 5) return 2;
      Crn r;
      FILE* f = std::fopen(argv[3], "rb");
      if (!f) {
        std::perror(argv[3]);
        return 2;
      }
      const size_t N = m.N, K = m.K, T = m.T;
      auto vec = [&](std::vector<double>& v, size_t n) {
        v.resize(n);
        rd(f, v.data(), n);
      };
      vec(r.zPAI, K * N);
      vec(r.zA, N * (N - 1) / 2);
      vec(r.uSV, N * T);
      vec(r.zSV, N * (T + 1));
      vec(r.zPHI, N * (T + m.dPHI));
      std::fclose(f);
      std::vector<double> kai;
      sweep(m, s, r, &kai);
      FILE* o = std::fopen(argv[4], "wb");
      for (auto* v : {&s.PAI, &s.A, &s.sqrtht, &s.h, &s.sqrtPHI, &kai}) std::fwrite(v->data(), sizeof(double), v->size(), o);
      std::fclose(o);
    } else {
      return 2;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "cpu_sweep: %s\n", e.what());
    return 3;
  }
  return 0;
}
