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
// Block-hybrid extension (the C++ restatement of the block-hybrid sweep as written,
// mcmcVARshadowrateBlockHybrid.m:332-520): CTAsys.m:57-108 with one design per equation (actual-rate X for
// the macro block, the chain's shadow-rate X for the others), the same A / SV / PHI blocks, the ELB
// state space (:400-416), gibbsdrawShadowrates.m:1-245 as written (the QR smoothing weights of :74-127 by
// dgeqrf, the conditional betas of :130-145, the deterministic Y0 path with its one-period lag, 100 + 1
// Gibbs passes with drawTruncNormal.m's inverse CDF -- AS241 for -sqrt(2) erfcinv(2 u PHIbar)), and the
// rebuild of X, Y from the shadow draws (:501-509).  Selected by the BH block of state.bin.
//
// Algorithmic form (modes bench-syrk / crn-syrk; BASELINE.md §2's second CPU line, SURVEY §8d "a second CPU
// line with the algorithmic (SYRK) form keeps the comparison honest"): the CTA / CTAsys draw by the identity
// X_j'X_j = X' diag(w) X, X_j'Y_j = X' v (w_t = sum_{i>=j} A(i,j)^2 / sqrtht(t,i)^2) -- one dsyrk of the
// T x K design scaled by sqrt(w), dpotrf, and PAI(:,j) = L' \ (L \ rhs + z) by two dtrsv -- instead of the
// kron-materialised T(N-j+1) x K array and the explicit inverse; every other block as above.
//
// Usage:
//   cpu_sweep bench[-syrk] <state.bin> <seconds> <seed>   sweeps of one chain for `seconds` (at least one),
//                                                          JSON line out
//   cpu_sweep crn[-syrk] <state.bin> <crn.bin> <out.bin>  one sweep on injected common random numbers
// state.bin: int32 N, K, T, dPHI, then doubles Y (T x N), X (T x K), iVdiag, iVb (K x N), sPHI (N x N),
// h0mean (N), h0vcvsqrt (N x N), logy2offset, PAI (K x N), A (N x N), sqrtht (T x N), h (T x N),
// sqrtPHI (N x N); all column-major; then optionally the BH block: int32 magic 0x31304842 ("BH01"), p,
// Ns, elbT0, elbT, gibbsburn, Nobs; doubles ELB, Xactual (T x K), actualrateBlock (N, 0/1), ndxS (Ns,
// 0-based), sNaN (Ns x elbT, 0/1), Ydata (Nobs x N, censored cells 0); Y and X above are then the chain's
// shadow-rate data.  crn.bin: zPAI (K x N), zA (N(N-1)/2), uSV (N x T), zSV (N x (T+1)), zPHI
// (N x (T+dPHI)) (oracle.crn_sizes), BH: then uELB (Ns x elbT x (gibbsburn+1)).  out.bin: PAI, A, sqrtht,
// h, sqrtPHI, kai (N x T as doubles), BH: then shadowrate (Ns x elbT).
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
typedef void (*dgeqrf_t)(const int*, const int*, double*, const int*, double*, double*, const int*, int*);
typedef void (*dtrsm_t)(const char*, const char*, const char*, const char*, const int*, const int*, const double*,
                        const double*, const int*, double*, const int*);

dgemm_t dgemm;
dsyrk_t dsyrk;
dpotrf_t dpotrf;
dtrtri_t dtrtri;
dgemv_t dgemv;
dsymv_t dsymv;
dtrmv_t dtrmv;
dtrsv_t dtrsv;
dgeqrf_t dgeqrf;
dtrsm_t dtrsm;

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
  dgeqrf = (dgeqrf_t)sym(h, "dgeqrf_");
  dtrsm = (dtrsm_t)sym(h, "dtrsm_");
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
  // block hybrid (bh): Y, X are the chain's shadow-rate data (updated by the ELB step)
  bool bh = false;
  int p = 0, Ns = 0, elbT0 = 0, elbT = 0, gibbsburn = 0, Nobs = 0;
  double elb = 0.0;
  std::vector<double> Xactual, Ydata;
  std::vector<int> actual, ndxS;
  std::vector<uint8_t> sNaN;  // Ns x elbT
};
struct State {
  std::vector<double> PAI, A, sqrtht, h, sqrtPHI;
  std::vector<double> shadow;  // bh: Ns x elbT, the last ELB draw
};
struct Crn {  // one sweep's random numbers (oracle.crn_sizes order; bh: + uELB)
  std::vector<double> zPAI, zA, uSV, zSV, zPHI, uELB;
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

// ---------------------------------------------------------------- CTA.m:57-98 / CTAsys.m:57-108 as written
// Xs[j] = the design of equation j (CTA: every Xs[j] = X; CTAsys: one design per equation)
void cta(const Model& m, State& s, const double* z, const std::vector<const double*>& Xs) {
  const int N = m.N, K = m.K, T = m.T;
  const double one = 1.0, zero = 0.0, mone = -1.0;
  const int i1 = 1;
  std::vector<double> E((size_t)T * N), YA((size_t)T * N), Xj((size_t)T * N * K), Yj((size_t)T * N),
      iV((size_t)K * K), Vc((size_t)K * K), V((size_t)K * K), rhs(K), b(K), zc(K);
  for (int j = 0; j < N; ++j) {
    for (int k = 0; k < K; ++k) M2(s.PAI.data(), K, k, j) = 0.0;  // PAI(:,j) = 0 (:63)
    // (Y - X*PAI) * A(j:N,:)'  (:67; CTAsys: column jj of X*PAI on equation jj's design)
    E = m.Y;
    for (int jj = 0; jj < N; ++jj)
      dgemv("N", &T, &K, &mone, Xs[jj], &T, &M2(s.PAI.data(), K, 0, jj), &i1, &one, &E[(size_t)jj * T], &i1);
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
        const double* xk = Xs[j] + (size_t)k * T;
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

// ---------------------------------------------------------------- the same draw, algorithmic form
// L L' = iV + X' diag(w) X, rhs = iVb + X' v, PAI(:,j) = L' \ (L \ rhs + z): the draw of CTA.m:95-96 with
// V = (L L')^-1 and Vchol = L^-T, without forming either
void cta_syrk(const Model& m, State& s, const double* z, const std::vector<const double*>& Xs) {
  const int N = m.N, K = m.K, T = m.T;
  const double one = 1.0, zero = 0.0, mone = -1.0;
  const int i1 = 1;
  std::vector<double> E((size_t)T * N), Xw((size_t)T * K), G((size_t)K * K), w(T), v(T), rhs(K);
  for (int j = 0; j < N; ++j) {
    for (int k = 0; k < K; ++k) M2(s.PAI.data(), K, k, j) = 0.0;  // PAI(:,j) = 0 (:63)
    E = m.Y;
    for (int jj = 0; jj < N; ++jj)
      dgemv("N", &T, &K, &mone, Xs[jj], &T, &M2(s.PAI.data(), K, 0, jj), &i1, &one, &E[(size_t)jj * T], &i1);
    // w_t = sum_{i>=j} A(i,j)^2 / sqrtht(t,i)^2;  v_t = sum_{i>=j} A(i,j) (E A(i,:)')_t / sqrtht(t,i)^2
    for (int t = 0; t < T; ++t) {
      double wt = 0.0, vt = 0.0;
      for (int i = j; i < N; ++i) {
        const double a = M2(s.A.data(), N, i, j), h = M2(s.sqrtht.data(), T, t, i);
        double ea = 0.0;
        for (int q = 0; q <= i; ++q) ea += M2(E.data(), T, t, q) * M2(s.A.data(), N, i, q);
        const double ih2 = 1.0 / (h * h);
        wt += a * a * ih2;
        vt += a * ea * ih2;
      }
      w[t] = wt;
      v[t] = vt;
    }
    const double* X = Xs[j];
    for (int k = 0; k < K; ++k)
      for (int t = 0; t < T; ++t) Xw[(size_t)k * T + t] = X[(size_t)k * T + t] * std::sqrt(w[t]);
    dsyrk("L", "T", &K, &T, &one, Xw.data(), &T, &zero, G.data(), &K);  // X' diag(w) X
    for (int k = 0; k < K; ++k) M2(G.data(), K, k, k) += M2(m.iVdiag.data(), K, k, j);
    int info = 0;
    dpotrf("L", &K, G.data(), &K, &info);
    if (info) throw std::runtime_error("CTA chol (the QR branch of CTA.m:80-92 is not restated here)");
    for (int k = 0; k < K; ++k) rhs[k] = M2(m.iVb.data(), K, k, j);
    dgemv("T", &T, &K, &one, X, &T, v.data(), &i1, &one, rhs.data(), &i1);  // iVb + X' v
    dtrsv("L", "N", "N", &K, G.data(), &K, rhs.data(), &i1);                // L \ rhs
    for (int k = 0; k < K; ++k) rhs[k] += z[(size_t)j * K + k];
    dtrsv("L", "T", "N", &K, G.data(), &K, rhs.data(), &i1);                // L' \ (. + z)
    for (int k = 0; k < K; ++k) M2(s.PAI.data(), K, k, j) = rhs[k];
  }
}
bool g_syrk = false;  // modes bench-syrk / crn-syrk

// ---------------------------------------------------------------- one sweep (mcmcVAR.m:228-274)
void elb_step(Model& m, State& s, const Crn& r, const std::vector<double>& invA);
void sweep(Model& m, State& s, const Crn& r, std::vector<double>* kai_out) {
  const int N = m.N, K = m.K, T = m.T, dPHI = m.dPHI;
  const double one = 1.0, zero = 0.0, mone = -1.0;
  const int i1 = 1;
  // designs: CTA (one X) or CTAsys (block hybrid: actual-rate X for the macro block, :343)
  std::vector<const double*> Xs(N, m.X.data());
  if (m.bh)
    for (int j = 0; j < N; ++j)
      if (m.actual[j]) Xs[j] = m.Xactual.data();
  if (g_syrk)
    cta_syrk(m, s, r.zPAI.data(), Xs);
  else
    cta(m, s, r.zPAI.data(), Xs);
  // RESID = Y - X*PAI (:233; block hybrid per equation, :350)
  std::vector<double> RESID = m.Y;
  for (int jj = 0; jj < N; ++jj)
    dgemv("N", &T, &K, &mone, Xs[jj], &T, &M2(s.PAI.data(), K, 0, jj), &i1, &one, &RESID[(size_t)jj * T], &i1);
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
  if (m.bh && m.T > m.elbT0) {
    // invA = A \ I (:372) by forward substitution (A unit lower)
    std::vector<double> invA((size_t)NN, 0.0);
    for (int c = 0; c < N; ++c)
      for (int i = c; i < N; ++i) {
        double v = (i == c) ? 1.0 : 0.0;
        for (int q = c; q < i; ++q) v -= M2(s.A.data(), N, i, q) * M2(invA.data(), N, q, c);
        M2(invA.data(), N, i, c) = v;
      }
    elb_step(m, s, r, invA);
  }
}

// ---------------------------------------------------------------- ELB step (block hybrid)
// Phi^-1(p) by Wichura's AS241 (PPND16): drawTruncNormal.m:47-48's -sqrt(2) erfcinv(2 u PHIbar)
double ppnd16(double p) {
  const double q = p - 0.5;
  if (std::fabs(q) <= 0.425) {
    const double r = 0.180625 - q * q;
    return q * (((((((2509.0809287301226727 * r + 33430.575583588128105) * r + 67265.770927008700853) * r +
                    45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
                  133.14166789178437745) * r + 3.387132872796366608) /
           (((((((5226.495278852545925 * r + 28729.085735721942674) * r + 39307.89580009271061) * r +
                21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
             42.313330701600911252) * r + 1.0);
  }
  double r = (q < 0.0) ? p : 1.0 - p;
  r = std::sqrt(-std::log(r));
  double z;
  if (r <= 5.0) {
    r -= 1.6;
    z = (((((((7.7454501427834140764e-4 * r + 0.0227238449892691845833) * r + 0.24178072517745061177) * r +
             1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r +
          4.6303378461565452959) * r + 1.42343711074968357734) /
        (((((((1.05075007164441684324e-9 * r + 5.475938084995344946e-4) * r + 0.0151986665636164571966) * r +
             0.14810397642748007459) * r + 0.68976733498510000455) * r + 1.6763848301838038494) * r +
          2.05319162663775882187) * r + 1.0);
  } else {
    r -= 5.0;
    z = (((((((2.01033439929228813265e-7 * r + 2.71155556874348757815e-5) * r + 0.0012426609473880784386) * r +
             0.026532189526576123093) * r + 0.29656057182850489123) * r + 1.7848265399172913358) * r +
          5.4637849111641143699) * r + 6.6579046435011037772) /
        (((((((2.04426310338993978564e-15 * r + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5) * r +
             7.868691311456132591e-4) * r + 0.0148753612908506148525) * r + 0.13692988092273580531) * r +
          0.59983220655588793769) * r + 1.0);
  }
  return (q < 0.0) ? -z : z;
}

// drawTruncNormal.m:31-56: one draw from N(mu, sig^2) truncated to (-inf, elb]
double draw_trunc_normal(double mu, double sig, double elb, double u) {
  const double tol = 1e-10, eps = 2.220446049250313080847e-16;
  sig = std::fabs(sig);
  if (sig > tol) {
    const double ub = (elb - mu) / sig;
    const double PHIbar = 0.5 * std::erfc(-std::sqrt(0.5) * ub);
    const double zz = (PHIbar > eps) ? ppnd16(u * PHIbar) : ub;
    return mu + sig * zz;
  }
  return mu;
}

// C = A * B (dense, column-major), n x k times k x m
void gemm_nn(int n, int m, int k, const double* A, int lda, const double* B, int ldb, double* C, int ldc) {
  const double one = 1.0, zero = 0.0;
  dgemm("N", "N", &n, &m, &k, &one, A, &lda, B, &ldb, &zero, C, &ldc);
}

// lower factor L = R' of qr(M') for a square M (numpy qr(M.T, mode='r').T): dgeqrf of M'
void qr_lower(int n, const std::vector<double>& M, std::vector<double>& L) {
  std::vector<double> Mt((size_t)n * n), tau(n);
  for (int c = 0; c < n; ++c)
    for (int r = 0; r < n; ++r) M2(Mt.data(), n, c, r) = M2(M.data(), n, r, c);
  int lwork = -1, info = 0;
  double wq = 0.0;
  dgeqrf(&n, &n, Mt.data(), &n, tau.data(), &wq, &lwork, &info);
  lwork = (int)wq;
  std::vector<double> work(std::max(lwork, 1));
  dgeqrf(&n, &n, Mt.data(), &n, tau.data(), work.data(), &lwork, &info);
  L.assign((size_t)n * n, 0.0);
  for (int c = 0; c < n; ++c)
    for (int r = c; r < n; ++r) M2(L.data(), n, r, c) = M2(Mt.data(), n, c, r);  // L = R'
}

// mcmcVARshadowrateBlockHybrid.m:400-520 with gibbsdrawShadowrates.m:1-245 as written
void elb_step(Model& m, State& s, const Crn& r, const std::vector<double>& invA) {
  const int N = m.N, K = m.K, p = m.p, Ns = m.Ns, T = m.elbT, T0 = m.elbT0, Tm = m.T;
  const int Ny = N, Nstate = Ny * p, Nx = Ny - Ns, Nw = Ny;
  const double one = 1.0, zero = 0.0, mone = -1.0;
  const int i1 = 1;
  std::vector<int> isS(N, 0), ndxX;
  for (int a = 0; a < Ns; ++a) isS[m.ndxS[a]] = 1;
  for (int i = 0; i < N; ++i)
    if (!isS[i]) ndxX.push_back(i);
  // ---- state space (:400-416): lagmask = the shadow rates' lag columns of X
  std::vector<int> lagmask(K, 0);
  for (int l = 0; l < p; ++l)
    for (int a = 0; a < Ns; ++a) lagmask[1 + l * N + m.ndxS[a]] = 1;
  std::vector<double> Yhat((size_t)N * T, 0.0);  // Yhatactual N x elbT
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < N; ++i) {
      if (!m.actual[i]) continue;
      double v = 0.0;
      for (int k = 0; k < K; ++k)
        if (lagmask[k]) v += M2(m.Xactual.data(), Tm, T0 + t, k) * M2(s.PAI.data(), K, k, i);
      M2(Yhat.data(), N, i, t) = v;
    }
  std::vector<double> C((size_t)K * K, 0.0);  // elb.A
  C[0] = 1.0;
  for (int q = 0; q < N * (p - 1); ++q) M2(C.data(), K, 1 + N + q, 1 + q) = 1.0;
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < K; ++k)
      M2(C.data(), K, 1 + i, k) = (lagmask[k] && m.actual[i]) ? 0.0 : M2(s.PAI.data(), K, k, i);  // PAIshadow'
  // SVol = sqrtht(elbT0+1:end, :)'; PSIt(:,:,t) = psi diag(SVol(:,t)), psi = invA
  std::vector<double> PSIt((size_t)N * N * T);
  for (int t = 0; t < T; ++t)
    for (int c = 0; c < N; ++c)
      for (int i = 0; i < N; ++i)
        PSIt[((size_t)t * N + c) * N + i] = M2(invA.data(), N, i, c) * M2(s.sqrtht.data(), Tm, T0 + t, c);
  // cc = C(2:end, 2:end); Cp(:,:,k) = cc^k (:, 1:Ny), k = 0..p
  std::vector<double> cc((size_t)Nstate * Nstate);
  for (int c = 0; c < Nstate; ++c)
    for (int i = 0; i < Nstate; ++i) M2(cc.data(), Nstate, i, c) = M2(C.data(), K, 1 + i, 1 + c);
  std::vector<double> Cp((size_t)Nstate * Ny * (p + 1), 0.0);
  for (int i = 0; i < Ny; ++i) Cp[(size_t)i * Nstate + i] = 1.0;
  for (int k = 1; k <= p; ++k)
    gemm_nn(Nstate, Ny, Nstate, cc.data(), Nstate, &Cp[(size_t)(k - 1) * Nstate * Ny], Nstate,
            &Cp[(size_t)k * Nstate * Ny], Nstate);
  auto cpk = [&](int k) { return &Cp[(size_t)k * Nstate * Ny]; };
  const int nJ = Nstate + Nx;
  std::vector<double> J((size_t)Ns * nJ * T, std::nan("")), sqrtOm((size_t)Ns * Ns * T, std::nan(""));
  auto cens = [&](int t) {
    for (int a = 0; a < Ns; ++a)
      if (m.sNaN[(size_t)t * Ns + a]) return true;
    return false;
  };
  std::vector<double> Mx, Lq, tmp((size_t)Nstate * Nw);
  // ---- smoothing weights (:74-95), t = 1 .. T - p (1-based)
  int t1 = 0;
  for (t1 = 1; t1 <= T - p; ++t1) {
    if (!cens(t1 - 1)) continue;
    const int n = Nstate + Nw;  // square: Nw (p + 1) columns
    Mx.assign((size_t)n * n, 0.0);
    for (int j = 0; j <= p; ++j)
      gemm_nn(Nstate, Nw, Ny, cpk(p - j), Nstate, &PSIt[(size_t)(t1 - 1 + j) * N * N], N, &Mx[(size_t)Nw * j * n], n);
    for (int c = 0; c < Nw; ++c) {
      for (int x = 0; x < Nx; ++x) M2(Mx.data(), n, Nstate + x, c) = PSIt[((size_t)(t1 - 1) * N + c) * N + ndxX[x]];
      for (int a = 0; a < Ns; ++a)
        M2(Mx.data(), n, Nstate + Nx + a, c) = PSIt[((size_t)(t1 - 1) * N + c) * N + m.ndxS[a]];
    }
    qr_lower(n, Mx, Lq);
    // J = R(n1+1:n1+Ns, 1:n1) / L11 (L11 lower): J L11 = R21
    std::vector<double> R21((size_t)Ns * nJ);
    for (int c = 0; c < nJ; ++c)
      for (int a = 0; a < Ns; ++a) M2(R21.data(), Ns, a, c) = M2(Lq.data(), n, nJ + a, c);
    dtrsm("R", "L", "N", "N", &Ns, &nJ, &one, Lq.data(), &n, R21.data(), &Ns);
    std::memcpy(&J[(size_t)(t1 - 1) * Ns * nJ], R21.data(), sizeof(double) * Ns * nJ);
    for (int b = 0; b < Ns; ++b)
      for (int a = 0; a < Ns; ++a)
        sqrtOm[((size_t)(t1 - 1) * Ns + b) * Ns + a] = M2(Lq.data(), n, nJ + a, nJ + b);
  }
  int t = (T - p < 1) ? 0 : T - p;
  // ---- tail (:101-127)
  while (t < T) {
    ++t;
    if (!cens(t - 1)) continue;
    const int k = T - t, Nsig = Ny * k + Nx, n = Nsig + Ns;
    Mx.assign((size_t)n * n, 0.0);
    for (int j = 0; j <= k; ++j) {
      gemm_nn(Nstate, Nw, Ny, cpk(k - j), Nstate, &PSIt[(size_t)(t - 1 + j) * N * N], N, tmp.data(), Nstate);
      for (int c = 0; c < Nw; ++c)
        for (int i = 0; i < Nsig; ++i) M2(Mx.data(), n, i, Nw * j + c) = M2(tmp.data(), Nstate, i, c);
    }
    for (int c = 0; c < Nw; ++c) {
      for (int x = 0; x < Nx; ++x) M2(Mx.data(), n, k * Ny + x, c) = PSIt[((size_t)(t - 1) * N + c) * N + ndxX[x]];
      for (int a = 0; a < Ns; ++a) M2(Mx.data(), n, Nsig + a, c) = PSIt[((size_t)(t - 1) * N + c) * N + m.ndxS[a]];
    }
    qr_lower(n, Mx, Lq);
    double* Jt = &J[(size_t)(t - 1) * Ns * nJ];
    for (int q = 0; q < Ns * nJ; ++q) Jt[q] = 0.0;
    std::vector<double> R21((size_t)Ns * std::max(Nsig, 1));
    for (int c = 0; c < Nsig; ++c)
      for (int a = 0; a < Ns; ++a) M2(R21.data(), Ns, a, c) = M2(Lq.data(), n, Nsig + a, c);
    if (Nsig > 0) dtrsm("R", "L", "N", "N", &Ns, &Nsig, &one, Lq.data(), &n, R21.data(), &Ns);
    for (int c = 0; c < Nsig; ++c)
      for (int a = 0; a < Ns; ++a) M2(Jt, Ns, a, Ny * (p - k) + c) = M2(R21.data(), Ns, a, c);
    for (int b = 0; b < Ns; ++b)
      for (int a = 0; a < Ns; ++a) sqrtOm[((size_t)(t - 1) * Ns + b) * Ns + a] = M2(Lq.data(), n, Nsig + a, Nsig + b);
  }
  // ---- conditional weights for Ns > 1 (:130-145)
  std::vector<double> sqrtOm1((size_t)Ns * T, std::nan("")), beta1((size_t)Ns * std::max(Ns - 1, 1) * T, 0.0);
  if (Ns > 1)
    for (int tt = 0; tt < T; ++tt) {
      if (!cens(tt)) continue;
      const double* so = &sqrtOm[(size_t)tt * Ns * Ns];
      std::vector<double> vcv((size_t)Ns * Ns);
      for (int a = 0; a < Ns; ++a)
        for (int b = 0; b < Ns; ++b) {
          double v = 0.0;
          for (int q = 0; q < Ns; ++q) v += so[(size_t)q * Ns + a] * so[(size_t)q * Ns + b];
          vcv[(size_t)b * Ns + a] = v;
        }
      for (int a = 0; a < Ns; ++a) {
        std::vector<int> o;
        for (int b = 0; b < Ns; ++b)
          if (b != a) o.push_back(b);
        const int no = Ns - 1;
        std::vector<double> Aoo((size_t)no * no), bo(no);
        for (int x = 0; x < no; ++x) {
          bo[x] = vcv[(size_t)o[x] * Ns + a];  // vcv(s, o)
          for (int y = 0; y < no; ++y) Aoo[(size_t)y * no + x] = vcv[(size_t)o[x] * Ns + o[y]];  // vcv(o, o)'
        }
        chol_lower(no, Aoo.data());  // vcv(o, o) is SPD: solve by Cholesky
        dtrsv("L", "N", "N", &no, Aoo.data(), &no, bo.data(), &i1);
        dtrsv("L", "T", "N", &no, Aoo.data(), &no, bo.data(), &i1);
        double bv = 0.0;
        for (int x = 0; x < no; ++x) {
          beta1[((size_t)tt * Ns + a) * (Ns - 1) + x] = bo[x];
          bv += bo[x] * vcv[(size_t)a * Ns + o[x]];
        }
        sqrtOm1[(size_t)tt * Ns + a] = std::sqrt(vcv[(size_t)a * Ns + a] - bv);
      }
    }
  // ---- deterministic path (:157-165; Y0(:,1) = H STATE0 before advancing) and Ytilde
  std::vector<double> Yw((size_t)N * T), Y0((size_t)N * T), st0(K), st1(K);
  for (int tt = 0; tt < T; ++tt)
    for (int i = 0; i < N; ++i) M2(Yw.data(), N, i, tt) = M2(m.Y.data(), Tm, T0 + tt, i);
  for (int k = 0; k < K; ++k) st0[k] = M2(m.Xactual.data(), Tm, T0, k);  // elb.X0 = X(elbT0+1, :)'
  for (int tt = 0; tt < T; ++tt) {
    for (int i = 0; i < N; ++i) M2(Y0.data(), N, i, tt) = st0[1 + i] + M2(Yhat.data(), N, i, tt);
    dgemv("N", &K, &K, &one, C.data(), &K, st0.data(), &i1, &zero, st1.data(), &i1);
    st0.swap(st1);
  }
  // CCpp1 = Cex1^(p+1) (repeated squaring), HC = Cex1(1:Ny, :)
  std::vector<double> P1(cc), Racc((size_t)Nstate * Nstate, 0.0), W1((size_t)Nstate * Nstate);
  for (int i = 0; i < Nstate; ++i) Racc[(size_t)i * Nstate + i] = 1.0;
  for (int e = p + 1; e > 0; e >>= 1) {
    if (e & 1) {
      gemm_nn(Nstate, Nstate, Nstate, Racc.data(), Nstate, P1.data(), Nstate, W1.data(), Nstate);
      Racc.swap(W1);
    }
    if (e > 1) {
      gemm_nn(Nstate, Nstate, Nstate, P1.data(), Nstate, P1.data(), Nstate, W1.data(), Nstate);
      P1.swap(W1);
    }
  }
  const std::vector<double>& CCpp1 = Racc;
  std::vector<double> Yt((size_t)N * T);
  for (size_t q = 0; q < Yt.size(); ++q) Yt[q] = Yw[q] - Y0[q];
  std::vector<double> S((size_t)Ns * T);
  for (int tt = 0; tt < T; ++tt)
    for (int a = 0; a < Ns; ++a) S[(size_t)tt * Ns + a] = M2(Yw.data(), N, m.ndxS[a], tt);
  // ---- Gibbs passes (:171-245)
  const int total = m.gibbsburn + 1;
  std::vector<double> lag(Nstate), YY((size_t)N * (T + p)), yh(N), fut(Nstate), stt(nJ), Sp(Ns);
  for (int n = 0; n < total; ++n) {
    std::fill(lag.begin(), lag.end(), 0.0);
    std::fill(YY.begin(), YY.end(), 0.0);
    std::memcpy(YY.data(), Yt.data(), sizeof(double) * N * T);
    for (int tt = 0; tt < T; ++tt) {
      if (cens(tt)) {
        // Yhat = HC STATElag; Xresid; STATEtilde = STATEfuture - CCpp1 STATElag
        for (int i = 0; i < N; ++i) {
          double v = 0.0;
          for (int q = 0; q < Nstate; ++q) v += M2(cc.data(), Nstate, i, q) * lag[q];
          yh[i] = v;
        }
        for (int l = 0; l < p; ++l)  // columns t+p, ..., t+1
          for (int i = 0; i < N; ++i) fut[(size_t)l * N + i] = M2(YY.data(), N, i, tt + p - l);
        dgemv("N", &Nstate, &Nstate, &mone, CCpp1.data(), &Nstate, lag.data(), &i1, &one, fut.data(), &i1);
        for (int q = 0; q < Nstate; ++q) stt[q] = fut[q];
        for (int x = 0; x < Nx; ++x) stt[Nstate + x] = M2(Yt.data(), N, ndxX[x], tt) - yh[ndxX[x]];
        const double* Jt = &J[(size_t)tt * Ns * nJ];
        for (int a = 0; a < Ns; ++a) {
          double v = yh[m.ndxS[a]] + M2(Y0.data(), N, m.ndxS[a], tt);
          for (int q = 0; q < nJ; ++q) v += M2(Jt, Ns, a, q) * stt[q];
          Sp[a] = v;
        }
        const double* u = &r.uELB[((size_t)n * T + tt) * Ns];
        if (Ns == 1) {
          S[tt] = draw_trunc_normal(Sp[0], sqrtOm[(size_t)tt], m.elb, u[0]);
        } else {
          for (int a = 0; a < Ns; ++a) {
            if (!m.sNaN[(size_t)tt * Ns + a]) continue;
            double mu = Sp[a];
            int y = 0;
            for (int b = 0; b < Ns; ++b) {
              if (b == a) continue;
              mu += beta1[((size_t)tt * Ns + a) * (Ns - 1) + y] * (S[(size_t)tt * Ns + b] - Sp[b]);
              ++y;
            }
            S[(size_t)tt * Ns + a] = draw_trunc_normal(mu, sqrtOm1[(size_t)tt * Ns + a], m.elb, u[a]);
          }
        }
        for (int a = 0; a < Ns; ++a) {
          M2(Yw.data(), N, m.ndxS[a], tt) = S[(size_t)tt * Ns + a];
        }
        for (int i = 0; i < N; ++i) M2(Yt.data(), N, i, tt) = M2(Yw.data(), N, i, tt) - M2(Y0.data(), N, i, tt);
      }
      if (tt + 1 >= p) {
        for (int l = 0; l < p; ++l)
          for (int i = 0; i < N; ++i) lag[(size_t)l * N + i] = M2(Yt.data(), N, i, tt - l);
      } else {
        for (int q = Nstate - 1; q >= N; --q) lag[q] = lag[q - N];
        for (int i = 0; i < N; ++i) lag[i] = M2(Yt.data(), N, i, tt);
      }
    }
  }
  s.shadow = S;
  // ---- rebuild X, Y from the shadow draws (:480, 501-509)
  for (int tt = 0; tt < T; ++tt)
    for (int a = 0; a < Ns; ++a) M2(m.Ydata.data(), m.Nobs, p + T0 + tt, m.ndxS[a]) = S[(size_t)tt * Ns + a];
  for (int row = 0; row < Tm; ++row) {
    for (int i = 0; i < N; ++i) M2(m.Y.data(), Tm, row, i) = M2(m.Ydata.data(), m.Nobs, p + row, i);
    M2(m.X.data(), Tm, row, 0) = 1.0;
    for (int l = 1; l <= p; ++l)
      for (int i = 0; i < N; ++i) M2(m.X.data(), Tm, row, 1 + (l - 1) * N + i) = M2(m.Ydata.data(), m.Nobs, p + row - l, i);
  }
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
  int32_t bh[7];
  if (std::fread(bh, sizeof(int32_t), 7, f) == 7 && bh[0] == 0x31304842) {
    m.bh = true;
    m.p = bh[1];
    m.Ns = bh[2];
    m.elbT0 = bh[3];
    m.elbT = bh[4];
    m.gibbsburn = bh[5];
    m.Nobs = bh[6];
    rd(f, &m.elb, 1);
    vec(m.Xactual, T * K);
    std::vector<double> a;
    vec(a, N);
    m.actual.assign(N, 0);
    for (size_t i = 0; i < N; ++i) m.actual[i] = a[i] != 0.0;
    vec(a, m.Ns);
    m.ndxS.assign(m.Ns, 0);
    for (int i = 0; i < m.Ns; ++i) m.ndxS[i] = (int)a[i];
    vec(a, (size_t)m.Ns * m.elbT);
    m.sNaN.assign(a.size(), 0);
    for (size_t i = 0; i < a.size(); ++i) m.sNaN[i] = a[i] != 0.0;
    vec(m.Ydata, (size_t)m.Nobs * N);
  }
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
  if (m.bh) fill(r.uELB, (size_t)m.Ns * m.elbT * (m.gibbsburn + 1), true);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: cpu_sweep bench[-syrk] <state.bin> <seconds> <seed> | crn[-syrk] <state.bin> <crn.bin> <out.bin>\n");
    return 2;
  }
  load_blas();
  Model m;
  State s;
  read_state(argv[2], m, s);
  std::string mode = argv[1];
  if (mode.size() > 5 && mode.compare(mode.size() - 5, 5, "-syrk") == 0) {
    g_syrk = true;
    mode.resize(mode.size() - 5);
  }
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
      if (m.bh) vec(r.uELB, (size_t)m.Ns * m.elbT * (m.gibbsburn + 1));
      std::fclose(f);
      std::vector<double> kai;
      sweep(m, s, r, &kai);
      FILE* o = std::fopen(argv[4], "wb");
      for (auto* v : {&s.PAI, &s.A, &s.sqrtht, &s.h, &s.sqrtPHI, &kai, &s.shadow})
        std::fwrite(v->data(), sizeof(double), v->size(), o);
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
