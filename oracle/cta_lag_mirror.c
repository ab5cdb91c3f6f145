/*
 * cta_lag_mirror.c -- TEST INFRASTRUCTURE ONLY (oracle; never linked into the product).
 *
 * The CTA coefficient block of CTA.m:57-98 in the algorithmic (weighted-SYRK) form, evaluated
 * in the exact floating-point operation order of the device's lag-structured path
 * (ccmm_lag.hip k_gram_chol_lag / k_cta_solve_lag, ccmm_kernels.hip k_cta_weights /
 * k_resid_multi), so that the device Gram can be checked bit for bit and the draws at the
 * conditioning of the real data (cond(iV_post) ~ 1e9) without the ~1e-8 spread a different
 * summation order causes.
 *
 * The order of v_mfma_f64_16x16x4_f64 was measured on the device
 * (tools/probe_mfma_order.py, tests/test_gpu_mfma_order.py): D = C + sum_k A(i,k) B(k,j) is
 * four fused multiply-adds in k order, fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0,c)))).  The
 * Gram's k index is time, t = 4 ks + k, so every Gram entry is one fma chain over t = 0..T-1.
 *
 * Column-major arrays as in MATLAB.  Compiled by oracle/Makefile with -ffp-contract=off (every
 * fused operation below is an explicit fma()).
 */
#include <math.h>
#include <string.h>

/* k_cta_weights: sw_t = sqrt(sum_{i>=j} (A(i,j)/sqrtht(t,i))^2) as fma(a, a, w), i ascending,
 * and ih2(t, i) = 1/(sqrtht(t,i)^2) */
void ccmm_mirror_weights(int T, int N, int j, const double* A, const double* sqrtht, double* sw) {
  for (int t = 0; t < T; ++t) {
    double w = 0.0;
    for (int i = j; i < N; ++i) {
      const double a = A[i + (size_t)j * N] / sqrtht[t + (size_t)i * T];
      w = fma(a, a, w);
    }
    sw[t] = sqrt(w);
  }
}

/* k_gram_chol_lag SYRK stage: G (K x K, no prior) with G(0,0) = c, G(1+a,0) = b_a,
 * G(1+a,1+b) = M(a,b):
 *   f_a(t) = X(t,1+a) * sw_t (rounded);  M(a,b) = fma chain over t of f_a f_b;
 *   b_a = (s0 + s1) + (s2 + s3),  s_q = fma chain over t = q mod 4 of f_a(t) sw_t;
 *   c   = (c0 + c1) + (c2 + c3),  c_q = fma chain over t = q mod 4 of sw_t sw_t. */
void ccmm_mirror_gram(int T, int K, const double* X, const double* sw, double* G) {
  const int L = K - 1;
  static double f[4096];
  memset(G, 0, sizeof(double) * (size_t)K * K);
  double cq[4] = {0.0, 0.0, 0.0, 0.0};
  static double bs[4][4096];  /* b_a partial sums per residue of t mod 4 */
  if (L > 4096) return;
  for (int q = 0; q < 4; ++q)
    for (int a = 0; a < L; ++a) bs[q][a] = 0.0;
  for (int t = 0; t < T; ++t) {
    const double s = sw[t];
    for (int a = 0; a < L; ++a) f[a] = X[t + (size_t)(1 + a) * T] * s;
    for (int b = 0; b < L; ++b)
      for (int a = b; a < L; ++a) {
        double* g = &G[(size_t)(1 + a) + (size_t)(1 + b) * K];
        *g = fma(f[a], f[b], *g);
      }
    const int q = t & 3;
    for (int a = 0; a < L; ++a) bs[q][a] = fma(f[a], s, bs[q][a]);
    cq[q] = fma(s, s, cq[q]);
  }
  for (int b = 0; b < L; ++b)
    for (int a = b + 1; a < L; ++a) G[(size_t)(1 + b) + (size_t)(1 + a) * K] = G[(size_t)(1 + a) + (size_t)(1 + b) * K];
  for (int a = 0; a < L; ++a) {
    const double v = (bs[0][a] + bs[1][a]) + (bs[2][a] + bs[3][a]);
    G[1 + a] = v;
    G[(size_t)(1 + a) * K] = v;
  }
  G[0] = (cq[0] + cq[1]) + (cq[2] + cq[3]);
}

/* k_resid_multi: E(:,j) = Y(:,j) - fma chain over a = 0..K-1 of X(t,a) PAI(a,j) */
void ccmm_mirror_resid(int T, int K, int N, const double* Y, const double* X, const double* PAI, double* E) {
  for (int j = 0; j < N; ++j)
    for (int t = 0; t < T; ++t) {
      double acc = 0.0;
      for (int a = 0; a < K; ++a) acc = fma(X[t + (size_t)a * T], PAI[a + (size_t)j * K], acc);
      E[t + (size_t)j * T] = Y[t + (size_t)j * T] - acc;
    }
}

/* k_cta_solve_lag phase 1: v_t = sum_{i>=j} fma(A(i,j) ea_i, ih2(t,i), .), ea_i = fma chain over
 * k = 0..i of e_k A(i,k), e = E with column j replaced by Y(:,j); ih2 = 1/(sqrtht^2) */
void ccmm_mirror_v(int T, int N, int j, const double* A, const double* sqrtht, const double* Y, const double* E,
                   double* v) {
  for (int t = 0; t < T; ++t) {
    double acc = 0.0;
    for (int i = j; i < N; ++i) {
      double ea = 0.0;
      for (int k = 0; k <= i; ++k) {
        const double e = (k == j) ? Y[t + (size_t)k * T] : E[t + (size_t)k * T];
        ea = fma(e, A[i + (size_t)k * N], ea);
      }
      const double sh = sqrtht[t + (size_t)i * T];
      const double w2 = 1.0 / (sh * sh);
      acc = fma(A[i + (size_t)j * N] * ea, w2, acc);
    }
    v[t] = acc;
  }
}

/* phase 2: rhs(1+a) = (h0 + h1) + iVb(1+a): per half [0, th), [th, T) (th = (T+1)/2) four
 * strided fma chains p0..p3 (t = t0 + 4m + r), remainder into p0, h = (p0 + p1) + (p2 + p3);
 * the intercept row: plain sums of v per half */
void ccmm_mirror_rhs(int T, int K, const double* X, const double* v, const double* iVb, double* rhs) {
  const int th = (T + 1) >> 1;
  for (int a = 0; a < K; ++a) {
    double part[2];
    for (int h = 0; h < 2; ++h) {
      const int t0 = h ? th : 0, t1 = h ? T : th;
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
      if (a == 0) {
        for (int t = t0; t < t1; ++t) p0 += v[t];
      } else {
        const double* col = X + (size_t)a * T;
        int t = t0;
        for (; t + 3 < t1; t += 4) {
          p0 = fma(col[t], v[t], p0);
          p1 = fma(col[t + 1], v[t + 1], p1);
          p2 = fma(col[t + 2], v[t + 2], p2);
          p3 = fma(col[t + 3], v[t + 3], p3);
        }
        for (; t < t1; ++t) p0 = fma(col[t], v[t], p0);
      }
      part[h] = (p0 + p1) + (p2 + p3);
    }
    rhs[a] = part[0] + part[1] + iVb[a];
  }
}

/* phase 5: E(:,j) = Y(:,j) - ((s0 + s1) + (s2 + s3)), s0 starting at x_0, s_r = fma chain over the
 * lag columns a = r mod 4 (a ascending) of X(t,1+a) x_{1+a} */
void ccmm_mirror_resid_update(int T, int K, const double* X, const double* Yj, const double* x, double* Ej) {
  const int L = K - 1;
  for (int t = 0; t < T; ++t) {
    /* the device runs over 16 NT >= L lag columns in groups of four; the padded columns read a
     * zero data column, fma(0, x, s) = s, so they are skipped here without changing a chain */
    double s[4] = {x[0], 0.0, 0.0, 0.0};
    for (int a = 0; a < L; ++a) s[a & 3] = fma(X[t + (size_t)(1 + a) * T], x[1 + a], s[a & 3]);
    Ej[t] = Yj[t] - ((s[0] + s[1]) + (s[2] + s[3]));
  }
}
