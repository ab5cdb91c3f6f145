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

/* ------------------------------------------------------------------------------------------
 * Factorisation and solves of the lag-structured path (ccmm_lag.hip gram_lag_factor /
 * gl_factor_inv / k_cta_solve_lag phases 3-4), operation for operation.  Tiles: NT = ceil((K-1)
 * / 16) lag tiles, KL = 16 NT padded lag columns (zero data, prior precision 1).  Slot (ti, tj),
 * ti >= tj, is the device's register tile: S[a][b] = element (row a, column b) of the UPPER tile
 * (tj, ti) of the symmetric matrix, i.e. M(16 tj + a, 16 ti + b).  Every v_mfma_f64_16x16x4_f64
 * is four fused multiply-adds in k order (measured), so a product of two 16 x 16 tiles is an fma
 * chain over m = 0..15 per entry.  Pivots: 1 / sqrt(d) by the device's deterministic integer-seed
 * fourth-order iteration (gl_rsqrt_det).  The intercept pivot L00 = sqrt(c + iv0), 1 / L00 uses the IEEE
 * (correctly rounded) sqrt and division on both sides.
 * ------------------------------------------------------------------------------------------ */
#define MT 16
typedef double tile_t[MT][MT];

/* gl_rsqrt_det: integer seed 0x5fe6eb50c7b537a9 - (bits >> 1), two fourth-order steps */
static double rsqrt_det(double d) {
  long long bits;
  memcpy(&bits, &d, sizeof bits);
  bits = 0x5fe6eb50c7b537a9LL - (bits >> 1);
  double r;
  memcpy(&r, &bits, sizeof r);
  for (int it = 0; it < 2; ++it) {
    const double e = fma(-(d * r), r, 1.0);
    const double q = fma(fma(0.3125, e, 0.375), e, 0.5);
    r = fma(r * e, q, r);
  }
  return r;
}

/* gl_factor_inv: Linv[i][c] = (L^-1)(i, c) of the lower Cholesky factor of the 16 x 16 tile D
 * (lower triangle read); returns 1 for a non-positive pivot */
static int mirror_factor_inv(const tile_t D, tile_t Linv) {
  double row[MT][MT], rdiag[MT], W[MT][MT];
  double dmin = 1.0;
  for (int i = 0; i < MT; ++i)
    for (int m = 0; m < MT; ++m) row[i][m] = (m <= i) ? D[i][m] : 0.0;
  for (int i = 0; i < MT; ++i) rdiag[i] = 1.0;
  for (int kk = 0; kk < MT; ++kk) {
    const double dkk = row[kk][kk];
    dmin = fmin(dmin, dkk);
    const double rp = rsqrt_det(fmax(dkk, 1e-300));
    rdiag[kk] = rp;
    double lik[MT];
    for (int i = 0; i < MT; ++i) {
      lik[i] = (i > kk) ? row[i][kk] * rp : 0.0;
      row[i][kk] = lik[i];
    }
    for (int i = 0; i < MT; ++i)
      for (int m = kk + 1; m < MT; ++m) row[i][m] = fma(-lik[i], lik[m], row[i][m]);
  }
  for (int i = 0; i < MT; ++i)
    for (int m = 0; m < MT; ++m) W[i][m] = (m < i) ? row[i][m] : ((m == i) ? rdiag[i] : 0.0);
  for (int c = 0; c < MT; ++c) {
    double x[MT];
    for (int i = 0; i < MT; ++i) {
      double s0 = (i == c) ? 1.0 : 0.0, s1 = 0.0;
      for (int m = 0; m < i; m += 2) {
        s0 = fma(-W[i][m], x[m], s0);
        if (m + 1 < i) s1 = fma(-W[i][m + 1], x[m + 1], s1);
      }
      x[i] = (i >= c) ? (s0 + s1) * W[i][i] : 0.0;
    }
    for (int i = 0; i < MT; ++i) Linv[i][c] = x[i];
  }
  return dmin > 0.0 ? 0 : 1;
}

static int slot_index(int NT, int ti, int tj) { return ti + tj * NT; }  /* dense NT x NT table */

/* gram_lag_factor: G = [c b'; b M] (K x K, ccmm_mirror_gram, no prior), iv = iVdiag (K) ->
 *   S   NT x NT x 16 x 16 (slot (ti, tj) at ti + tj NT, ti >= tj): off-diagonal M'_{tj,ti}, diagonal
 *       U_pp^-1 = L_pp^-T, as the device writes its factor tiles
 *   l   KL: L(1 + a, 0) = b_a / L00;  *rL00 = 1 / L00.  Returns 1 for a non-positive pivot. */
int ccmm_mirror_factor(int K, const double* G, const double* iv, double* S_, double* l, double* rL00_out) {
  const int L = K - 1, NT = (L + MT - 1) / MT, KL = MT * NT;
  tile_t* S = (tile_t*)S_;
  static double b[4096], ivk[4096 + 1];
  static tile_t Pn[256], Linv;
  if (KL > 4096 || NT > 256) return 1;
  int bad = 0;
  for (int a = 0; a < KL; ++a) {
    b[a] = (a < L) ? G[1 + a] : 0.0;
    ivk[1 + a] = (a < L) ? iv[1 + a] : 1.0;
  }
  const double G00 = G[0] + iv[0];
  if (!(G00 > 0.0)) bad = 1;
  const double L00 = sqrt(G00 > 0.0 ? G00 : 1.0);
  const double rL00 = 1.0 / L00;
  /* SYRK slots, + diag(iV~) - l l' (intercept peel) */
  for (int tj = 0; tj < NT; ++tj)
    for (int ti = tj; ti < NT; ++ti) {
      double(*s)[MT] = S[slot_index(NT, ti, tj)];
      for (int a = 0; a < MT; ++a)
        for (int c = 0; c < MT; ++c) {
          const int ra = MT * tj + a, cb = MT * ti + c;
          const double m = (ra < L && cb < L) ? G[(size_t)(1 + ra) + (size_t)(1 + cb) * K] : 0.0;
          const double lc = b[cb] * rL00;
          double v = fma(-(b[ra] * rL00), lc, m);
          if (ti == tj && a == c) v += ivk[1 + ra];
          s[a][c] = v;
        }
    }
  for (int a = 0; a < KL; ++a) l[a] = b[a] * rL00;
  *rL00_out = rL00;
  bad |= mirror_factor_inv((const double(*)[MT])S[slot_index(NT, 0, 0)], Linv);
  for (int p = 0; p < NT; ++p) {
    for (int ti = p; ti < NT; ++ti) {
      double(*s)[MT] = S[slot_index(NT, ti, p)];
      if (ti == p) {
        for (int a = 0; a < MT; ++a)
          for (int c = 0; c < MT; ++c) s[a][c] = Linv[c][a];
      } else {
        double(*u)[MT] = Pn[ti];
        for (int a = 0; a < MT; ++a)
          for (int c = 0; c < MT; ++c) {
            double acc = 0.0;
            for (int m = 0; m < MT; ++m) acc = fma(Linv[a][m], s[m][c], acc);
            u[a][c] = acc;
          }
        for (int a = 0; a < MT; ++a)
          for (int c = 0; c < MT; ++c) {
            double acc = 0.0;
            for (int m = 0; m < MT; ++m) acc = fma(Linv[m][a], u[m][c], acc);
            s[a][c] = acc;
          }
      }
    }
    if (p + 1 < NT) {
      for (int tj = p + 1; tj < NT; ++tj)
        for (int ti = tj; ti < NT; ++ti) {
          double(*s)[MT] = S[slot_index(NT, ti, tj)];
          for (int a = 0; a < MT; ++a)
            for (int c = 0; c < MT; ++c) {
              double acc = s[a][c];
              for (int m = 0; m < MT; ++m) acc = fma(-Pn[tj][m][a], Pn[ti][m][c], acc);
              s[a][c] = acc;
            }
        }
      bad |= mirror_factor_inv((const double(*)[MT])S[slot_index(NT, p + 1, p + 1)], Linv);
    }
  }
  return bad;
}

/* sum over the 16 lanes of a row group in the device's butterfly order (xor 8, 4, 2, 1) */
static double tree16(const double* v) {
  double P[8], Q[4], R[2];
  for (int y = 0; y < 8; ++y) P[y] = v[y] + v[y + 8];
  for (int y = 0; y < 4; ++y) Q[y] = P[y] + P[y + 4];
  for (int y = 0; y < 2; ++y) R[y] = Q[y] + Q[y + 2];
  return R[0] + R[1];
}

/* colsum: out[c] = sum_a s[a][c] u[a], four lanes (a mod 4) each an fma chain over a = q + 4r,
 * then (v0 + v1) + (v2 + v3) (permlane16 / permlane32 swaps) */
static void colsum(const double (*s)[MT], const double* u, double* out) {
  for (int c = 0; c < MT; ++c) {
    double v[4];
    for (int q = 0; q < 4; ++q) {
      double acc = s[q][c] * u[q];
      for (int r = 1; r < 4; ++r) acc = fma(s[q + 4 * r][c], u[q + 4 * r], acc);
      v[q] = acc;
    }
    out[c] = (v[0] + v[1]) + (v[2] + v[3]);
  }
}

/* fold: out[a] = sum_c s[a][c] u[c] in the tree16 order */
static void fold(const double (*s)[MT], const double* u, double* out) {
  for (int a = 0; a < MT; ++a) {
    double v[MT];
    for (int c = 0; c < MT; ++c) v[c] = s[a][c] * u[c];
    out[a] = tree16(v);
  }
}

/* k_cta_solve_lag phases 3-4: x = L' \ (L \ rhs + z) with the factor of ccmm_mirror_factor;
 * rhs, z, x K-space (0 = intercept) */
void ccmm_mirror_solve(int K, const double* S_, const double* l, double rL00, const double* rhs, const double* z,
                       double* x) {
  const int L = K - 1, NT = (L + MT - 1) / MT, KL = MT * NT;
  const tile_t* S = (const tile_t*)S_;
  static double r[4096 + 1], y[4096 + 1], tmp[MT];
  if (KL > 4096) return;
  for (int a = 0; a < KL; ++a) r[1 + a] = (1 + a < K) ? rhs[1 + a] : 0.0;
  r[0] = rhs[0];
  /* the padded rows of rhs: iVb padding 0 and zero data, so rl = 0 on the device as well */
  for (int a = 0; a < KL; ++a) r[1 + a] = fma(-l[a], r[0] * rL00, r[1 + a]);
  y[0] = r[0] * rL00;
  for (int p = 0; p + 1 < NT; ++p)
    for (int ti = p + 1; ti < NT; ++ti) {
      colsum(S[slot_index(NT, ti, p)], r + 1 + MT * p, tmp);
      for (int c = 0; c < MT; ++c) r[1 + MT * ti + c] -= tmp[c];
    }
  for (int ti = 0; ti < NT; ++ti) colsum(S[slot_index(NT, ti, ti)], r + 1 + MT * ti, y + 1 + MT * ti);
  /* c = y + z */
  for (int k = 0; k <= KL; ++k) r[k] = y[k] + ((k < K) ? z[k] : 0.0);
  for (int ti = 0; ti < NT; ++ti) fold(S[slot_index(NT, ti, ti)], r + 1 + MT * ti, y + 1 + MT * ti);
  for (int p = NT - 1; p >= 1; --p)
    for (int tj = 0; tj < p; ++tj) {
      fold(S[slot_index(NT, p, tj)], y + 1 + MT * p, tmp);
      for (int a = 0; a < MT; ++a) y[1 + MT * tj + a] -= tmp[a];
    }
  /* l' x~: per wave of 64 threads a binary tree in lane order, then the 8 wave sums in order */
  double sacc = 0.0;
  for (int w = 0; w < 8; ++w) {
    double v[64];
    for (int q = 0; q < 64; ++q) {
      const int a = 64 * w + q;
      v[q] = (a < KL) ? l[a] * y[1 + a] : 0.0;
    }
    /* xor-1, xor-2 quad permutes, half-row and row mirrors, then (r0 + r1) + (r2 + r3) over the
       four rows: a binary tree over adjacent lanes */
    for (int h = 1; h < 64; h <<= 1)
      for (int q = 0; q < 64; q += 2 * h) v[q] = v[q] + v[q + h];
    sacc += v[0];
  }
  y[0] = (r[0] - sacc) * rL00;
  for (int k = 0; k < K; ++k) x[k] = y[k];
}
