/*
 * cta_big_mirror.c -- TEST INFRASTRUCTURE ONLY (oracle; never linked into the product).
 *
 * The CTA coefficient block of CTA.m:57-98 in the algorithmic (weighted-SYRK) form, evaluated in
 * the exact floating-point operation order of the device's large-system path (ccmm_big.hip:
 * k_gram_big -> k_chol_big -> k_cta_solve_big; ccmm_kernels.hip k_cta_weights / k_resid), the path
 * of every system that is not a plain VAR design: the hybrid model's K = 1 + (N + Ns) p design
 * (mcmcVARhybridGibbs.m:74-84), K > 512 (S120) or N > 32.
 *
 * Order of v_mfma_f64_16x16x4_f64 (measured, tools/probe_mfma_order.py): D = C + sum_k A(i,k) B(k,j)
 * as four fused multiply-adds in k order, so every MFMA contraction below is one fma chain over the
 * contracted index in increasing order, started from the accumulator's initial value.  The 64-lane
 * reductions follow wave_sum_dpp (ccmm_internal.h): v += v[i^1], v += v[i^2], v += row_half_mirror,
 * v += row_mirror, (v0 + v16) + (v32 + v48).  Pivots: rsqrt_det (the deterministic integer-seed
 * iteration of ccmm_internal.h).
 *
 * Column-major arrays as in MATLAB; KP = K rounded up to 64 (padded coefficients: zero data,
 * identity prior).  Compiled by oracle/Makefile with -ffp-contract=off.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define BT 64

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

/* wave_sum_dpp over the 64 lane values v (v is overwritten) */
static double wave_sum(double* v) {
  double w[64];
  for (int i = 0; i < 64; ++i) w[i] = v[i] + v[i ^ 1];
  for (int i = 0; i < 64; ++i) v[i] = w[i] + w[i ^ 2];
  for (int i = 0; i < 64; ++i) w[i] = v[i] + v[(i & ~7) | (7 - (i & 7))];
  for (int i = 0; i < 64; ++i) v[i] = w[i] + w[(i & ~15) | (15 - (i & 15))];
  return (v[0] + v[16]) + (v[32] + v[48]);
}

#define AT(M, ld, r, c) (M)[(size_t)(c) * (ld) + (r)]

/* k_gram_big: G(a, b) = fma chain over t = 0..T-1 of (X(t,a) w_t) X(t,b), a >= b by 64-blocks (the
 * lower tiles; the diagonal tiles in full), KP x KP column-major, zero elsewhere.  X is T x K. */
static void gram(int T, int K, int KP, const double* X, const double* w, double* G) {
  memset(G, 0, sizeof(double) * (size_t)KP * KP);
  double* xa = (double*)malloc(sizeof(double) * (size_t)KP);
  for (int t = 0; t < T; ++t) {
    for (int a = 0; a < KP; ++a) xa[a] = (a < K) ? AT(X, T, t, a) * w[t] : 0.0 * w[t];
    for (int b = 0; b < K; ++b) {
      const double xb = AT(X, T, t, b);
      const int a0 = (b / BT) * BT;
      for (int a = a0; a < K; ++a) {
        double* g = &AT(G, KP, a, b);
        *g = fma(xb, xa[a], *g);
      }
    }
  }
  free(xa);
}

/* 16 x 16 tile factor + inverse of k_chol_big's factor phase (wave 0, lane = row): T (ld) in/out
 * lower, rd[i] = 1 / L_ii, Li (ld) := L^-1 (lower).  Returns 1 for a non-positive pivot. */
static int tile_factor_inv(double* Tq, int ld, double* rd, double* Li) {
  double row[16][16], rdg[16];
  int bad = 0;
  for (int i = 0; i < 16; ++i) {
    rdg[i] = 1.0;
    for (int m = 0; m < 16; ++m) row[i][m] = (m <= i) ? Tq[i * ld + m] : 0.0;
  }
  for (int kk = 0; kk < 16; ++kk) {
    double dkk = row[kk][kk];
    if (!(dkk > 0.0)) {
      bad = 1;
      dkk = 1.0;
    }
    const double rp = rsqrt_det(dkk);
    row[kk][kk] = dkk * rp;
    rdg[kk] = rp;
    for (int i = kk + 1; i < 16; ++i) row[i][kk] *= rp;
    double lik[16];
    for (int i = 0; i < 16; ++i) lik[i] = row[i][kk];
    for (int m = kk + 1; m < 16; ++m)
      for (int i = m; i < 16; ++i) row[i][m] = fma(-lik[i], lik[m], row[i][m]);
  }
  for (int i = 0; i < 16; ++i) {
    rd[i] = rdg[i];
    for (int m = 0; m < 16; ++m) Tq[i * ld + m] = (m <= i) ? row[i][m] : 0.0;
  }
  for (int c = 0; c < 16; ++c) {
    double x[16];
    for (int i = 0; i < 16; ++i) {
      double s0 = (i == c) ? 1.0 : 0.0, s1 = 0.0;
      for (int m = 0; m < i; m += 2) {
        s0 = fma(-row[i][m], x[m], s0);
        if (m + 1 < i) s1 = fma(-row[i][m + 1], x[m + 1], s1);
      }
      x[i] = (i >= c) ? (s0 + s1) * rdg[i] : 0.0;
    }
    for (int i = 0; i < 16; ++i) Li[i * ld + c] = x[i];
  }
  return bad;
}

/* k_chol_big on A = G + diag(iv) (KP x KP column-major, lower read and written): left-looking
 * 64-wide block columns; Dinv (nb x 64 x 64, row-major blocks) := the diagonal blocks' inverses.
 * Returns 1 for a non-positive pivot. */
static int chol(int KP, double* A, const double* iv, double* Dinv) {
  const int nb = KP / BT;
  int bad = 0;
  static double Lk[BT * BT], Li[BT * BT];
  for (int a = 0; a < KP; ++a) AT(A, KP, a, a) += iv[a];
  for (int kb = 0; kb < nb; ++kb) {
    const int kcol = kb * BT;
    /* 1. update of block column kb, rows kcol.. (negated accumulator, k ascending) */
    for (int j = kcol; j < kcol + BT; ++j)
      for (int i = kcol; i < KP; ++i) {
        double acc = -AT(A, KP, i, j);
        for (int k = 0; k < kcol; ++k) acc = fma(AT(A, KP, i, k), AT(A, KP, j, k), acc);
        AT(A, KP, i, j) = -acc;
      }
    /* 2. the diagonal block as a 4 x 4 grid of 16 x 16 tiles */
    for (int i = 0; i < BT; ++i)
      for (int k = 0; k < BT; ++k) {
        Lk[i * BT + k] = (k <= i) ? AT(A, KP, kcol + i, kcol + k) : 0.0;
        Li[i * BT + k] = 0.0;
      }
    double rdv[16];
    for (int q = 0; q < 4; ++q) {
      bad |= tile_factor_inv(Lk + 16 * q * BT + 16 * q, BT, rdv, Li + 16 * q * BT + 16 * q);
      for (int r = q + 1; r < 4; ++r) {  /* L_rq = A_rq L_qq^-T */
        double out[16][16];
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            double acc = 0.0;
            for (int m = 0; m < 16; ++m)
              acc = fma(Lk[(16 * r + i) * BT + 16 * q + m], Li[(16 * q + j) * BT + 16 * q + m], acc);
            out[i][j] = acc;
          }
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) Lk[(16 * r + i) * BT + 16 * q + j] = out[i][j];
      }
      if (q < 3)  /* trailing tiles A_rs -= L_rq L_sq' */
        for (int r = q + 1; r < 4; ++r)
          for (int s2 = q + 1; s2 <= r; ++s2)
            for (int i = 0; i < 16; ++i)
              for (int j = 0; j < 16; ++j) {
                double acc = Lk[(16 * r + i) * BT + 16 * s2 + j];
                for (int m = 0; m < 16; ++m)
                  acc = fma(-Lk[(16 * r + i) * BT + 16 * q + m], Lk[(16 * s2 + j) * BT + 16 * q + m], acc);
                Lk[(16 * r + i) * BT + 16 * s2 + j] = acc;
              }
    }
    for (int dist = 1; dist < 4; ++dist)  /* inverse tiles below the diagonal, by distance */
      for (int qq = 0; qq + dist < 4; ++qq) {
        const int r = qq + dist;
        double S[16][16], x[16][16];
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            double acc = 0.0;
            for (int kt = qq; kt < r; ++kt)
              for (int m = 0; m < 16; ++m)
                acc = fma(Lk[(16 * r + i) * BT + 16 * kt + m], Li[(16 * kt + m) * BT + 16 * qq + j], acc);
            S[i][j] = acc;
          }
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            double acc = 0.0;
            for (int m = 0; m < 16; ++m) acc = fma(-Li[(16 * r + i) * BT + 16 * r + m], S[m][j], acc);
            x[i][j] = acc;
          }
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) Li[(16 * r + i) * BT + 16 * qq + j] = x[i][j];
      }
    for (int i = 0; i < BT; ++i)
      for (int k = 0; k <= i; ++k) AT(A, KP, kcol + i, kcol + k) = Lk[i * BT + k];
    memcpy(Dinv + (size_t)kb * BT * BT, Li, sizeof(double) * BT * BT);
    /* 3. panel below: L(r, kb) = C(r, kb) L_kk^-T */
    for (int rt = kb + 1; rt < nb; ++rt) {
      const int r0 = rt * BT;
      static double out[BT * BT];
      for (int i = 0; i < BT; ++i)
        for (int j = 0; j < BT; ++j) {
          double acc = 0.0;
          for (int k = 0; k < BT; ++k) acc = fma(AT(A, KP, r0 + i, kcol + k), Li[j * BT + k], acc);
          out[i * BT + j] = acc;
        }
      for (int i = 0; i < BT; ++i)
        for (int j = 0; j < BT; ++j) AT(A, KP, r0 + i, kcol + j) = out[i * BT + j];
    }
  }
  return bad;
}

/* One chain's CTA draw through the large-system path (CTA: all equations on the design X, T x K):
 *   Y T x N, X T x K, A N x N (unit lower), sqrtht T x N, iVdiag / iVb K x N, PAI K x N (the current
 *   draw: the residuals E = Y - X PAI of k_resid enter the first equations' right-hand sides),
 *   z K x N (randn(K,N) of CTA.m:58) -> PAIout K x N.  Returns 1 for a non-positive pivot. */
int ccmm_bmirror_cta(int T, int N, int K, const double* Y, const double* X, const double* A, const double* sqrtht,
                     const double* iVdiag, const double* iVb, const double* PAI, const double* z, double* PAIout) {
  const int KP = (K + BT - 1) / BT * BT, nb = KP / BT;
  int bad = 0;
  double* L = (double*)malloc(sizeof(double) * (size_t)N * KP * KP);
  double* Dinv = (double*)malloc(sizeof(double) * (size_t)N * nb * BT * BT);
  double* w = (double*)malloc(sizeof(double) * (size_t)T);
  double* iv = (double*)malloc(sizeof(double) * (size_t)KP);
  /* k_cta_weights + k_gram_big + k_chol_big for every equation */
  for (int j = 0; j < N; ++j) {
    for (int t = 0; t < T; ++t) {
      double wt = 0.0;
      for (int i = j; i < N; ++i) {
        const double a = AT(A, N, i, j) / AT(sqrtht, T, t, i);
        wt = fma(a, a, wt);
      }
      w[t] = wt;
    }
    double* Lj = L + (size_t)j * KP * KP;
    gram(T, K, KP, X, w, Lj);
    for (int a = 0; a < KP; ++a) iv[a] = (a < K) ? AT(iVdiag, K, a, j) : 1.0;
    bad |= chol(KP, Lj, iv, Dinv + (size_t)j * nb * BT * BT);
  }
  /* k_resid: E(:,j) = Y(:,j) - fma chain over a of X(t,a) PAI(a,j) */
  double* E = (double*)malloc(sizeof(double) * (size_t)T * N);
  double* U = (double*)malloc(sizeof(double) * (size_t)T * N);
  for (int j = 0; j < N; ++j)
    for (int t = 0; t < T; ++t) {
      double acc = 0.0;
      for (int a = 0; a < K; ++a) acc = fma(AT(X, T, t, a), AT(PAI, K, a, j), acc);
      AT(E, T, t, j) = AT(Y, T, t, j) - acc;
    }
  /* k_cta_solve_big: U = E A' */
  for (int i = 0; i < N; ++i)
    for (int t = 0; t < T; ++t) {
      double u = 0.0;
      for (int k = 0; k <= i; ++k) u = fma(AT(E, T, t, k), AT(A, N, i, k), u);
      AT(U, T, t, i) = u;
    }
  double* v = (double*)malloc(sizeof(double) * (size_t)T);
  double* yv = (double*)malloc(sizeof(double) * (size_t)KP);
  double lanes[64], part[64], ri[64];
  const int per = (K + 8 - 1) / 8;
  for (int j = 0; j < N; ++j) {
    const double* Lj = L + (size_t)j * KP * KP;
    const double* Dm = Dinv + (size_t)j * nb * BT * BT;
    /* E(:,j) = Y(:,j); U(:,i) += dE A(i,j), i >= j; v_t */
    for (int t = 0; t < T; ++t) {
      const double yj = AT(Y, T, t, j);
      const double dl = yj - AT(E, T, t, j);
      AT(E, T, t, j) = yj;
      double acc = 0.0;
      for (int i = j; i < N; ++i) {
        const double aij = AT(A, N, i, j);
        const double u = fma(dl, aij, AT(U, T, t, i));
        AT(U, T, t, i) = u;
        const double h = AT(sqrtht, T, t, i);
        acc += aij * (u / h) / h;
      }
      v[t] = acc;
    }
    /* rhs = iVb_j + X' v: lane l an fma chain over t = l, l + 64, ..., then wave_sum_dpp */
    for (int a = 0; a < KP; ++a) {
      for (int l = 0; l < 64; ++l) {
        double p = 0.0;
        if (a < K)
          for (int t = l; t < T; t += 64) p = fma(AT(X, T, t, a), v[t], p);
        lanes[l] = p;
      }
      const double tot = wave_sum(lanes);
      yv[a] = ((a < K) ? AT(iVb, K, a, j) : 0.0) + tot;
    }
    /* forward substitution: y_b = Linv_bb r_b (four chains by k mod 4), then the rows below */
    for (int b = 0; b < nb; ++b) {
      const int r0 = b * BT;
      const double* Db = Dm + (size_t)b * BT * BT;
      double yi[BT];
      for (int i = 0; i < BT; ++i) {
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = 0; k < BT; ++k) a4[k & 3] = fma(Db[i * BT + k], yv[r0 + k], a4[k & 3]);
        yi[i] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      }
      for (int i = 0; i < BT; ++i) yv[r0 + i] = yi[i];
      for (int r = r0 + BT; r < KP; ++r) {
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = 0; k < BT; ++k) a4[k & 3] = fma(AT(Lj, KP, r, r0 + k), yv[r0 + k], a4[k & 3]);
        yv[r] -= (a4[0] + a4[1]) + (a4[2] + a4[3]);
      }
    }
    for (int a = 0; a < K; ++a) yv[a] += AT(z, K, a, j);
    /* back substitution, left-looking by 64-column blocks */
    for (int b = nb - 1; b >= 0; --b) {
      const int r0 = b * BT, rb = r0 + BT;
      for (int c = 0; c < BT; ++c) {
        for (int l = 0; l < 64; ++l) {
          double p = 0.0;
          for (int r = rb + l; r < KP; r += 64) p = fma(AT(Lj, KP, r, r0 + c), yv[r], p);
          lanes[l] = p;
        }
        part[c] = wave_sum(lanes);
      }
      const double* Db = Dm + (size_t)b * BT * BT;
      for (int i = 0; i < BT; ++i) ri[i] = yv[r0 + i] - part[i];
      for (int i = 0; i < BT; ++i) {
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = 0; k < BT; ++k) a4[k & 3] = fma(Db[k * BT + i], ri[k], a4[k & 3]);
        yv[r0 + i] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      }
    }
    for (int a = 0; a < K; ++a) AT(PAIout, K, a, j) = yv[a];
    for (int a = K; a < KP; ++a) yv[a] = 0.0;
    /* E(:,j) = Y(:,j) - X x (eight slices of the K columns, four chains each), U update */
    for (int t = 0; t < T; ++t) {
      double xp = 0.0;
      for (int sl = 0; sl < 8; ++sl) {
        const int a_lo = sl * per, a_hi = (a_lo + per < K) ? a_lo + per : K;
        double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
        int a = a_lo;
        for (; a + 15 < a_hi; a += 16)
          for (int q = 0; q < 16; q += 4) {
            c0 = fma(AT(X, T, t, a + q), yv[a + q], c0);
            c1 = fma(AT(X, T, t, a + q + 1), yv[a + q + 1], c1);
            c2 = fma(AT(X, T, t, a + q + 2), yv[a + q + 2], c2);
            c3 = fma(AT(X, T, t, a + q + 3), yv[a + q + 3], c3);
          }
        for (; a < a_hi; ++a) c0 = fma(AT(X, T, t, a), yv[a], c0);
        xp += (c0 + c1) + (c2 + c3);
      }
      AT(E, T, t, j) = AT(Y, T, t, j) - xp;
      for (int i = j; i < N; ++i) AT(U, T, t, i) = fma(-xp, AT(A, N, i, j), AT(U, T, t, i));
    }
  }
  free(L);
  free(Dinv);
  free(w);
  free(iv);
  free(E);
  free(U);
  free(v);
  free(yv);
  return bad;
}
