// Host CTA draw of one chain with the QR branch of CTA.m:80-92 (CTAsys.m:90-100): the
// fallback of the device coefficient block when a posterior precision's Cholesky meets a
// non-positive pivot (status bit 2), so one numerically indefinite system no longer
// invalidates the chain.
//
// Per equation j (CTA.m:61-96, algorithmic form: no kron materialisation):
//   E       = Y - X PAI with PAI(:, j) = 0 (columns < j: this call's draws, > j: previous)
//   ytil_i  = (E A(i, :)') ./ lambda_i,  lambda_i = sqrtht(:, i),  i >= j
//   w2(t)   = sum_{i >= j} A(i, j)^2 / lambda_i(t)^2
//   iV_post = diag(iVdiag_j) + X' diag(w2) X,  rhs = iVb_j + X' sum_{i >= j} A(i, j) ytil_i ./ lambda_i
//   Lp      = chol(iV_post, 'lower'), or, if that fails, R' of the Householder QR of
//             [chol(diag(iVdiag_j)); diag(sqrt(w2)) X]        (Kailath's array, CTA.m:84-89)
//   PAI(:, j) = Lp^{-T} (Lp^{-1} rhs + z_j)                    (CTA.m:94-95)
//
// The QR of the T-row weighted design has the same R as MATLAB's QR of the kron-stacked
// [iVchol, X_j']' (CTA.m:87): both have R'R = iV_post, and with a diagonal iV every
// Householder pivot is the positive sqrt(iVdiag(k)), so LAPACK's convention gives
// R(k, k) < 0 in both and R is unique.  (Hence the QR draw equals the Cholesky draw with
// z -> -z: same posterior, evaluated without squaring the condition number.)
#include <cmath>
#include <cstdint>
#include <vector>

namespace ccmm {

namespace {

// lower Cholesky in place (column-major n x n); false on a non-positive pivot
bool chol_lower(std::vector<double>& G, int n) {
  for (int j = 0; j < n; ++j) {
    double d = G[j + (size_t)j * n];
    for (int k = 0; k < j; ++k) d -= G[j + (size_t)k * n] * G[j + (size_t)k * n];
    if (!(d > 0.0)) return false;
    const double p = std::sqrt(d), ip = 1.0 / p;
    G[j + (size_t)j * n] = p;
    for (int i = j + 1; i < n; ++i) {
      double v = G[i + (size_t)j * n];
      for (int k = 0; k < j; ++k) v -= G[i + (size_t)k * n] * G[j + (size_t)k * n];
      G[i + (size_t)j * n] = v * ip;
    }
  }
  return true;
}

// R of the Householder QR of M (m x n column-major, m >= n), LAPACK dgeqr2 sign convention
// (beta = -sign(alpha) ||x||); returns Lp = R' (lower, n x n column-major)
std::vector<double> qr_lower(std::vector<double>& M, int m, int n) {
  std::vector<double> L((size_t)n * n, 0.0);
  std::vector<double> v(m);
  for (int k = 0; k < n; ++k) {
    double* col = &M[(size_t)k * m];
    const double alpha = col[k];
    double xn2 = 0.0;
    for (int i = k + 1; i < m; ++i) xn2 += col[i] * col[i];
    if (xn2 == 0.0) {  // H = I
      L[k + (size_t)k * n] = alpha;
      for (int c = k + 1; c < n; ++c) L[c + (size_t)k * n] = M[k + (size_t)c * m];
      continue;
    }
    const double beta = -std::copysign(std::sqrt(alpha * alpha + xn2), alpha);
    const double tau = (beta - alpha) / beta;
    const double sc = 1.0 / (alpha - beta);
    v[k] = 1.0;
    for (int i = k + 1; i < m; ++i) v[i] = col[i] * sc;
    for (int c = k + 1; c < n; ++c) {
      double* mc = &M[(size_t)c * m];
      double s = 0.0;
      for (int i = k; i < m; ++i) s += v[i] * mc[i];
      s *= tau;
      for (int i = k; i < m; ++i) mc[i] -= s * v[i];
    }
    L[k + (size_t)k * n] = beta;  // R(k, k)
    for (int c = k + 1; c < n; ++c) L[c + (size_t)k * n] = M[k + (size_t)c * m];  // R(k, c) -> Lp(c, k)
  }
  return L;
}

}  // namespace

// Y(t, i) at Y[i * ldy + t]; equation i's design X_i(t, k) at Xs[i][k * ldx + t];
// A column-major N x N (unit lower); sqrtht(t, i) at sqrtht[i * ldh + t];
// iVdiag / iVb / PAI: row j = equation j, (j, k) at [j * ldk + k]; z(k, j) at z[k + K * j].
// Aelb / atELB (CTAsysAswitching.m:61-92, optional): months t with atELB[t] != 0 use Aelb in
// place of A in the residual map and the weights.
// Returns bit 0: the QR branch ran for some equation; bit 1: a QR factor was singular.
int host_cta_chain(int N, int K, int T, const double* Y, int ldy, const double* const* Xs, int ldx,
                   const double* A0, const double* sqrtht, int ldh, const double* iVdiag,
                   const double* iVb, int ldk, double* PAI, const double* z, bool force_qr,
                   const double* Aelb, const uint8_t* atELB) {
  int flags = 0;
  const double* A = A0;
  auto At = [&](int t) { return (Aelb && atELB && atELB[t]) ? Aelb : A0; };
  if (Aelb)
    for (int q = 0; q < N * N; ++q)
      if (!std::isfinite(Aelb[q])) return 2;
  // a chain whose state is not finite is not redrawn (the QR branch cannot repair it)
  for (int i = 0; i < N; ++i)
    for (int t = 0; t < T; ++t)
      if (!std::isfinite(sqrtht[(size_t)i * ldh + t]) || !std::isfinite(Y[(size_t)i * ldy + t])) return 2;
  for (int q = 0; q < N * N; ++q)
    if (!std::isfinite(A[q])) return 2;
  // E(t, i) = Y - X_i PAI_i and EA(t, i) = sum_k E(t, k) A(i, k), kept current as the
  // columns of E change (CTA.m:68: (Y - X*PAI) * A_(j:N,:)')
  std::vector<double> E((size_t)N * T), EA((size_t)N * T, 0.0), col(T);
  auto resid_col = [&](int i, double* out) {
    const double* Xi = Xs[i];
    for (int t = 0; t < T; ++t) {
      double s = Y[(size_t)i * ldy + t];
      for (int k = 0; k < K; ++k) s -= Xi[(size_t)k * ldx + t] * PAI[(size_t)i * ldk + k];
      out[t] = s;
    }
  };
  auto set_col = [&](int i) {  // E(:, i) <- Y_i - X_i PAI_i, EA updated by the change
    resid_col(i, col.data());
    for (int t = 0; t < T; ++t) {
      const double dlt = col[t] - E[(size_t)i * T + t];
      E[(size_t)i * T + t] = col[t];
      const double* Am = At(t);
      for (int r = i; r < N; ++r) EA[(size_t)r * T + t] += dlt * Am[r + (size_t)i * N];
    }
  };
  for (int i = 0; i < N; ++i) set_col(i);
  std::vector<double> G((size_t)K * K), rhs(K), w2(T), u(T), xw(K);
  for (int j = 0; j < N; ++j) {
    const double* X = Xs[j];
    for (int k = 0; k < K; ++k) PAI[(size_t)j * ldk + k] = 0.0;
    set_col(j);
    // w2 and u(t) = sum_{i >= j} A(i, j) ytil_i(t) / lambda_i(t), ytil_i = EA(:, i) / lambda_i
    for (int t = 0; t < T; ++t) {
      double a = 0.0, b = 0.0;
      const double* Am = At(t);
      for (int i = j; i < N; ++i) {
        const double lam = sqrtht[(size_t)i * ldh + t];
        const double aij = Am[i + (size_t)j * N];
        a += aij * aij / (lam * lam);
        b += aij * EA[(size_t)i * T + t] / (lam * lam);
      }
      w2[t] = a;
      u[t] = b;
    }
    for (int k = 0; k < K; ++k) {
      double s = iVb[(size_t)j * ldk + k];
      for (int t = 0; t < T; ++t) s += X[(size_t)k * ldx + t] * u[t];
      rhs[k] = s;
    }
    bool ok = false;
    std::vector<double> Lp;
    if (!force_qr) {
      for (int c = 0; c < K; ++c)
        for (int r = c; r < K; ++r) {
          double s = (r == c) ? iVdiag[(size_t)j * ldk + r] : 0.0;
          const double* xr = X + (size_t)r * ldx;
          const double* xc = X + (size_t)c * ldx;
          for (int t = 0; t < T; ++t) s += xr[t] * w2[t] * xc[t];
          G[r + (size_t)c * K] = s;
        }
      ok = chol_lower(G, K);
      if (ok) Lp.swap(G);
    }
    if (!ok) {  // CTA.m:84-89: qrM = [iVchol, X_j'], R = triu(qr(qrM', 0))'
      flags |= 1;
      const int m = K + T;
      std::vector<double> M((size_t)m * K, 0.0);
      for (int k = 0; k < K; ++k) {
        M[k + (size_t)k * m] = std::sqrt(iVdiag[(size_t)j * ldk + k]);
        const double* xk = X + (size_t)k * ldx;
        for (int t = 0; t < T; ++t) M[K + t + (size_t)k * m] = std::sqrt(w2[t]) * xk[t];
      }
      Lp = qr_lower(M, m, K);
      for (int k = 0; k < K; ++k)
        if (Lp[k + (size_t)k * K] == 0.0) flags |= 2;
      G.assign((size_t)K * K, 0.0);
    }
    // PAI(:, j) = Lp^{-T} (Lp^{-1} rhs + z_j)
    for (int r = 0; r < K; ++r) {
      double s = rhs[r];
      for (int k = 0; k < r; ++k) s -= Lp[r + (size_t)k * K] * xw[k];
      xw[r] = s / Lp[r + (size_t)r * K];
    }
    for (int r = 0; r < K; ++r) xw[r] += z[r + (size_t)K * j];
    for (int r = K - 1; r >= 0; --r) {
      double s = xw[r];
      for (int k = r + 1; k < K; ++k) s -= Lp[k + (size_t)r * K] * xw[k];
      xw[r] = s / Lp[r + (size_t)r * K];
    }
    for (int k = 0; k < K; ++k) PAI[(size_t)j * ldk + k] = xw[k];
    if (G.size() != (size_t)K * K) G.assign((size_t)K * K, 0.0);
    set_col(j);
  }
  return flags;
}

}  // namespace ccmm
