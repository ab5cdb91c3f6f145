// Predictive density of one kept draw per chain (mcmcVAR.m:298-381,
// mcmcVARshadowrateBlockHybrid.m:550-669): SV shock paths, the linear companion
// simulation (ltitr), the censored simulation, the Rao-Blackwellised mean path
// and the one-step predictive log scores (logscoreGaussian.m,
// logscoreGaussianCensored.m).
//
// k_fcst: one single-wave workgroup per (forecast draw nn, chain), plus one for the linear
// model's zero-shock mean path: PAI (Kx x N) staged in LDS, the lag state a ring of p blocks of N
// values in LDS (the companion shift x(1+N+r) <- x(1+r) becomes a head-pointer move), the shock
// side of the simulation formed ahead of the recursion in chunks of horizons.  k_fcst_scores: the
// four one-step log scores of each draw, one single-wave workgroup per (draw, chain), over an
// N x N LDS scratch (N <= 32): ~N^3 flop per draw.
#include "ccmm_fcst.h"

namespace ccmm {


__device__ inline double ncdf(double x) { return 0.5 * erfc(-x * 0.70710678118654752440); }

// Genz (2004) BVNU: P(X > dh, Y > dk), correlation r (Drezner & Wesolowsky 1990 form)
__device__ double bvnu(double dh, double dk, double r, const GLNodes& gl) {
  int ng, lg;
  const double ar = fabs(r);
  if (ar < 0.3) { ng = 0; lg = 3; }
  else if (ar < 0.75) { ng = 1; lg = 6; }
  else { ng = 2; lg = 10; }
  double h = dh, k = dk, hk = h * k, bvn = 0.0;
  const double twopi = 6.283185307179586477;
  if (ar < 0.925) {
    const double hs = (h * h + k * k) * 0.5, asr = asin(r);
    for (int i = 0; i < lg; ++i) {
      double sn = sin(asr * (gl.x[ng][i] + 1.0) * 0.5);
      bvn += gl.w[ng][i] * exp((sn * hk - hs) / (1.0 - sn * sn));
      sn = sin(asr * (-gl.x[ng][i] + 1.0) * 0.5);
      bvn += gl.w[ng][i] * exp((sn * hk - hs) / (1.0 - sn * sn));
    }
    return fmax(0.0, fmin(1.0, bvn * asr / (2.0 * twopi) + ncdf(-h) * ncdf(-k)));
  }
  if (r < 0) { k = -k; hk = -hk; }
  if (ar < 1.0) {
    const double as = (1.0 - r) * (1.0 + r);
    double a = sqrt(as);
    const double bs = (h - k) * (h - k);
    const double c = (4.0 - hk) / 8.0, d = (12.0 - hk) / 16.0;
    bvn = a * exp(-(bs / as + hk) * 0.5) *
          (1.0 - c * (bs - as) * (1.0 - d * bs / 5.0) / 3.0 + c * d * as * as / 5.0);
    if (hk > -160.0) {
      const double b = sqrt(bs);
      bvn -= exp(-hk * 0.5) * sqrt(twopi) * ncdf(-b / a) * b * (1.0 - c * bs * (1.0 - d * bs / 5.0) / 3.0);
    }
    a *= 0.5;
    for (int i = 0; i < lg; ++i) {
      for (int sgn = -1; sgn <= 1; sgn += 2) {
        double xs = a * (sgn * gl.x[ng][i] + 1.0);
        xs *= xs;
        const double rs = sqrt(1.0 - xs);
        bvn += a * gl.w[ng][i] *
               (exp(-bs / (2.0 * xs) - hk / (1.0 + rs)) / rs - exp(-(bs / xs + hk) * 0.5) * (1.0 + c * xs * (1.0 + d * xs)));
      }
    }
    bvn = -bvn / twopi;
  }
  // the result clamped to [0, 1] as Genz's BVNU returns it (BVNU = MAX(0, MIN(1, BVN))) and
  // MATLAB's bivariate mvncdf with it: far in the tails the cancellation below can leave a
  // probability of order -1e-17, whose log would turn the draw's score (and the vintage's log
  // mean exp) into NaN
  if (r > 0) return fmax(0.0, fmin(1.0, bvn + ncdf(-fmax(h, k))));
  bvn = -bvn;
  if (k > h) bvn += ncdf(k) - ncdf(h);
  return fmax(0.0, fmin(1.0, bvn));
}

// Trivariate normal P(X <= x), X ~ N(0, L L') with L lower 3x3 (ld kFcstMaxN at M):
// P = int_{-inf}^{x1/L11} phi(z) BVN(h(z), k(z); rho) dz with the conditional
// bivariate of (X2, X3) | z (Genz BVN inside).  The integrand steps where h or k
// changes sign, so the outer interval is split there and each segment integrated
// on panels graded geometrically towards both ends (20-point Gauss-Legendre):
// panel j of a side spans [w0 (2^j - 1), min(w0 (2^(j+1) - 1), half)] from that end.
// MATLAB's mvncdf (trivariate rule, absolute tolerance 1e-8) is the reference.
// Called by all 64 lanes of a wave with identical arguments: the (segment, side, panel,
// node) evaluations are spread over the lanes and summed with one wave reduction.
__device__ double tvn_cdf(const double* x, const double* M, const GLNodes& gl, int lane) {
  const double l11 = M[0], l21 = M[1], l31 = M[2];
  const double l22 = M[1 + kFcstMaxN], l32 = M[2 + kFcstMaxN], l33 = M[2 + 2 * kFcstMaxN];
  const double s3 = sqrt(l32 * l32 + l33 * l33), rho = l32 / s3;
  const double b = x[0] / l11;
  const double lo = -10.0, w0 = 1e-4;
  if (b <= lo) return 0.0;
  double brk[4];
  int nb = 0;
  brk[nb++] = lo;
  double cand[2] = {l21 != 0.0 ? x[1] / l21 : lo, l31 != 0.0 ? x[2] / l31 : lo};
  if (cand[0] > cand[1]) { const double t = cand[0]; cand[0] = cand[1]; cand[1] = t; }
  for (int i = 0; i < 2; ++i)
    if (cand[i] > brk[nb - 1] + 1e-12 && cand[i] < b - 1e-12) brk[nb++] = cand[i];
  brk[nb++] = b;
  // panels per side of each segment
  int npan[3];
  int total = 0;
  for (int sgm = 0; sgm + 1 < nb; ++sgm) {
    const double half = 0.5 * (brk[sgm + 1] - brk[sgm]);
    int n = 0;
    double pos = 0.0, w = fmin(w0, half);
    while (pos < half) {
      pos += fmin(w, half - pos);
      w *= 2.0;
      ++n;
    }
    npan[sgm] = n;
    total += 2 * n * 20;
  }
  double acc = 0.0;
  for (int q = lane; q < total; q += 64) {
    int rem = q, sgm = 0;
    while (rem >= 2 * npan[sgm] * 20) { rem -= 2 * npan[sgm] * 20; ++sgm; }
    const int side = rem / (npan[sgm] * 20);
    rem -= side * npan[sgm] * 20;
    const int j = rem / 20, node = rem - j * 20;
    const double a0 = brk[sgm], a1 = brk[sgm + 1];
    const double half = 0.5 * (a1 - a0);
    const double wj = fmin(w0, half) * exp2((double)j);
    const double u0 = (j == 0) ? 0.0 : fmin(w0, half) * (exp2((double)j) - 1.0);
    const double u1 = fmin(u0 + wj, half);
    const double c = 0.5 * (u0 + u1), r = 0.5 * (u1 - u0);
    const int i = node >> 1;
    const double sg = (node & 1) ? 1.0 : -1.0;
    const double u = c + sg * r * gl.x[2][i];
    const double z = side == 0 ? a0 + u : a1 - u;
    const double h = (x[1] - l21 * z) / l22, k = (x[2] - l31 * z) / s3;
    acc += gl.w[2][i] * exp(-0.5 * z * z) * bvnu(-h, -k, rho, gl) * r;
  }
  return fmax(0.0, fmin(1.0, wave_sum(acc) * 0.39894228040143267794));  // Genz TVNU: MAX(0, MIN(1, TVN))
}

// P(X <= x) for X ~ N(0, L L'), L lower d x d (ld kFcstMaxN), 4 <= d <= kMvnMaxD: MATLAB's mvncdf
// integrates four or more dimensions by randomised quasi-Monte Carlo (absolute error tolerance
// 1e-4), which no restatement can reproduce draw for draw.  This is a deterministic estimate
// inside that tolerance: Genz's separation of variables (e_1 = Phi(x_1 / L_11), then
// y_{i-1} = Phi^-1(w_{i-1} e_{i-1}), e_i = Phi((x_i - sum_j L_ij y_j) / L_ii), integrand
// e_1 ... e_d) on a fixed rank-1 lattice of kMvnPts points (generators frac(sqrt(prime_i)),
// tent-periodised) spread over the lanes, summed by one wave reduction.  Typical error ~1e-7 at 65536 points
// (tests: against an independent randomised lattice rule at 1e-6, and bit-level against the
// oracle's restatement of this rule, oracle/ccmm_oracle_fcst.mvn_lattice_cdf).
constexpr int kMvnMaxD = 12;
constexpr int kMvnPts = 64 * 1024;
__device__ double mvn_lattice_cdf(const double* x, const double* M, int d, int lane) {
  const double alpha[kMvnMaxD - 1] = {1.4142135623730951, 1.7320508075688772, 2.2360679774997898,
                                      2.6457513110645907, 3.3166247903554, 3.605551275463989,
                                      4.123105625617661, 4.358898943540674, 4.795831523312719,
                                      5.385164807134504, 5.5677643628300215};
  const double e1 = ncdf(x[0] / M[0]);
  if (!(e1 > 0.0)) return 0.0;
  double acc = 0.0;
  for (int q = lane; q < kMvnPts; q += 64) {
    double yv[kMvnMaxD];
    double e = e1, f = e1;
    for (int i = 1; i < d && f > 0.0; ++i) {
      double w = (double)(q + 1) * alpha[i - 1];
      w -= floor(w);
      w = fabs(2.0 * w - 1.0);
      const double pw = fmin(fmax(w * e, 1e-300), 1.0 - 1e-16);
      yv[i - 1] = normcdfinv(pw);
      double sdot = 0.0;
      for (int j = 0; j < i; ++j) sdot = fma(M[i + j * kFcstMaxN], yv[j], sdot);
      e = ncdf((x[i] - sdot) / M[i + i * kFcstMaxN]);
      f *= e;
    }
    acc += f;
  }
  return fmax(0.0, fmin(1.0, wave_sum(acc) / (double)kMvnPts));
}

// in-place lower Cholesky of an n x n LDS matrix (ld = kFcstMaxN); false if not SPD.
// Called by all 64 lanes of a wave with identical arguments: lane r computes row j + 1 + r
// of column j (n <= 32: one pass), every entry with the same operation order as the
// serial column-by-column form, so the factor is bit-identical to it.
__device__ bool chol_lds(double* M, int n, int lane) {
  for (int j = 0; j < n; ++j) {
    double s = M[j + j * kFcstMaxN];
    for (int k = 0; k < j; ++k) s -= M[j + k * kFcstMaxN] * M[j + k * kFcstMaxN];
    if (!(s > 0.0)) return false;
    const double dj = sqrt(s);
    const int i = j + 1 + lane;
    double v = 0.0;
    if (i < n) {
      v = M[i + j * kFcstMaxN];
      for (int k = 0; k < j; ++k) v -= M[i + k * kFcstMaxN] * M[j + k * kFcstMaxN];
      v = v / dj;
    }
    wave_lds_sync();
    if (lane == 0) M[j + j * kFcstMaxN] = dj;
    if (i < n) M[i + j * kFcstMaxN] = v;
    wave_lds_sync();
  }
  return true;
}

// Omega = S(rows) S(rows)' for the index list rows[0..n) of S = invA diag(sv) (lower
// triangular): M = chol(Omega, 'lower') (the chol(sqrtOmega(ndx,:)*sqrtOmega(ndx,:)')
// of mcmcVAR.m:342,347 and logscoreGaussianCensored.m:54-56).  Lanes split the Gram
// entries (same k order per entry as the serial loop).
__device__ bool gram_rows_chol(const double* invA, const double* sv, const int* rows, int n,
                               int N, double* M, int lane) {
  wave_lds_sync();
  for (int e = lane; e < n * n; e += 64) {
    const int a = e / n, b = e - a * n;
    if (b > a) continue;
    const int ra = rows[a], rb = rows[b];
    const int kmax = ra < rb ? ra : rb;
    double s = 0.0;
    for (int k = 0; k <= kmax; ++k) s += invA[ra + k * N] * invA[rb + k * N] * sv[k] * sv[k];
    M[a + b * kFcstMaxN] = s;
    M[b + a * kFcstMaxN] = s;
  }
  wave_lds_sync();
  return chol_lds(M, n, lane);
}

// logscoreGaussian.m:15-20 with lower-triangular L (ld kFcstMaxN), dev = y - mu (overwritten)
__device__ double score_gauss(const double* L, int n, double* dev, double logdet) {
  double ss = 0.0;
  for (int i = 0; i < n; ++i) {
    double v = dev[i];
    for (int k = 0; k < i; ++k) v -= L[i + k * kFcstMaxN] * dev[k];
    v /= L[i + i * kFcstMaxN];
    dev[i] = v;
    ss += v * v;
  }
  return -0.5 * (n * 1.8378770664093454836 + logdet + ss);
}

__device__ double logdet_chol(const double* L, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += log(L[i + i * kFcstMaxN]);
  return 2.0 * s;
}

// logscoreGaussianCensored.m:13-88 as written.  sel[0..n) = the series scored (in
// order), cens[i] whether series sel[i] may be censored.  Four or more series at the ELB: the
// deterministic lattice estimate above (MATLAB mvncdf's randomised QMC, tolerance 1e-4); NaN (and
// *unsupported) above kMvnMaxD.
__device__ double score_censored(const double* invA, const double* sv, const double* mu,
                                 const double* y, const int* sel, const uint8_t* cens, int n,
                                 int N, double elb, double* M, double* dev, int* order,
                                 const GLNodes& gl, bool* unsupported, int lane) {
  int noff = 0, nat = 0;
  for (int i = 0; i < n; ++i)
    if (!(cens[i] && y[sel[i]] <= elb)) order[noff++] = sel[i];
  for (int i = 0; i < n; ++i)
    if (cens[i] && y[sel[i]] <= elb) { order[noff + nat] = sel[i]; ++nat; }
  if (nat > kMvnMaxD) { *unsupported = true; return NAN; }
  if (!gram_rows_chol(invA, sv, order, n, N, M, lane)) return NAN;
  double llf1 = 0.0;
  double y21[kMvnMaxD], yat[kMvnMaxD];
  for (int a = 0; a < nat; ++a) { y21[a] = mu[order[noff + a]]; yat[a] = y[order[noff + a]]; }
  if (noff > 1) {
    for (int i = 0; i < noff; ++i) dev[i] = y[order[i]] - mu[order[i]];
    llf1 = score_gauss(M, noff, dev, logdet_chol(M, noff));  // dev now z1
    for (int a = 0; a < nat; ++a)
      for (int k = 0; k < noff; ++k) y21[a] += M[(noff + a) + k * kFcstMaxN] * dev[k];
  }
  double llf2;
  const double l11 = M[noff + noff * kFcstMaxN];
  if (nat == 1) {
    llf2 = log(ncdf((yat[0] - y21[0]) / l11));
  } else if (nat == 2) {
    // Sigma22 = L22 L22': sd1 = l11, cov = l11 l21, var2 = l21^2 + l22^2
    const double l21 = M[(noff + 1) + noff * kFcstMaxN];
    const double l22 = M[(noff + 1) + (noff + 1) * kFcstMaxN];
    const double s2 = sqrt(l21 * l21 + l22 * l22);
    const double rho = l21 / s2;
    const double h = (yat[0] - y21[0]) / l11, k = (yat[1] - y21[1]) / s2;
    llf2 = log(bvnu(-h, -k, rho, gl));
  } else if (nat == 3) {
    const double xv[3] = {yat[0] - y21[0], yat[1] - y21[1], yat[2] - y21[2]};
    llf2 = log(tvn_cdf(xv, M + noff + noff * kFcstMaxN, gl, lane));
  } else {
    double xv[kMvnMaxD];
    for (int a = 0; a < nat; ++a) xv[a] = yat[a] - y21[a];
    llf2 = log(mvn_lattice_cdf(xv, M + noff + noff * kFcstMaxN, nat, lane));
  }
  return llf1 + llf2;
}

// Linear model (mcmcVAR.m:298-381): ring l = the linear simulation, ring c = the
// censored simulation (yields floored inside the recursion, :354-372), plus the
// zero-shock mean path.  Block hybrid (mcmcVARshadowrateBlockHybrid.m:566-625): ONE
// simulation on the Nstates = K + Nyields p state; ring l holds the shadow lags, ring c
// the same lags with every yield replaced by its actual rate max(y, ELB) (:623, the
// actual-rate states fcstX0(ndxfcstActual)); the actual-rate equations read ring c (their
// PAIactual on the yield lags, PAIshadow zero there: :567-574), the others ring l.
//
// k_fcst: one single-wave workgroup per (forecast draw, chain) -- job Nd is the linear model's
// zero-shock mean path.  The shock side of the simulation does not depend on the simulated
// path, so it is formed for a chunk of hc horizons at once by all 64 lanes before the
// recursion: the SV normals and their sqrtPHI products, the log-volatility random walk
// (mcmcVAR.m:302-312), the structural shocks w = sv .* z and their impact nu = invA w.  The
// recursion itself (one horizon after the other) then only carries the companion product
// fcstA * state, its 2 N p lag products spread over G lane groups (lane = i + N g takes the lags
// l = g mod G) whose partials lane i adds by shuffles.  The draw's SV at horizon 1 goes to
// a.sv1 for k_fcst_scores.
//

template <int RN>
__global__ __launch_bounds__(64, 2) void k_fcst(FcstArgs a) {
  extern __shared__ double sm[];
  const int job = blockIdx.x, c = blockIdx.y;
  const int N = a.N, K = a.K, p = a.p, H = a.H, Nd = a.Nd, Kx = a.Kx, hc = a.hc;
  const int lane = threadIdx.x;
  const int njobs = a.bh ? Nd : Nd + 1;
  if (job >= njobs) return;
  const bool mean_path = job == Nd;
  constexpr bool REG = RN > 0;
  double* sPAI = sm;                          // Kx x N (column i = equation i); none when REG
  double* sSq = sPAI + (REG ? 0 : (size_t)Kx * N);  // sqrtPHI, N x N column-major
  double* sinvA = sSq + N * N;                // invA, N x N column-major
  double* ringl = sinvA + N * N;              // p x N
  double* ringc = ringl + p * N;              // p x N
  double* Wb = ringc + p * N;                 // hc x N: zz, then w = sv .* zz
  double* NUb = Wb + (size_t)hc * N;          // hc x N: sqrtPHI dev, then nu = invA w
  double* DVb = NUb + (size_t)hc * N;         // hc x N: the SV normals dev
  const int sl = a.slot ? a.slot[c] : 0;
  const bool hy = a.bh == 2;
  const double* PAIc = a.PAI + (size_t)c * a.ldPAI * N;
  if (!REG)
    for (int e = lane; e < Kx * N; e += 64) {
      const int j = e / Kx, k = e - j * Kx;
      sPAI[e] = PAIc[(size_t)j * a.ldPAI + k];
    }
  const double* Xj = a.Xj + (size_t)c * a.ldXj;
  for (int e = lane; e < N * N; e += 64) {
    sinvA[e] = a.invA[(size_t)c * N * N + e];
    sSq[e] = a.sqrtPHI[(size_t)c * N * N + e];
  }
  int hs[kElbNsMax] = {-1, -1, -1, -1, -1};  // hybrid: indices of the shadow-rate variables
  if (hy)
    for (int q = 0; q < a.Ns && q < kElbNsMax; ++q) hs[q] = a.ndxS[q];
  const int tsv = a.svT ? a.svT[sl] - 1 : 0;
  const double* svz = a.svz ? a.svz + (size_t)c * a.crnStride : nullptr;
  const double* zc = a.z ? a.z + (size_t)c * a.crnStride : nullptr;
  const bool isact = a.bh == 1 && lane < N && a.actual[lane];
  const bool isyield = lane < N && a.ndxYields[lane];
  const bool isrec = lane < N && (a.recFloor ? a.recFloor[lane] : a.ndxYields[lane]);
  Rng rng;
  rng.crn = nullptr;
  rng.seed = a.seed;
  rng.chain = a.ids ? a.ids[c] : (uint32_t)c;
  rng.sweep = a.sweep;
  const int nsv = N * H * Nd;
  // ring blocks: slot (head - l) mod p holds lag l+1 (l = 0..p-1)
  for (int e = lane; e < p * N; e += 64) {
    const int l = e / N, j = e - l * N;  // lag l+1 goes to slot (-l) mod p
    const int slot = (l == 0) ? 0 : p - l;
    ringl[slot * N + j] = Xj[1 + e];
    // block hybrid: yields carry their actual-rate lags (Xjumpoff(K+1:end), :93-96);
    // hybrid: the shadow-rate variables carry theirs (Xjumpoff(Kshadow+1:end), :111-121)
    double cv = Xj[1 + e];
    if (a.bh == 1 && a.ndxYields[j]) cv = Xj[K + e];
    if (hy)
      for (int q = 0; q < a.Ns && q < kElbNsMax; ++q)
        if (hs[q] == j) cv = Xj[K + l * a.Ns + q];
    ringc[slot * N + j] = cv;
  }
  double logsv = (lane < N) ? a.logSV[((size_t)c * N + lane) * a.ldSV + tsv] : 0.0;
  const int G = N <= 21 ? 3 : (N <= 32 ? 2 : 1);  // lane groups of the lag sums (G N <= 64)
  const int g = lane / N, gi = lane - g * N;
  const double* pcol = sPAI + (size_t)(g < G ? gi : 0) * Kx;
  // REG: lane (gi, g) holds PAI(1 + l N + j, gi) for its lags l = g + G m, and the intercept
  double cf[REG ? kFcstRegLags : 1][REG ? RN : 1];
  double c0 = 0.0;
  if (REG) {
    const double* pg = PAIc + (size_t)(g < G ? gi : 0) * a.ldPAI;
    c0 = pg[0];
#pragma unroll
    for (int m = 0; m < (REG ? kFcstRegLags : 1); ++m) {
      const int l = g + G * m;
#pragma unroll
      for (int j = 0; j < (REG ? RN : 1); ++j)
        cf[m][j] = (g < G && l < p && j < N) ? pg[1 + l * N + j] : 0.0;
    }
  }
  int head = 0;
  __syncthreads();
  for (int h0 = 0; h0 < ((a.mode & 2) ? 0 : H); h0 += hc) {
    const int nh = min(hc, H - h0);
    if (!mean_path) {
      // SV normals randn(N, H*Nd) column hh + job H (mcmcVAR.m:302) and the shock normals
      // randn(N, H, Nd) (:306) of the chunk's horizons
      for (int q = lane; q < nh * N; q += 64) {
        const int hh = h0 + q / N, i = q - (q / N) * N;
        const int col = hh + job * H;
        DVb[q] = svz ? svz[(size_t)col * N + i] : rng.normal(CCMM_RNG_FCST, (uint32_t)(col * N + i));
        const size_t zi = ((size_t)job * H + hh) * N + i;
        Wb[q] = zc ? zc[zi] : rng.normal(CCMM_RNG_FCST, (uint32_t)(nsv + zi));
      }
      wave_lds_sync();
      for (int q = lane; q < nh * N; q += 64) {  // sqrtPHI * dev, j in order
        const int hq = q / N, i = q - hq * N;
        const double* dv = DVb + (size_t)hq * N;
        double shock = 0.0;
        for (int j = 0; j < N; ++j) shock = fma(sSq[i + j * N], dv[j], shock);
        NUb[q] = shock;
      }
      wave_lds_sync();
      if (lane < N)  // the log-volatility random walk and w = sv .* z
        for (int hq = 0; hq < nh; ++hq) {
          logsv += NUb[hq * N + lane];
          const double sv = exp(logsv * 0.5);
          Wb[hq * N + lane] *= sv;
          if (h0 + hq == 0) a.sv1[((size_t)c * Nd + job) * N + lane] = sv;
        }
      wave_lds_sync();
      for (int q = lane; q < nh * N; q += 64) {  // nu = invA w (invA unit lower, j = 0..i)
        const int hq = q / N, i = q - hq * N;
        const double* wv = Wb + (size_t)hq * N;
        double nu = 0.0;
        for (int j = 0; j <= i; ++j) nu = fma(sinvA[i + j * N], wv[j], nu);
        NUb[q] = nu;
      }
      wave_lds_sync();
    }
    for (int hq = 0; hq < nh; ++hq) {
      const int hh = h0 + hq;
      // fcstA * state on the lane groups
      double sl2 = 0.0, sc = 0.0;
      if (REG) {
        if (g < G) {
          if (g == 0) sl2 = sc = Xj[0] * c0;
#pragma unroll
          for (int m = 0; m < (REG ? kFcstRegLags : 1); ++m) {
            const int l = g + G * m;
            if (l < p) {
              int slot = head - l;
              slot += (slot < 0) ? p : 0;
              const double* rl = ringl + slot * N;
              const double* rc = ringc + slot * N;
              if (RN % 2 == 0) {  // N even: the ring rows are 16-byte aligned, two lags' entries a read
#pragma unroll
                for (int j = 0; j < (REG ? RN : 1); j += 2)
                  if (j < N) {
                    const double2 vl = *reinterpret_cast<const double2*>(rl + j);
                    const double2 vc = *reinterpret_cast<const double2*>(rc + j);
                    sl2 = fma(cf[m][j], vl.x, sl2);
                    sc = fma(cf[m][j], vc.x, sc);
                    sl2 = fma(cf[m][j + 1], vl.y, sl2);
                    sc = fma(cf[m][j + 1], vc.y, sc);
                  }
              } else {
#pragma unroll
                for (int j = 0; j < (REG ? RN : 1); ++j)
                  if (j < N) {
                    sl2 = fma(cf[m][j], rl[j], sl2);
                    sc = fma(cf[m][j], rc[j], sc);
                  }
              }
            }
          }
        }
      } else if (g < G) {
        if (g == 0) sl2 = sc = Xj[0] * pcol[0];  // constant state stays 1 (fcstA(1,1) = 1)
        for (int l = g; l < p; l += G) {
          int slot = head - l;
          slot += (slot < 0) ? p : 0;
          const double* rl = ringl + slot * N;
          const double* rc = ringc + slot * N;
          const double* pc = pcol + 1 + l * N;
#pragma unroll 4
          for (int j = 0; j < N; ++j) {
            sl2 = fma(pc[j], rl[j], sl2);
            sc = fma(pc[j], rc[j], sc);
          }
          if (hy)  // fcstA(ndxfcstY, Kshadow+1:end) on the actual-rate ring (:626)
            for (int q = 0; q < a.Ns && q < kElbNsMax; ++q) sl2 = fma(pcol[K + l * a.Ns + q], rc[hs[q]], sl2);
        }
      }
      // every group's partial is read before any lane adds (lane i + N is also the source of
      // lane i's group-2 partial through lane i + 2N ... and must still hold its own)
      double pl[2] = {0.0, 0.0}, pcs[2] = {0.0, 0.0};
      for (int q = 1; q < G; ++q) {
        pl[q - 1] = __shfl(sl2, lane + q * N, 64);
        pcs[q - 1] = __shfl(sc, lane + q * N, 64);
      }
      for (int q = 1; q < G; ++q) {
        sl2 += pl[q - 1];
        sc += pcs[q - 1];
      }
      double yl = 0.0, yc = 0.0;
      if (lane < N) {
        const double nu = mean_path ? 0.0 : NUb[hq * N + lane];
        if (hy) {
          yl = sl2 + nu;
          yc = (isyield && yl < a.elb) ? a.elb : yl;  // yields floored (:707-711); ring: max(shadow, ELB) (:634)
        } else if (a.bh) {
          yl = (isact ? sc : sl2) + nu;               // fcstA * fcstX0 + fcstB * shocks (:615)
          yc = (isyield && yl < a.elb) ? a.elb : yl;  // actual rate max(shadow, ELB) (:623)
        } else {
          yl = sl2 + nu;
          yc = sc + nu;
          if (isrec && yc < a.elb) yc = a.elb;        // censored simulation (mcmcVAR.m:360-366)
        }
        if (mean_path) {
          a.yhat[((size_t)c * H + hh) * N + lane] = yl;
        } else {
          const size_t o = (((size_t)c * Nd + job) * H + hh) * N + lane;
          a.fY[o] = yl;
          a.fYc[o] = yc;
        }
      }
      wave_lds_sync();  // every lane has read the oldest lag block before it is overwritten
      head = (head + 1 == p) ? 0 : head + 1;
      if (lane < N) {
        ringl[head * N + lane] = yl;
        ringc[head * N + lane] = yc;
      }
      wave_lds_sync();
    }
  }
}

// One-step predictive log scores of draw `job` of chain c (mcmcVAR.m:326-352; block hybrid
// :577-608), one single-wave workgroup per (draw, chain): every lane runs the same scalar algebra
// (uniform control flow, identical LDS writes); the trivariate mvncdf quadrature and the lattice
// rule spread their nodes over the lanes.  Reads the draw's SV at horizon 1 (a.sv1, k_fcst).

__global__ __launch_bounds__(64) void k_fcst_scores(FcstArgs a) {
  extern __shared__ double sm[];
  const int job = blockIdx.x, c = blockIdx.y;
  const int N = a.N, K = a.K, Kx = a.Kx, Nd = a.Nd;
  const int lane = threadIdx.x;
  if (job >= Nd || (a.mode & 1)) return;
  double* invA = sm;                  // N x N
  double* mu = invA + N * N;          // muY (N)
  double* y = mu + N;                 // yrealized(:,1) (N)
  double* sv1 = y + N;                // SV at horizon 1 (N)
  double* dev = sv1 + N;              // N
  int* order = (int*)(dev + N);       // N ints
  int* sel = (int*)(dev + 2 * N);     // N ints
  uint8_t* cens = (uint8_t*)(sel + N);  // N bytes (same N-double slot)
  double* M = dev + 3 * N;            // kFcstMaxN^2
  int* syl = (int*)(M + kFcstMaxN * kFcstMaxN);  // yield flags (N ints in N doubles)
  const int sl = a.slot ? a.slot[c] : 0;
  for (int e = lane; e < N * N; e += 64) invA[e] = a.invA[(size_t)c * N * N + e];
  if (lane < N) {
    y[lane] = a.yreal[(size_t)sl * a.ldY + lane];
    sv1[lane] = a.sv1[((size_t)c * Nd + job) * N + lane];
    syl[lane] = a.ndxYields[lane];
  }
  __syncthreads();
  // muY = fcstA(ndxfcstY, :) * Xjumpoff (mcmcVAR.m:326-328; block hybrid :577-580: the actual-rate
  // equations read the yields' actual-rate lags)
  const double* Xj = a.Xj + (size_t)c * a.ldXj;
  const double* PAIc = a.PAI + (size_t)c * a.ldPAI * N;
  if (lane < N) {
    const int i = lane;
    const bool act = a.bh == 1 && a.actual[i];
    const double* col = PAIc + (size_t)i * a.ldPAI;
    double s = 0.0;
    for (int k = 0; k < K; ++k) {
      const double xv = (act && k > 0 && syl[(k - 1) % N]) ? Xj[K + k - 1] : Xj[k];
      s += col[k] * xv;
    }
    for (int k = K; k < Kx; ++k) s += col[k] * Xj[k];  // hybrid: actual-rate lags (:592-594)
    mu[i] = s;
  }
  __syncthreads();
  int nx = 0, ni = 0, natelb = 0;
  for (int i = 0; i < N; ++i) {
    if (a.ndxYields[i]) {
      ++ni;
      natelb += (y[i] <= a.elb);
    } else {
      ++nx;
    }
  }
  double sc[4];
  bool unsupported = false;
  // (1) full vector: sqrtOmegaY = invA diag(sv1) is lower triangular, logdet = sum logSV(:,1)
  {
    double ld = 0.0;
    for (int i = 0; i < N; ++i) {
      M[i + i * kFcstMaxN] = sv1[i];  // unit-diagonal invA times sv
      for (int r2 = i + 1; r2 < N; ++r2) M[r2 + i * kFcstMaxN] = invA[r2 + i * N] * sv1[i];
      ld += 2.0 * log(sv1[i]);
      dev[i] = y[i] - mu[i];
    }
    sc[0] = score_gauss(M, N, dev, ld);
  }
  // (2) censored full vector (ndxYIELDS censorable); the block-hybrid fcstLogscoreDraws
  if (natelb > 0) {
    for (int i = 0; i < N; ++i) {
      order[i] = i;
      cens[i] = a.ndxYields[i];
    }
    for (int i = 0; i < N; ++i) sel[i] = i;
    sc[1] = score_censored(invA, sv1, mu, y, sel, cens, N, N, a.elb, M, dev, order, a.gl, &unsupported, lane);
  } else {
    sc[1] = sc[0];
  }
  // (3) macro block
  {
    int q = 0;
    for (int i = 0; i < N; ++i)
      if (!a.ndxYields[i]) sel[q++] = i;
    if (gram_rows_chol(invA, sv1, sel, nx, N, M, lane)) {
      for (int i = 0; i < nx; ++i) dev[i] = y[sel[i]] - mu[sel[i]];
      sc[2] = score_gauss(M, nx, dev, logdet_chol(M, nx));
    } else {
      sc[2] = NAN;
    }
  }
  // (4) yields block: every yield censorable
  {
    int q = 0;
    for (int i = 0; i < N; ++i)
      if (a.ndxYields[i]) {
        sel[q] = i;
        cens[q] = 1;
        ++q;
      }
    if (natelb > 0) {
      sc[3] = score_censored(invA, sv1, mu, y, sel, cens, ni, N, a.elb, M, dev, order, a.gl, &unsupported, lane);
    } else if (gram_rows_chol(invA, sv1, sel, ni, N, M, lane)) {
      for (int i = 0; i < ni; ++i) dev[i] = y[sel[i]] - mu[sel[i]];
      sc[3] = score_gauss(M, ni, dev, logdet_chol(M, ni));
    } else {
      sc[3] = NAN;
    }
  }
  if (lane == 0) {
    for (int q = 0; q < 4; ++q) a.scores[((size_t)c * Nd + job) * 4 + q] = sc[q];
    if (unsupported) atomicOr(&a.status[c], 2);
  }
}

// Xjumpoff of every chain from its resident data (mcmcVAR.m:108-115;
// mcmcVARshadowrateBlockHybrid.m:511-520): [1, y(T), ..., y(T-p+1)] from the chain's Y
// slab (block hybrid: the shadow-rate data), then p blocks of N lags of the slot's
// actual data (the block-hybrid actual-rate states, data(Nobs-(l-1), ndxYIELDS)).
// Hybrid (Ns > 0): the tail holds p blocks of the Ns shadow-rate variables' actual data floored at
// the ELB, XjumpoffActualYieldLags (mcmcVARhybridGibbs.m:111-121, 536).
__global__ void k_fcst_jumpoff(int N, int p, int K, int TP, const int* __restrict__ Tslot,
                               const int* __restrict__ slot, const double* __restrict__ ypool,
                               const int* __restrict__ yidx, int ldXj, double* __restrict__ Xj, int Ns,
                               const int* __restrict__ ndxS, double elb) {
  const int c = blockIdx.x;
  const int s = slot[c];
  const int T = Tslot[s];
  const double* Ych = ypool + (size_t)yidx[c] * N * TP;
  const double* Ysl = ypool + (size_t)s * N * TP;
  for (int e = threadIdx.x; e < ldXj; e += blockDim.x) {
    double v = 1.0;
    if (e > 0 && e < K) {
      const int q = e - 1, l = q / N, i = q - l * N;
      v = Ych[(size_t)i * TP + T - 1 - l];
    } else if (e >= K && Ns > 0) {
      const int q = e - K, l = q / Ns, si = q - l * Ns;
      v = 0.0;
      if (l < p) {
        const double yv = Ysl[(size_t)ndxS[si] * TP + T - 1 - l];
        v = yv < elb ? elb : yv;
      }
    } else if (e >= K) {
      const int q = e - K, l = q / N, i = q - l * N;
      v = Ysl[(size_t)i * TP + T - 1 - l];
    }
    Xj[(size_t)c * ldXj + e] = v;
  }
}

// Per kept draw: running sums of the paths over the Nd draws (the means of
// mcmcVAR.m:400-414 / BlockHybrid.m:693-742), the score draws into the store at index m
// (fcstLogscore*Draws(:, thisMCMCdraw)), and optionally the paths themselves.
__global__ void k_fcst_accum(int N, int H, int Nd, int cap, int m, const double* __restrict__ fY,
                             const double* __restrict__ fYc, const double* __restrict__ yhat,
                             const double* __restrict__ sc, double* __restrict__ sum,
                             double* __restrict__ sumc, double* __restrict__ sumhat,
                             double* __restrict__ scStore, double* __restrict__ paths,
                             double* __restrict__ pathsc) {
  const int c = blockIdx.x;
  const size_t HN = (size_t)H * N, per = (size_t)Nd * HN;
  const double* y = fY + (size_t)c * per;
  const double* yc = fYc + (size_t)c * per;
  for (size_t q = threadIdx.x; q < HN; q += blockDim.x) {
    double a = 0.0, b = 0.0;
    for (int job = 0; job < Nd; ++job) {
      a += y[(size_t)job * HN + q];
      b += yc[(size_t)job * HN + q];
    }
    sum[(size_t)c * HN + q] += a;
    sumc[(size_t)c * HN + q] += b;
    if (yhat) sumhat[(size_t)c * HN + q] += yhat[(size_t)c * HN + q];
  }
  for (int q = threadIdx.x; q < Nd * 4; q += blockDim.x)
    scStore[((size_t)c * cap + m) * Nd * 4 + q] = sc[(size_t)c * Nd * 4 + q];
  if (paths)
    for (size_t q = threadIdx.x; q < per; q += blockDim.x) {
      paths[((size_t)c * cap + m) * per + q] = y[q];
      pathsc[((size_t)c * cap + m) * per + q] = yc[q];
    }
}


// ---------------------------------------------------------------- instantiations launched by ccmm_abi.hip
template __global__ void k_fcst<0>(FcstArgs);
template __global__ void k_fcst<kFcstRegN - 1>(FcstArgs);
template __global__ void k_fcst<kFcstRegN>(FcstArgs);

}  // namespace ccmm
