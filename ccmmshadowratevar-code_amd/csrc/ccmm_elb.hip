// ELB shadow-rate step of the block-hybrid sampler (mcmcVARshadowrateBlockHybrid.m:395-520,
// gibbsdrawShadowrates.m, drawTruncNormal.m) for B chains.
//
// The reference computes, per censored month t, the smoothing weights J_t and the
// conditional covariance of the Ns shadow rates S_t by QR of a 260 x 260 matrix
// (gibbsdrawShadowrates.m:74-145).  They are the moments of the Gaussian
// S_t | X_t, past, y_{t+1..t+p} in the zero-mean VAR on Ytilde = Y - Y0, which
// factorises exactly into the prior of y_t given the past and p lag-equation
// likelihoods of the future months (oracle/elb_fast.py states the algebra):
//
//   Ω_t = (Λ_t,SS + Σ_k B_k' Λ_{t+k} B_k)^{-1},   Λ_τ = A' diag(SVol_τ)^-2 A,
//   Spost_t = Y0_S,t + Ω_t g_t(Ytilde),   B_k = Φ_k[:, S],
//
// g linear in Ytilde.  The kernels evaluate the same conditionals in a residual
// form that never builds Y0 (see k_elb_prep).  Per censored month we store the affine map
// Spost_t = a_t + Σ G_t[k'][s'] S(s', t ± k') over the censored neighbours, and
// the sequential Gibbs passes cost 2p Ns^2 multiply-adds per month.
//
//   k_elb_prep    per chain: Φ, Yhatactual, base residuals ε_τ (stable form, no Y0 path)
//   k_elb_cond    per (chain, censored month): Ω_t, a_t, G_t, conditional betas
//   k_elb_gibbs   per chain: burnin + 1 sequential passes, inverse-CDF truncated normals
//   k_elb_rebuild per chain: splice the shadow rates into the chain's Y and X (:501-509)
#include "ccmm_elb.h"

namespace ccmm {



// spec mode: the PS decision of this sweep for chain c: 0 undecided, 1 accepted, 2 rejected (sc1 load)
__device__ __forceinline__ int elb_ps_decision(const ElbDev& e, int c) {
  const unsigned long long v = __hip_atomic_load(&e.psState[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (v >> 1) != e.psEpoch ? 0 : ((v & 1) ? 1 : 2);
}


// ---------------------------------------------------------------- prep (per chain)
// Stable residual form (oracle/elb_fast.py, gibbsdraw_shadowrates_stable): the
// reference's Ytilde = Y - Y0 is never formed.  Y0 enters the conditionals only
// through the lag-equation residuals of its path,
//   e0_τ = [τ = 0: w_{-1};  τ >= 1: c + Σ_{l=τ+1..p} Φ_l w_{τ-1-l}] + yhat_τ - Σ_{l<=τ} Φ_l yhat_{τ-l}
// (w_{-1-i} = lag block i of elb.X0), bounded by the data even when the companion
// matrix is explosive, where the as-written form loses all digits to cancellation.
//   Yt[τ] = Yb_τ   (the chain's Y with censored shadow-rate cells at 0)
//   Et[τ] = ε_τ = Yb_τ - Σ_{l<=τ} Φ_l Yb_{τ-l} - e0_τ
// phi_lds bit 0: stage Φ in LDS (N (Np + 1) doubles; N <= 32); else it is read back from e.Phi
// rows > 0 (small batches, phi_lds & 2): workgroup blockIdx.y forms the residual rows
// [rows y, rows (y + 1)) of the window only, from the Yb / Z rows p months before them (the lag sums);
// the same values and operation order per row as one workgroup per chain
__global__ __launch_bounds__(kElbPrepThreads) void k_elb_prep(Dims d, ElbDev e, XSel xs, ChainState cs, int phi_lds,
                                                              int rows) {
  extern __shared__ double sm[];
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int N = d.N, KP = d.KP, TP = d.TP, p = e.p, Ns = e.Ns;
  const int Np = N * p, ldp = Np + 1;
  const int T0 = e.elbT0[s], T = e.elbT[s];
  if (T <= 0) return;
  // this workgroup's residual rows [ta, tb) and the Yb / Z rows they read [tz, tb)
  const int ta = rows > 0 ? blockIdx.y * rows : 0;
  if (ta >= T) return;
  const int tb = rows > 0 ? min(T, ta + rows) : T;
  const int tz = max(0, ta - p);
  const bool lead = blockIdx.y == 0;  // writes the chain-wide outputs (Φ, the Gibbs start values)
  const int tid = threadIdx.x;
  const double* PAI = cs.PAI + (size_t)c * N * KP;  // PAI(k, i) at [i*KP + k]
  double* Phi = e.Phi + (size_t)c * N * Np;
  double* Zg = e.Y0 + (size_t)c * e.elbTmax * N;    // Yb - yhat
  double* Ytg = e.Yt + (size_t)c * e.elbTmax * N;
  double* Et = e.Et + (size_t)c * e.elbTmax * N;
  double* X0 = sm;                   // K: elb.X0 = X(elbT0+1, :)'
  double* sPhi = sm + (2 + Np);      // N x ldp (phi_lds & 1)
  // phi_lds & 2: Yb - yhat and Yb also staged in LDS (T x N each), so that the lag sums of the residual
  // pass below read LDS instead of global memory (same values, same operation order)
  const bool zy_lds = (phi_lds & 2) != 0;
  double* Z = zy_lds ? sPhi + (size_t)N * ldp : Zg;
  double* Yt = zy_lds ? Z + (size_t)e.elbTmax * N : Ytg;
  // Φ = PAIshadow(2:1+Np, :)' with (ndxSHADOWRATELAGS, actualrateBlock) zeroed (:404-407)
  for (int q = tid; q < N * Np; q += kElbPrepThreads) {
    const int i = q / Np, kp = q % Np;
    bool zero = false;
    if (e.actual[i])
      for (int si = 0; si < Ns; ++si) zero |= (kp % N) == e.ndxS[si];
    const double v = zero ? 0.0 : PAI[(size_t)i * KP + 1 + kp];
    if (lead) Phi[q] = v;
    if (phi_lds & 1) sPhi[i * ldp + kp] = v;
  }
  const double* Xa = e.Xactual + (size_t)s * KP * TP;        // Xactual(t, k) at [k*TP + t]
  const double* Yc = xs.ypool + (size_t)xs.yidx[c] * N * TP;  // chain's Y(t, i) at [i*TP + t]
  for (int k = tid; k < 1 + Np; k += kElbPrepThreads) X0[k] = Xa[(size_t)k * TP + T0];
  const uint8_t* sN = e.sNaN + (size_t)s * e.elbTmax * Ns;
  // Yb and Z = Yb - Yhatactual;  Yhatactual(:,t) = (Xactual(elbT0+t, lagmask) * PAIactual)' (:400-403)
  for (int q = tz * N + tid; q < tb * N; q += kElbPrepThreads) {
    const int t = q / N, i = q % N;
    double yh = 0.0;
    if (e.yhat) {  // gibbsdrawShadowrates' YHAT0 argument (ccmm_gibbs_shadowrates)
      yh = e.yhat[((size_t)c * e.elbTmax + t) * N + i];
    } else {
      // hybrid: Yhatactual = Xffrlags(elbT0+t, :) * PAIactual (mcmcVARhybridGibbs.m:429-431)
      for (int k = e.kshadow; k < e.K; ++k) yh = fma(Xa[(size_t)k * TP + T0 + t], PAI[(size_t)i * KP + k], yh);
      // block hybrid: Yhatactual from the actual-rate block's shadow-rate lags (:400-403)
      if (e.actual[i])
        for (int l = 0; l < p; ++l)
          for (int si = 0; si < Ns; ++si) {
            const int k = 1 + l * N + e.ndxS[si];
            yh = fma(Xa[(size_t)k * TP + T0 + t], PAI[(size_t)i * KP + k], yh);
          }
    }
    double yb = Yc[(size_t)i * TP + T0 + t];
    for (int si = 0; si < Ns; ++si)
      if (e.ndxS[si] == i && sN[t * Ns + si]) yb = 0.0;
    Yt[q] = yb;
    Z[q] = yb - yh;
    if (zy_lds && t >= ta) {
      Ytg[q] = yb;
      Zg[q] = yb - yh;
    }
  }
  // Gibbs start values: the chain's current shadow rates (gibbsdrawShadowrates.m:171)
  double* Sc = e.Scur + (size_t)c * e.elbTmax * Ns;
  if (lead)
    for (int q = tid; q < T * Ns; q += kElbPrepThreads) Sc[q] = Yc[(size_t)e.ndxS[q % Ns] * TP + T0 + q / Ns];
  __syncthreads();
  // ε_τ = Z_τ - Σ_{l<=τ} Φ_l Z_{τ-l} - [τ = 0: w_{-1};  τ >= 1: c + Σ_{l>τ} Φ_l w_{τ-1-l}]
  for (int q = ta * N + tid; q < tb * N; q += kElbPrepThreads) {
    const int t = q / N, i = q % N;
    const double* ph = (phi_lds & 1) ? sPhi + i * ldp : Phi + (size_t)i * Np;
    double v = Z[q];
    for (int l = 1; l <= p && t - l >= 0; ++l) {
      const double* zl = Z + (size_t)(t - l) * N;
      for (int r = 0; r < N; ++r) v = fma(-ph[(l - 1) * N + r], zl[r], v);
    }
    if (t == 0) {
      v -= X0[1 + i];
    } else {
      double w = PAI[(size_t)i * KP] * X0[0];
      for (int l = t + 1; l <= p; ++l) {
        const double* wl = X0 + 1 + (l - t) * N;
        for (int r = 0; r < N; ++r) w = fma(ph[(l - 1) * N + r], wl[r], w);
      }
      v -= w;
    }
    Et[q] = v;
    if (e.ps || e.b3) {
      // PS model (mcmcVARshadowrateBlockHybrid.m:423-426): ε_τ = Yb_τ - c - yhat_τ
      //   - Σ_{l<=τ} Φ_l Yb_{τ-l} - Σ_{l>τ} Φ_l w_{τ-l}   (w_{-1-i} = lag block i of elb.X0)
      double u = Z[q] - PAI[(size_t)i * KP] * X0[0];  // Z = Yb - yhat
      for (int l = 1; l <= p; ++l) {
        if (t - l >= 0) {
          const double* yl = Yt + (size_t)(t - l) * N;
          for (int r = 0; r < N; ++r) u = fma(-ph[(l - 1) * N + r], yl[r], u);
        } else {
          const double* wl = X0 + 1 + (l - t - 1) * N;
          for (int r = 0; r < N; ++r) u = fma(-ph[(l - 1) * N + r], wl[r], u);
        }
      }
      if (e.ps) e.EtPS[(size_t)c * e.elbTmax * N + q] = u;
      if (e.b3) Et[q] = u;  // gibbsdrawShadowratesB3.m:178-185: Yhat = C A STATElag, no Y0 path
    }
  }
}

// ---------------------------------------------------------------- conditionals
// One wave per (censored month, chain).  Lanes own elements lane, lane + 64 of N-vectors;
// neighbour columns are spread over lanes; Ns x Ns algebra runs redundantly.
__device__ inline void elb_small_inverse(const double* M, double* Minv, int n) {
  double W[kElbNsMax * kElbNsMax];
  for (int q = 0; q < n * n; ++q) {
    W[q] = M[q];
    Minv[q] = 0.0;
  }
  for (int x = 0; x < n; ++x) Minv[x * n + x] = 1.0;
  for (int col = 0; col < n; ++col) {
    const double ip = 1.0 / W[col * n + col];
    for (int y = 0; y < n; ++y) {
      W[col * n + y] *= ip;
      Minv[col * n + y] *= ip;
    }
    for (int x = 0; x < n; ++x) {
      if (x == col) continue;
      const double f = W[x * n + col];
      for (int y = 0; y < n; ++y) {
        W[x * n + y] -= f * W[col * n + y];
        Minv[x * n + y] -= f * Minv[col * n + y];
      }
    }
  }
}

template <int NS>  // = e.Ns: compile-time, so the per-shadow-rate arrays below stay in registers
__global__ __launch_bounds__(256) void k_elb_cond(Dims d, ElbDev e, ChainState cs, int a_lds, int kb) {
  extern __shared__ double sm[];
  __shared__ double red[4 * kElbNsMax];  // per-wave partial sums (blockDim.x = 64 or 256)
  const int c = blockIdx.y;
  const int s = cs.slot[c];
  const int ci = blockIdx.x;
  if (ci >= e.ncens[s]) return;
  const int N = d.N, p = e.p, Np = N * p;
  constexpr int Ns = NS;
  const int T = e.elbT[s], T0 = e.elbT0[s];
  const int t = e.cens[(size_t)s * e.elbTmax + ci];
  // two waves for N <= 64; four for larger N (the N x p x Ns staging alone then fills one CU's LDS)
  const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, wv = tid >> 6, nwv = nth >> 6;
  const int ncol = 2 * p * Ns;
  const double* Phi = e.Phi + (size_t)c * N * Np;
  const double* Yt = e.Yt + (size_t)c * e.elbTmax * N;
  const double* Et = e.Et + (size_t)c * e.elbTmax * N;
  const double* Ag = cs.A + (size_t)c * N * N;  // column-major A(i,j), unit lower
  const int kmax = min(p, T - 1 - t);
  double* Q = sm;                              // (p+1) x Ns x N
  double* gS = Q + (p + 1) * Ns * N;           // (1 + ncol) x Ns
  double* Pm = gS + (1 + ncol) * Ns;           // Ns x Ns
  double* Om = Pm + Ns * Ns;                   // Ns x Ns
  double* Wl = Om + Ns * Ns;                   // kb x N x Ns: W_k = diag(1/SVol^2) (A or A Φ_k)[:, S]
  double* PS = Wl + kb * N * Ns;               // N x p x Ns: Φ's shadow-rate columns
                                               //   PS[(j p + l) Ns + b] = Φ_{l+1}(j, S_b)
  int S[kElbNsMax];
  for (int a = 0; a < kElbNsMax; ++a) S[a] = a < Ns ? e.ndxS[a] : 0;
  // every Φ read below is a shadow-rate column: stage those N p Ns values once per wave;
  // A too when it fits (a_lds: N <= 64), so the dependent sums below read LDS, not L1/L2
  for (int q = tid; q < N * p * Ns; q += nth) {
    const int b = q % Ns, jl = q / Ns, l = jl % p, jj = jl / p;
    PS[q] = Phi[(size_t)jj * Np + l * N + e.ndxS[b]];
  }
  double* Al = PS + N * p * Ns;
  if (a_lds && !e.Amon)
    for (int q = tid; q < N * N; q += nth) Al[q] = Ag[q];
  __syncthreads();
  const double* A = a_lds ? Al : Ag;
  // ---- Q_0 = Λ_t[S, :], Q_k = B_k' Λ_{t+k};  Λ = A' diag(1/SVol^2) A (B3: A of month t + k).
  //      kb lags at a time (all kmax + 1 when the LDS holds their W): one pass over (k, i) for the
  //      W_k, one over (k, a, j) for the Q_k, two barriers per batch instead of two per lag (the
  //      per-lag passes kept 20-60 of the workgroup's threads busy between barriers).  Every
  //      entry's sum is the per-lag form's, in the same order.
  auto A_of = [&](int k) -> const double* {
    return e.Amon ? e.Amon + ((size_t)c * e.elbTmax + t + k) * N * N : A;
  };
  for (int k0 = 0; k0 <= kmax; k0 += kb) {
    const int k1 = min(kmax + 1, k0 + kb);
    for (int q = tid; q < (k1 - k0) * N; q += nth) {
      const int kl = q / N, i = q - kl * N, k = k0 + kl;
      const double* Ak = A_of(k);
      double w[kElbNsMax] = {0.0, 0.0, 0.0, 0.0};
      const double sv = cs.sqrtht[((size_t)c * N + i) * d.TP + T0 + t + k];
      const double iv = 1.0 / (sv * sv);
      for (int a = 0; a < Ns; ++a) {
        double v = 0.0;
        if (k == 0) {
          v = Ak[i + S[a] * N];
        } else {
          const int jend = e.Afull ? N - 1 : i;
          for (int j = 0; j <= jend; ++j) v = fma(Ak[i + j * N], PS[(j * p + k - 1) * Ns + a], v);
        }
        w[a] = v * iv;
      }
      for (int a = 0; a < Ns; ++a) Wl[((size_t)kl * N + i) * Ns + a] = w[a];
    }
    __syncthreads();
    // Q_k[a][j] = Σ_{i >= j} W_k[i][a] A(i,j)   (Σ over every i when A is full)
    for (int q = tid; q < (k1 - k0) * Ns * N; q += nth) {
      const int kl = q / (Ns * N), r = q - kl * Ns * N, a = r / N, j = r - a * N, k = k0 + kl;
      const double* Ak = A_of(k);
      double v = 0.0;
      for (int i = e.Afull ? 0 : j; i < N; ++i) v = fma(Wl[((size_t)kl * N + i) * Ns + a], Ak[i + j * N], v);
      Q[((size_t)k * Ns + a) * N + j] = v;
    }
    __syncthreads();
  }
  // ---- P = Λ_t,SS + Σ_k Q_k B_k
  if (tid < Ns * Ns) {
    const int a = tid / Ns, b = tid % Ns;
    double v = Q[(size_t)a * N + S[b]];
    for (int k = 1; k <= kmax; ++k) {
      const double* Qk = Q + ((size_t)k * Ns + a) * N;
      for (int j = 0; j < N; ++j) v = fma(Qk[j], PS[(j * p + k - 1) * Ns + b], v);
    }
    Pm[tid] = v;
  }
  // ---- base g0 = -Q_0 ε'_t + Σ_k Q_k ε'_{t+k}, ε' = ε with S_t = 0:
  //      ε'_t = ε_t - E_S Yb_S,t,  ε'_{t+k} = ε_{t+k} + Φ_k[:,S] Yb_S,t
  {
    double g0[kElbNsMax] = {0.0, 0.0, 0.0, 0.0};
    for (int j = tid; j < N; j += nth) {
      bool isS = false;
      for (int a = 0; a < Ns; ++a) isS |= (S[a] == j);
      const double et = Et[(size_t)t * N + j];
      const double u0 = isS ? Yt[(size_t)t * N + j] - et : -et;  // -ε'_t
      for (int a = 0; a < Ns; ++a) g0[a] = fma(Q[(size_t)a * N + j], u0, g0[a]);
      for (int k = 1; k <= kmax; ++k) {
        double r = Et[(size_t)(t + k) * N + j];
        for (int b = 0; b < Ns; ++b)
          r = fma(PS[(j * p + k - 1) * Ns + b], Yt[(size_t)t * N + S[b]], r);
        for (int a = 0; a < Ns; ++a) g0[a] = fma(Q[((size_t)k * Ns + a) * N + j], r, g0[a]);
      }
    }
    for (int a = 0; a < Ns; ++a) {
      const double tot = wave_sum_dpp(g0[a]);
      if (lane == 0) red[wv * kElbNsMax + a] = tot;  // summed over the waves after the barrier below
    }
  }
  // ---- unit responses, one neighbour column per lane
  //   past  (s', t-kp): Q_0 Φ_kp[:,s'] - Σ_{k + kp <= p} Q_k Φ_{k+kp}[:,s']
  //   future(s', t+kp): Q_kp[:,s']     - Σ_{k = kp+1..kmax} Q_k Φ_{k-kp}[:,s']
  //   (one (column, a) pair per thread)
  for (int w = tid; w < ncol * Ns; w += nth) {
    const int col = w / Ns, a = w - col * Ns;
    const int kk = col / Ns, sp = col % Ns;
    const int q = S[sp];
    double v = 0.0;
    if (kk < p) {
      const int kp = kk + 1;
      if (t - kp >= 0) {
        for (int j = 0; j < N; ++j) v = fma(Q[(size_t)a * N + j], PS[(j * p + kp - 1) * Ns + sp], v);
        for (int k = 1; k <= kmax && k + kp <= p; ++k) {
          const double* Qk = Q + ((size_t)k * Ns + a) * N;
          for (int j = 0; j < N; ++j) v = fma(-Qk[j], PS[(j * p + k + kp - 1) * Ns + sp], v);
        }
      }
    } else {
      const int kp = kk - p + 1;
      if (kp <= kmax) {
        v = Q[((size_t)kp * Ns + a) * N + q];
        for (int k = kp + 1; k <= kmax; ++k) {
          const double* Qk = Q + ((size_t)k * Ns + a) * N;
          for (int j = 0; j < N; ++j) v = fma(-Qk[j], PS[(j * p + k - kp - 1) * Ns + sp], v);
        }
      }
    }
    gS[(size_t)(1 + col) * Ns + a] = v;
  }
  __syncthreads();
  if (tid < Ns) {
    double tot = red[tid];
    for (int x = 1; x < nwv; ++x) tot += red[x * kElbNsMax + tid];
    gS[tid] = tot;
  }
  __syncthreads();
  // ---- Ω = P^-1, a_t = Ω g0, betas (gibbsdrawShadowrates.m:130-145)
  double* rec = e.cond + ((size_t)c * e.elbTmax + ci) * e.condStride;
  double* beta = rec + Ns;
  double* so = beta + Ns * (Ns - 1);
  double* iso = so + Ns;
  double* Orec = iso + Ns;
  double* G = Orec + Ns * Ns;
  if (tid == 0) {
    double Pl[kElbNsMax * kElbNsMax], Oi[kElbNsMax * kElbNsMax];
    for (int q = 0; q < Ns * Ns; ++q) Pl[q] = Pm[q];
    elb_small_inverse(Pl, Oi, Ns);
    for (int q = 0; q < Ns * Ns; ++q) {
      Om[q] = Oi[q];
      Orec[q] = Oi[q];
    }
    for (int a = 0; a < Ns; ++a) {
      double v = 0.0;
      for (int b = 0; b < Ns; ++b) v = fma(Oi[a * Ns + b], gS[b], v);
      rec[a] = v;
    }
    // beta1(s,:) = Ω(s,o) Ω(o,o)^-1, sqrtOmega1(s) = sqrt(Ω(s,s) - beta1 Ω(o,s))
    for (int a = 0; a < Ns; ++a) {
      if (Ns == 1) {
        so[0] = sqrt(Oi[0]);
        break;
      }
      int oi[kElbNsMax];
      int no = 0;
      for (int b = 0; b < Ns; ++b)
        if (b != a) oi[no++] = b;
      double M[kElbNsMax * kElbNsMax], Mi[kElbNsMax * kElbNsMax];
      for (int x = 0; x < no; ++x)
        for (int y = 0; y < no; ++y) M[x * no + y] = Oi[oi[x] * Ns + oi[y]];
      elb_small_inverse(M, Mi, no);
      double var = Oi[a * Ns + a];
      for (int y = 0; y < no; ++y) {
        double b = 0.0;
        for (int x = 0; x < no; ++x) b = fma(Oi[a * Ns + oi[x]], Mi[x * no + y], b);
        beta[a * (Ns - 1) + y] = b;
        var -= b * Oi[oi[y] * Ns + a];
      }
      so[a] = sqrt(var);
    }
    for (int a = 0; a < Ns; ++a) iso[a] = 1.0 / so[a];
  }
  __syncthreads();
  // G = Ω g(unit); zero for uncensored or out-of-window neighbours
  const uint8_t* sN = e.sNaN + (size_t)s * e.elbTmax * Ns;
  for (int col = tid; col < ncol; col += nth) {
    const int kk = col / Ns, sp = col % Ns;
    const int tn = (kk < p) ? t - (kk + 1) : t + (kk - p + 1);
    const bool live = tn >= 0 && tn < T && sN[(size_t)tn * Ns + sp];
    for (int a = 0; a < Ns; ++a) {
      double v = 0.0;
      if (live)
        for (int b = 0; b < Ns; ++b) v = fma(Om[a * Ns + b], gS[(size_t)(1 + col) * Ns + b], v);
      G[(size_t)col * Ns + a] = v;
    }
  }
  if (e.ps) {
    // PS precision record (ccmm_ps.hip): P, the PS model's linear term
    //   b_PS = -(Λ_t ε_t)_S + Σ_k B_k' Λ_{t+k} ε_{t+k}  (ε of the PS model, censored cells at 0),
    // and the past neighbours' unit responses
    double* ext = rec + elb_cond_ps_off(Ns, p);
    if (tid < Ns * Ns) ext[tid] = Pm[tid];
    const double* EP = e.EtPS + (size_t)c * e.elbTmax * N;
    double bp[kElbNsMax] = {0.0, 0.0, 0.0, 0.0};
    for (int j = tid; j < N; j += nth) {
      const double u0 = -EP[(size_t)t * N + j];
      for (int a = 0; a < Ns; ++a) bp[a] = fma(Q[(size_t)a * N + j], u0, bp[a]);
      for (int k = 1; k <= kmax; ++k) {
        const double r = EP[(size_t)(t + k) * N + j];
        for (int a = 0; a < Ns; ++a) bp[a] = fma(Q[((size_t)k * Ns + a) * N + j], r, bp[a]);
      }
    }
    __syncthreads();  // red is free again (read above before the last barrier)
    for (int a = 0; a < Ns; ++a) {
      const double tot = wave_sum_dpp(bp[a]);
      if (lane == 0) red[wv * kElbNsMax + a] = tot;
    }
    for (int q = tid; q < p * Ns * Ns; q += nth) ext[Ns * Ns + Ns + q] = gS[Ns + q];
    __syncthreads();
    if (tid < Ns) {
      double tot = red[tid];
      for (int x = 1; x < nwv; ++x) tot += red[x * kElbNsMax + tid];
      ext[Ns * Ns + tid] = tot;
    }
  }
}

// ---------------------------------------------------------------- truncated normal (device)
// drawTruncNormal.m: z = -sqrt(2) erfcinv(2 u Φbar(ub)), ub = (elb - mu)/sig
// Phi^{-1}(p) by Wichura's AS241 (PPND16, relative error ~1e-16): the truncated draw of
// drawTruncNormal.m:47-48, z = -sqrt(2) erfcinv(2 u PHIbar), is Phi^{-1}(u PHIbar).  Inline
// with wave-uniform branches (every lane draws the same cell); the library erfcinv inlined
// into k_elb_gibbs's month loop needs ~480 registers (one wave per SIMD).
// A double constant materialised in SGPRs at its use: the month loops of the Gibbs kernels would
// otherwise keep every AS241 coefficient live in VGPRs across the loop (two each), crowding the
// draw's working registers into scratch.  (The asm is empty: the value is unchanged.)
__device__ __forceinline__ double elb_k(double c) {
  asm volatile("" : "+s"(c));
  return c;
}

__device__ __forceinline__ double elb_ppnd16(double p) {
  // every multiply-add is an explicit fma and nothing else may contract, so the value does not
  // depend on the context it is inlined into (the Gibbs kernels precompute it for the pass's
  // uniforms, elb_trunc_normal_pz, and evaluate it on the draw path: both must agree bit for bit)
#pragma clang fp contract(off)
  const double q = p - 0.5;
  if (fabs(q) <= 0.425) {
    const double r = fma(-q, q, 0.180625);
    double num = elb_k(2509.0809287301226727);
    num = fma(num, r, elb_k(33430.575583588128105));
    num = fma(num, r, elb_k(67265.770927008700853));
    num = fma(num, r, elb_k(45921.953931549871457));
    num = fma(num, r, elb_k(13731.693765509461125));
    num = fma(num, r, elb_k(1971.5909503065514427));
    num = fma(num, r, elb_k(133.14166789178437745));
    num = fma(num, r, elb_k(3.387132872796366608));
    double den = elb_k(5226.495278852545925);
    den = fma(den, r, elb_k(28729.085735721942674));
    den = fma(den, r, elb_k(39307.89580009271061));
    den = fma(den, r, elb_k(21213.794301586595867));
    den = fma(den, r, elb_k(5394.1960214247511077));
    den = fma(den, r, elb_k(687.1870074920579083));
    den = fma(den, r, elb_k(42.313330701600911252));
    den = fma(den, r, 1.0);
    return q * num / den;
  }
  double r = (q < 0.0) ? p : 1.0 - p;
  r = sqrt(-log(r));
  double num, den;
  if (r <= 5.0) {
    r -= 1.6;
    num = elb_k(7.7454501427834140764e-4);
    num = fma(num, r, elb_k(0.0227238449892691845833));
    num = fma(num, r, elb_k(0.24178072517745061177));
    num = fma(num, r, elb_k(1.27045825245236838258));
    num = fma(num, r, elb_k(3.64784832476320460504));
    num = fma(num, r, elb_k(5.7694972214606914055));
    num = fma(num, r, elb_k(4.6303378461565452959));
    num = fma(num, r, elb_k(1.42343711074968357734));
    den = elb_k(1.05075007164441684324e-9);
    den = fma(den, r, elb_k(5.475938084995344946e-4));
    den = fma(den, r, elb_k(0.0151986665636164571966));
    den = fma(den, r, elb_k(0.14810397642748007459));
    den = fma(den, r, elb_k(0.68976733498510000455));
    den = fma(den, r, elb_k(1.6763848301838038494));
    den = fma(den, r, elb_k(2.05319162663775882187));
    den = fma(den, r, 1.0);
  } else {
    r -= 5.0;
    num = elb_k(2.01033439929228813265e-7);
    num = fma(num, r, elb_k(2.71155556874348757815e-5));
    num = fma(num, r, elb_k(0.0012426609473880784386));
    num = fma(num, r, elb_k(0.026532189526576123093));
    num = fma(num, r, elb_k(0.29656057182850489123));
    num = fma(num, r, elb_k(1.7848265399172913358));
    num = fma(num, r, elb_k(5.4637849111641143699));
    num = fma(num, r, elb_k(6.6579046435011037772));
    den = elb_k(2.04426310338993978564e-15);
    den = fma(den, r, elb_k(1.4215117583164458887e-7));
    den = fma(den, r, elb_k(1.8463183175100546818e-5));
    den = fma(den, r, elb_k(7.868691311456132591e-4));
    den = fma(den, r, elb_k(0.0148753612908506148525));
    den = fma(den, r, elb_k(0.13692988092273580531));
    den = fma(den, r, elb_k(0.59983220655588793769));
    den = fma(den, r, 1.0);
  }
  const double z = num / den;
  return (q < 0.0) ? -z : z;
}

__device__ __forceinline__ double elb_trunc_normal(double mu, double sig, double elb, double u, uint8_t& fl) {
#pragma clang fp contract(off)
  const double tol = 1e-10;
  const double eps = 2.220446049250313080847e-16;
  sig = fabs(sig);
  fl = 0;
  if (sig > tol) {  // drawTruncNormal.m branches: bit 0 sigma > tol (:31), bit 1 PHIbar > eps (:44)
    const double ub = (elb - mu) / sig;
    const double PHIbar = 0.5 * erfc(-0.70710678118654752440 * ub);
    fl = (PHIbar > eps) ? 3 : 1;
    const double z = (PHIbar > eps) ? elb_ppnd16(u * PHIbar) : ub;
    return fma(sig, z, mu);
  }
  return mu;
}

// The Gibbs kernels' draw: drawTruncNormal.m as elb_trunc_normal, with ub = (elb - mu) * isig from the
// record's 1 / sig (k_elb_cond) instead of the division (a product: ~80 fewer clocks of dependent latency
// per draw; ub may differ from the quotient in its last bit, the draws by rounding only).  Every Gibbs
// kernel evaluates this same function, so their draws stay bit-identical to each other; the drop-in
// drawTruncNormal (k_truncnorm, ccmm_draw_trunc_normal) keeps the quotient.
__device__ __forceinline__ double elb_gibbs_trunc_normal(double mu, double sig, double isig, double elb, double u,
                                                         uint8_t& fl) {
#pragma clang fp contract(off)
  const double tol = 1e-10;
  const double eps = 2.220446049250313080847e-16;
  fl = 0;
  if (fabs(sig) > tol) {
    const double ub = (elb - mu) * fabs(isig);
    const double PHIbar = 0.5 * erfc(-0.70710678118654752440 * ub);
    fl = (PHIbar > eps) ? 3 : 1;
    const double z = (PHIbar > eps) ? elb_ppnd16(u * PHIbar) : ub;
    return fma(fabs(sig), z, mu);
  }
  return mu;
}

// The same draw with zu = elb_ppnd16(u) computed beforehand (off the month-to-month path).  When
// ub = (elb - mu) / sig >= 9, erfc(-ub / sqrt 2) = 2 - erfc(ub / sqrt 2) with erfc(6.36) ~ 1e-19, below
// half an ulp of 2: PHIbar is exactly 1, u PHIbar = u, and the full evaluation returns mu + sig zu.  So
// the draw is bit-identical without erfc and AS241 on the path (two thirds of the floor vintage's draws,
// profiles/r06final_elb_ubhist.json).  A second-order path for 5 <= ub < 9 (a sixth of the draws: z moved
// from zu by the Taylor series of Phi^-1, the tail Q = Phi(-ub) from exp and a Mills-ratio polynomial)
// measured no faster at B = 1 and slower in the octet kernel (two exp per draw cost what erfc does): not
// kept (round 6).
constexpr double kElbFastUb = 9.0;
__device__ __forceinline__ double elb_trunc_normal_pz(double mu, double sig, double isig, double elb, double u,
                                                      double zu, uint8_t& fl) {
#pragma clang fp contract(off)
  const double as = fabs(sig);
  if (as > 1e-10 && (elb - mu) * fabs(isig) >= kElbFastUb) {
    fl = 3;
    return fma(as, zu, mu);
  }
  return elb_gibbs_trunc_normal(mu, sig, isig, elb, u, fl);
}

// timing-only ablation bits of ElbDev::mode (CCMM_ELB_MODE, read by the ablation build only; a
// default build compiles them out): 1 no draws (fmin), 2 fixed uniforms, 64 cycle attribution,
// 128 no record loads, 256 no predecessor wait, 512 no month sums
#ifdef CCMM_ABLATION
#define ELB_CLK(x) const unsigned long long x = (e.mode & 64) ? clock64() : 0ull
#define ELB_ABL(bit) ((e.mode & (bit)) != 0)
#else
#define ELB_CLK(x) const unsigned long long x = 0ull
#define ELB_ABL(bit) false
#endif

// ---------------------------------------------------------------- Gibbs passes (per chain)
// One wave per chain.  Each lane owns neighbour columns lane and lane + 64 of every
// month's record; the draws themselves run redundantly on all lanes (uniform control
// flow).  The serial month-to-month path touches only registers and LDS: the censored
// month list and its per-series censoring mask sit in LDS (Tm), and the next month's
// record is prefetched from global memory into the other half of a register ping-pong
// pair while the current month is drawn, so no global-load round trip (and no vmcnt(0)
// wait on the prefetch) lands between two months.
template <int NS>
__global__ __launch_bounds__(64) void k_elb_gibbs(Dims d, ElbDev e, ChainState cs, RngArgs ra) {
  extern __shared__ double sm[];
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int p = e.p;
  const int T = e.elbT[s], nc = e.ncens[s];
  if (nc == 0) return;
  if (e.psFlag && e.psFlag[c] > 0) return;  // a PS proposal was accepted (:453-454)
  const int lane = threadIdx.x;
  const Rng rng = ra.make(c);
  const int ncol = 2 * p * NS;
  const int head = elb_cond_head(NS);
  double* Sl = sm;                      // T x NS (t-major)
  double* Ul = sm + T * NS;             // this pass's uniforms, T x NS (t-major)
  double* Zl = sm + 2 * T * NS;         // their AS241 values elb_ppnd16(u) (elb_trunc_normal_pz)
  int* Tm = (int*)(sm + 3 * T * NS);    // censored months: t | (censored-series mask << 16)
  double* Sc = e.Scur + (size_t)c * e.elbTmax * NS;
  const uint8_t* sN = e.sNaN + (size_t)s * e.elbTmax * NS;
  const int* cl = e.cens + (size_t)s * e.elbTmax;
  const double* recs = e.cond + (size_t)c * e.elbTmax * e.condStride;
  for (int q = lane; q < T * NS; q += 64) Sl[q] = Sc[q];
  for (int q = lane; q < nc; q += 64) {
    const int t = cl[q];
    int m = 0;
    for (int a = 0; a < NS; ++a) m |= sN[t * NS + a] ? (1 << a) : 0;
    Tm[q] = t | (m << 16);
  }
  __syncthreads();
  // column geometry of this lane
  const int c0 = lane, c1 = lane + 64;
  const bool h0 = c0 < ncol, h1 = c1 < ncol;
  const int kk0 = c0 / NS, sp0 = c0 % NS, kk1 = c1 / NS, sp1 = c1 % NS;
  const int off0 = (kk0 < p) ? -(kk0 + 1) : (kk0 - p + 1);
  const int off1 = (kk1 < p) ? -(kk1 + 1) : (kk1 - p + 1);
  constexpr int kHd = NS + NS * (NS - 1) + 2 * NS;
  struct Rec {
    double hd[kHd], g0[NS], g1[NS];
  };
  // branch-free loads (clamped column, zeroed by select) so that the compiler's wait
  // counting sees the prefetch as straight-line code and waits only for the older month
  const int c0l = h0 ? c0 : 0, c1l = h1 ? c1 : 0;
  auto load_rec = [&](int ci, Rec& r_) {
    const double* r = recs + (size_t)ci * e.condStride;
    for (int q = 0; q < kHd; ++q) r_.hd[q] = r[q];
    for (int a = 0; a < NS; ++a) {
      r_.g0[a] = r[head + c0l * NS + a];
      r_.g1[a] = r[head + c1l * NS + a];
    }
  };
  // the pass's uniforms rand(Ns, elbT) (gibbsdrawShadowrates.m:173, page n) are data
  // independent: all lanes draw them up front (Philox pairs in parallel, or the CRN
  // page), so no generator sits on the serial month-to-month path
  auto uniforms = [&](int n) {
    if (rng.crn) {
      for (int q = lane; q < T * NS; q += 64) {
        const double uu = rng.uniform(CCMM_RNG_ELB, (uint32_t)(q + T * NS * n));
        Ul[q] = uu;
        Zl[q] = elb_ppnd16(uu);
      }
    } else {
      const uint32_t base = (uint32_t)(T * NS * n);  // even when T * NS is odd: handle by index
      for (int q = 2 * lane; q < T * NS + 1; q += 128) {
        // pair (base + q) >> 1 covers idx base+q and its partner; write both when in range
        const uint32_t i0 = base + (uint32_t)q - ((base + (uint32_t)q) & 1u);
        const u32x4 r = rng.raw(CCMM_RNG_ELB, i0 >> 1);
        const int q0 = (int)(i0 - base), q1 = q0 + 1;
        const double u0 = u01(r.x, r.y), u1 = u01(r.z, r.w);
        if (q0 >= 0 && q0 < T * NS) {
          Ul[q0] = u0;
          Zl[q0] = elb_ppnd16(u0);
        }
        if (q1 >= 0 && q1 < T * NS) {
          Ul[q1] = u1;
          Zl[q1] = elb_ppnd16(u1);
        }
      }
    }
    __syncthreads();
  };
  // month g of the flattened (pass, month) sequence: draw from rc, prefetch month g + 1
  // into rn; tm = Tm entry of month g, returns month g + 1's
  const int G = e.passes * nc;
  auto month = [&](int g, int tm, const Rec& rc, Rec& rn) -> int {
    const int n = g / nc, ci = g - n * nc;
    if (ci == 0) uniforms(n);
    const int cn = (ci + 1 < nc) ? ci + 1 : 0;  // wraps to month 0 of the next pass
    load_rec(cn, rn);  // past the last month: a harmless reload of month 0
    const int tmn = Tm[cn];
    const int t = tm & 0xffff, msk = tm >> 16;
    double u[NS], zu[NS];
    for (int a = 0; a < NS; ++a) {
      u[a] = ELB_ABL(2) ? 0.5 : Ul[t * NS + a];
      zu[a] = ELB_ABL(2) ? 0.0 : Zl[t * NS + a];
    }
    // Spost = a_t + Σ G S(neighbours)
    const int tn0 = t + off0, tn1 = t + off1;
    const double v0 = (h0 && tn0 >= 0 && tn0 < T) ? Sl[tn0 * NS + sp0] : 0.0;
    const double v1 = (h1 && tn1 >= 0 && tn1 < T) ? Sl[tn1 * NS + sp1] : 0.0;
    double sp[NS];
    for (int a = 0; a < NS; ++a) sp[a] = fma(h0 ? rc.g0[a] : 0.0, v0, (h1 ? rc.g1[a] : 0.0) * v1);
    wave_sum_dpp_n(sp);
    for (int a = 0; a < NS; ++a) sp[a] = rc.hd[a] + sp[a];
    // conditional draws in index order (gibbsdrawShadowrates.m:206-218)
    const double* beta = rc.hd + NS;
    const double* so = beta + NS * (NS - 1);
    double cur[NS];
    for (int a = 0; a < NS; ++a) cur[a] = Sl[t * NS + a];
    for (int a = 0; a < NS; ++a) {
      if (!((msk >> a) & 1)) continue;
      double mu = sp[a];
      int y = 0;
      for (int b = 0; b < NS; ++b) {
        if (b == a) continue;
        mu = fma(beta[a * (NS - 1) + y], cur[b] - sp[b], mu);
        ++y;
      }
      uint8_t fl = 0;
      cur[a] = ELB_ABL(1) ? fmin(mu, e.elb) : elb_trunc_normal_pz(mu, so[a], so[NS + a], e.elb, u[a], zu[a], fl);
      if (e.flags && lane == 0)  // drawTruncNormal.m branch taken (oracle.draw_trunc_normal flags)
        e.flags[(((size_t)c * e.passes + n) * e.elbTmax + t) * NS + a] = fl;
    }
    for (int a = 0; a < NS; ++a) Sl[t * NS + a] = cur[a];
    return tmn;
  };
  Rec ra_, rb_;
  load_rec(0, ra_);
  int tm = Tm[0];
  for (int g = 0; g < G; g += 2) {
    tm = month(g, tm, ra_, rb_);
    if (g + 1 < G) tm = month(g + 1, tm, rb_, ra_);
  }
  __syncthreads();
  for (int q = lane; q < T * NS; q += 64) Sc[q] = Sl[q];
}

// ---------------------------------------------------------------- Gibbs passes, wavefront
// The same draws as k_elb_gibbs, with W passes in flight at once (one wave each).  Pass n
// at censored month i reads the cells of months within p of t_i: the past ones as drawn
// by pass n, the future ones and its own as drawn by pass n - 1.  So pass n may draw i
// as soon as pass n - 1 has drawn every month up to reach(i) = max{j : t_j <= t_i + p}
// (and pass n + 1 may then only touch months whose whole neighbourhood pass n has left):
// the sequential order's reads are reproduced exactly, every cell sees the values it
// sees in k_elb_gibbs, and the draws, flags and uniforms are bit-identical.  Steps run in
// lock-step (one barrier each); progress counters are double-buffered by step parity so a
// wave reads only what its predecessor published before the last barrier.  Within a step
// the active months of different passes are more than p calendar months apart, so their
// reads and writes of Sl never overlap.
//
// ASYNC: no per-step barrier.  Each wave runs its passes month by month, waits (acquire) until its
// predecessor's published progress covers reach(i), draws, and publishes (release) its own; a wave
// with less work in a month (fewer censored series) no longer waits for the slowest wave of the step.
// The reads and writes are those of the lock-step form, so the draws stay bit-identical.
#ifdef CCMM_ABLATION
// timing-only attribution of the ASYNC month body (ablation build, CCMM_ELB_PROF=1): per wave,
// shader-clock cycles spent waiting for the predecessor, in the neighbour sums, in the draws and
// in the store/publish tail, plus the month count (read by ccmm_elb_prof)
__device__ unsigned long long g_elb_prof[8 * 6];
__device__ unsigned long long g_elb_ubhist[8];  // k_elb_gibbs_mp draws by ub = (elb - mu) / sig bin (mode 4096)
extern "C" int ccmm_elb_ubhist(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_elb_ubhist), sizeof(g_elb_ubhist)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_elb_ubhist), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
extern "C" int ccmm_elb_prof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_elb_prof), sizeof(g_elb_prof)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[8 * 6] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_elb_prof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
template <int NS, int W, bool ASYNC>
__global__ __launch_bounds__(64 * W) void k_elb_gibbs_wf(Dims d, ElbDev e, ChainState cs, RngArgs ra) {
  extern __shared__ double sm[];
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int p = e.p;
  const int T = e.elbT[s], nc = e.ncens[s];
  if (nc == 0) return;
  if (!e.spec && e.psFlag && e.psFlag[c] > 0) return;  // a PS proposal was accepted (:453-454)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Rng rng = ra.make(c);
  const int ncol = 2 * p * NS;
  const int head = elb_cond_head(NS);
  const int pg = e.elbTmax * NS;
  double* Sl = sm;                              // T x NS (t-major), shared by all passes
  double* Ul = sm + (size_t)pg * (1 + wave);    // this wave's pass uniforms, T x NS
  double* Zl = sm + (size_t)pg * (1 + W + wave);  // their elb_ppnd16(u) (elb_trunc_normal_pz)
  int* Tm = (int*)(sm + (size_t)pg * (1 + 2 * W));  // censored months: t | (mask << 16)
  int* reach = Tm + e.elbTmax;                  // reach(i)
  int* prog = reach + e.elbTmax;                // [2][W] next draw of each wave, n nc + i
  double* Sc = e.Scur + (size_t)c * e.elbTmax * NS;
  const uint8_t* sN = e.sNaN + (size_t)s * e.elbTmax * NS;
  const int* cl = e.cens + (size_t)s * e.elbTmax;
  const double* recs = e.cond + (size_t)c * e.elbTmax * e.condStride;
  const int P = e.passes;
  const int done_all = P * nc;
  for (int q = tid; q < T * NS; q += 64 * W) Sl[q] = Sc[q];
  for (int q = tid; q < nc; q += 64 * W) {
    const int t = cl[q];
    int m = 0;
    for (int a = 0; a < NS; ++a) m |= sN[t * NS + a] ? (1 << a) : 0;
    Tm[q] = t | (m << 16);
    int j = q;
    while (j + 1 < nc && cl[j + 1] <= t + p) ++j;
    reach[q] = j;
  }
  if (tid < 2 * W) {
    const int w = tid % W;
    prog[tid] = (w < P) ? w * nc : done_all;
  }
  __syncthreads();
  const int c0 = lane, c1 = lane + 64;
  const bool h0 = c0 < ncol, h1 = c1 < ncol;
  const int kk0 = c0 / NS, sp0 = c0 % NS, kk1 = c1 / NS, sp1 = c1 % NS;
  const int off0 = (kk0 < p) ? -(kk0 + 1) : (kk0 - p + 1);
  const int off1 = (kk1 < p) ? -(kk1 + 1) : (kk1 - p + 1);
  constexpr int kHd = NS + NS * (NS - 1) + 2 * NS;
  struct Rec {
    double hd[kHd], g0[NS], g1[NS];
  };
  const int c0l = h0 ? c0 : 0, c1l = h1 ? c1 : 0;
  auto load_rec = [&](int ci, Rec& r_) {
    const double* r = recs + (size_t)ci * e.condStride;
    for (int q = 0; q < kHd; ++q) r_.hd[q] = r[q];
    for (int a = 0; a < NS; ++a) {
      r_.g0[a] = r[head + c0l * NS + a];
      r_.g1[a] = r[head + c1l * NS + a];
    }
  };
  // pass n's uniforms rand(Ns, elbT) (gibbsdrawShadowrates.m:173, page n), drawn by this wave
  auto uniforms = [&](int n) {
    if (rng.crn) {
      for (int q = lane; q < T * NS; q += 64) {
        const double uu = rng.uniform(CCMM_RNG_ELB, (uint32_t)(q + T * NS * n));
        Ul[q] = uu;
        Zl[q] = elb_ppnd16(uu);
      }
    } else {
      const uint32_t base = (uint32_t)(T * NS * n);
      for (int q = 2 * lane; q < T * NS + 1; q += 128) {
        const uint32_t i0 = base + (uint32_t)q - ((base + (uint32_t)q) & 1u);
        const u32x4 r = rng.raw(CCMM_RNG_ELB, i0 >> 1);
        const int q0 = (int)(i0 - base), q1 = q0 + 1;
        const double u0 = u01(r.x, r.y), u1 = u01(r.z, r.w);
        if (q0 >= 0 && q0 < T * NS) {
          Ul[q0] = u0;
          Zl[q0] = elb_ppnd16(u0);
        }
        if (q1 >= 0 && q1 < T * NS) {
          Ul[q1] = u1;
          Zl[q1] = elb_ppnd16(u1);
        }
      }
    }
    wave_lds_sync();
  };
  int n = wave, i = 0;
  Rec rc, rn;
  load_rec(0, rc);
  int tm = Tm[0];
  if constexpr (ASYNC) {
    // one month of pass n (the same draw code as the lock-step body below); the censored-month
    // entries are fetched two months ahead, so no LDS round trip of them sits on the month's path
    const int pred = (wave + W - 1) % W;
    bool stuck = false;
    unsigned long long acc_w = 0, acc_s = 0, acc_d = 0, acc_t = 0, months = 0;
    int tmn = Tm[nc > 1 ? 1 : 0];
    bool aborted = false;  // spec mode: the PS branch accepted a proposal
    int dec = 0;           // spec mode: the decision loaded one month ago (checked one month later)
    for (; n < P && !stuck && !aborted; n += W) {
      uniforms(n);
      for (i = 0; i < nc; ++i) {
        ELB_CLK(t0);
        const int ni = (i + 1 < nc) ? i + 1 : 0;
        const int nni = (ni + 1 < nc) ? ni + 1 : 0;
        const int tmnn = Tm[nni];
        if (!ELB_ABL(128))
          load_rec(ni, rn);  // next month of this wave (month 0 of its next pass after the last)
        else
          rn = rc;  // (128: timing only, no record loads)
        if (e.spec && (i & 3) == 0) {  // the PS decision, loaded after the record (in-order completion) and
          if (dec == 1) {              // read four months later, so the poll never holds a month up
            aborted = true;
            break;
          }
          dec = elb_ps_decision(e, c);
        }
        if (n > 0 && !ELB_ABL(256)) {  // (256: timing only, no predecessor wait)
          const int need = (n - 1) * nc + reach[i] + 1;
          int it = 0;
          while (__hip_atomic_load(&prog[pred], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
            __builtin_amdgcn_s_sleep(1);
            if (++it > (1 << 24)) {
              stuck = true;
              break;
            }
          }
          if (stuck) break;
        }
        ELB_CLK(t1);
        const int t = __builtin_amdgcn_readfirstlane(tm) & 0xffff, msk = __builtin_amdgcn_readfirstlane(tm) >> 16;
        double u[NS], zu[NS];
        for (int a = 0; a < NS; ++a) {
          u[a] = ELB_ABL(2) ? 0.5 : Ul[t * NS + a];
          zu[a] = ELB_ABL(2) ? 0.0 : Zl[t * NS + a];
        }
        // the neighbour cells and the month's own cells, one LDS round trip
        const int tn0 = t + off0, tn1 = t + off1;
        const double v0 = (h0 && tn0 >= 0 && tn0 < T) ? Sl[tn0 * NS + sp0] : 0.0;
        const double v1 = (h1 && tn1 >= 0 && tn1 < T) ? Sl[tn1 * NS + sp1] : 0.0;
        double cur[NS];
        for (int a = 0; a < NS; ++a) cur[a] = Sl[t * NS + a];
        double sp[NS];
        for (int a = 0; a < NS; ++a) sp[a] = fma(h0 ? rc.g0[a] : 0.0, v0, (h1 ? rc.g1[a] : 0.0) * v1);
        if (!ELB_ABL(512)) wave_sum_dpp_n(sp);
        for (int a = 0; a < NS; ++a) sp[a] = rc.hd[a] + sp[a];
        const double* beta = rc.hd + NS;
        const double* so = beta + NS * (NS - 1);
        ELB_CLK(t2);
        for (int a = 0; a < NS; ++a) {
          if (!((msk >> a) & 1)) continue;
          double mu = sp[a];
          int y = 0;
          for (int b = 0; b < NS; ++b) {
            if (b == a) continue;
            mu = fma(beta[a * (NS - 1) + y], cur[b] - sp[b], mu);
            ++y;
          }
          uint8_t fl = 0;
          cur[a] = ELB_ABL(1) ? fmin(mu, e.elb) : elb_trunc_normal_pz(mu, so[a], so[NS + a], e.elb, u[a], zu[a], fl);
          if (e.flags && lane == 0)
            e.flags[(((size_t)c * e.passes + n) * e.elbTmax + t) * NS + a] = fl;
        }
        ELB_CLK(t3);
        for (int a = 0; a < NS; ++a) Sl[t * NS + a] = cur[a];
        rc = rn;
        tm = tmn;
        tmn = tmnn;
        if (lane == 0)
          __hip_atomic_store(&prog[wave], n * nc + i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef CCMM_ABLATION
        if (e.mode & 64) {
          ELB_CLK(t4);
          acc_w += t1 - t0;
          acc_s += t2 - t1;
          acc_d += t3 - t2;
          acc_t += t4 - t3;
          ++months;
        }
#endif
      }
    }
#ifdef CCMM_ABLATION
    if ((e.mode & 64) && lane == 0 && c == 0 && wave < 8) {
      atomicAdd(&g_elb_prof[wave * 6 + 0], acc_w);
      atomicAdd(&g_elb_prof[wave * 6 + 1], acc_s);
      atomicAdd(&g_elb_prof[wave * 6 + 2], acc_d);
      atomicAdd(&g_elb_prof[wave * 6 + 3], acc_t);
      atomicAdd(&g_elb_prof[wave * 6 + 4], months);
      atomicAdd(&g_elb_prof[wave * 6 + 5], 1ull);
    }
#endif
    if (lane == 0) __hip_atomic_store(&prog[wave], done_all, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (stuck && lane == 0) atomicOr(&cs.status[c], 32);
    __syncthreads();
    double* dst = e.spec ? e.ScurSpec + (size_t)c * e.elbTmax * NS : Sc;  // (spec: k_elb_spec_select picks)
    for (int q = tid; q < T * NS; q += 64 * W) dst[q] = Sl[q];
    return;
  }
  for (int step = 0;; ++step) {
    const int* prd = prog + ((step + 1) & 1) * W;  // published before the last barrier
    int* pwr = prog + (step & 1) * W;
    bool fin = true;
#pragma unroll
    for (int w = 0; w < W; ++w) fin &= prd[w] >= done_all;
    if (fin) break;
    bool can = n < P;
    if (can && n > 0) can = prd[(wave + W - 1) % W] >= (n - 1) * nc + reach[i] + 1;
    if (can) {
      if (i == 0) uniforms(n);
      int nn = n, ni = i + 1;
      if (ni == nc) {
        nn = n + W;
        ni = 0;
      }
      load_rec(ni, rn);  // this wave's next month (a harmless reload past its last pass)
      const int tmn = Tm[ni];
      const int t = tm & 0xffff, msk = tm >> 16;
      double u[NS], zu[NS];
      for (int a = 0; a < NS; ++a) {
        u[a] = ELB_ABL(2) ? 0.5 : Ul[t * NS + a];
        zu[a] = ELB_ABL(2) ? 0.0 : Zl[t * NS + a];
      }
      const int tn0 = t + off0, tn1 = t + off1;
      const double v0 = (h0 && tn0 >= 0 && tn0 < T) ? Sl[tn0 * NS + sp0] : 0.0;
      const double v1 = (h1 && tn1 >= 0 && tn1 < T) ? Sl[tn1 * NS + sp1] : 0.0;
      double sp[NS];
      for (int a = 0; a < NS; ++a) sp[a] = fma(h0 ? rc.g0[a] : 0.0, v0, (h1 ? rc.g1[a] : 0.0) * v1);
      wave_sum_dpp_n(sp);
    for (int a = 0; a < NS; ++a) sp[a] = rc.hd[a] + sp[a];
      const double* beta = rc.hd + NS;
      const double* so = beta + NS * (NS - 1);
      double cur[NS];
      for (int a = 0; a < NS; ++a) cur[a] = Sl[t * NS + a];
      for (int a = 0; a < NS; ++a) {
        if (!((msk >> a) & 1)) continue;
        double mu = sp[a];
        int y = 0;
        for (int b = 0; b < NS; ++b) {
          if (b == a) continue;
          mu = fma(beta[a * (NS - 1) + y], cur[b] - sp[b], mu);
          ++y;
        }
        uint8_t fl = 0;
        cur[a] = ELB_ABL(1) ? fmin(mu, e.elb) : elb_trunc_normal_pz(mu, so[a], so[NS + a], e.elb, u[a], zu[a], fl);
        if (e.flags && lane == 0)
          e.flags[(((size_t)c * e.passes + n) * e.elbTmax + t) * NS + a] = fl;
      }
      for (int a = 0; a < NS; ++a) Sl[t * NS + a] = cur[a];
      rc = rn;
      tm = tmn;
      n = nn;
      i = ni;
    }
    if (lane == 0) pwr[wave] = (n < P) ? n * nc + i : done_all;
    __syncthreads();
  }
  for (int q = tid; q < T * NS; q += 64 * W) Sc[q] = Sl[q];
}

// ---------------------------------------------------------------- Gibbs passes, wavefront over CUs
// k_elb_gibbs_wf's asynchronous wavefront with its W = WPC * PARTS passes in flight spread over PARTS
// workgroups (CUs) per chain, WPC drawing waves each: one drawing wave per SIMD instead of two, so a
// month's draw is no longer issue-bound on a shared SIMD (the one-chain-per-vintage floor of the OOS
// run, goVARshadowrateBlockHybrid.m:258-303, runs 8 waves on one CU otherwise).  Pass n runs on global
// wave n mod W (part = gw / WPC).  Every part keeps its own copy of the shadow rates in LDS.
//   within a part: the waves hand off through LDS progress words exactly as k_elb_gibbs_wf;
//   across parts: an exporter wave of part j (wave WPC + 1) follows the LDS progress of the part's last
//   drawing wave and publishes every cell it has drawn as a 16-byte granule {value, tag = epoch 2^16 +
//   pass + 1}, one write-through (sc1) store each (the data is the flag; no fence), up to eight months at
//   a time; an importer wave of part j + 1 (wave WPC) reads the granules of the censored months in order
//   with sc1 loads, up to eight months per round trip, copies them into its part's LDS copy and publishes
//   its progress in the predecessor's encoding, so wave 0 of part j + 1 waits on it as on a local
//   predecessor.  The drawing waves issue no global store: a write-through store's completion would
//   hold the next month's record loads behind it (vmcnt counts both in order).
// Why a copy can be refreshed late: in the one-copy kernel pass n overwrites month m only once every
// earlier pass is done with it, and pass n + 1 reads it only after pass n has drawn past reach(m); the
// import of pass n's value for m happens between those two events in the consumer part, so every read
// sees the value the sequential order gives it: draws, flags and states are bit-identical to
// k_elb_gibbs.  All PARTS workgroups of a chain must be resident together (the host checks occupancy);
// every spin is bounded (status bit 32, then the wave publishes "done" so its successors drain).
template <int NS, int WPC, int PARTS>
__global__ __launch_bounds__(64 * (WPC + 2)) void k_elb_gibbs_mp(Dims d, ElbDev e, ChainState cs, RngArgs ra,
                                                                 ElbXch xc) {
  constexpr int W = WPC * PARTS;
  extern __shared__ double sm[];
  const int c = blockIdx.x, part = blockIdx.y;
  const int s = cs.slot[c];
  const int p = e.p;
  const int T = e.elbT[s], nc = e.ncens[s];
  if (nc == 0) return;
  if (!e.spec && e.psFlag && e.psFlag[c] > 0) return;  // a PS proposal was accepted (:453-454)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // WPC: the importer, WPC + 1: the exporter
  const int gw = part * WPC + wave;
  const Rng rng = ra.make(c);
  const int ncol = 2 * p * NS;
  const int head = elb_cond_head(NS);
  const int pg = e.elbTmax * NS;
  double* Sl = sm;                                            // T x NS (t-major): this part's copy
  double* Ul = sm + (size_t)pg * (1 + min(wave, WPC - 1));    // this wave's pass uniforms
  double* Zl = sm + (size_t)pg * (1 + WPC + min(wave, WPC - 1));
  int* Tm = (int*)(sm + (size_t)pg * (1 + 2 * WPC));          // censored months: t | (mask << 16)
  int* reach = Tm + e.elbTmax;
  int* prog = reach + e.elbTmax;                              // [WPC + 1]: drawing waves, importer
  double* Sc = e.Scur + (size_t)c * e.elbTmax * NS;
  const uint8_t* sN = e.sNaN + (size_t)s * e.elbTmax * NS;
  const int* cl = e.cens + (size_t)s * e.elbTmax;
  const double* recs = e.cond + (size_t)c * e.elbTmax * e.condStride;
  const int P = e.passes;
  const int done_all = P * nc;
  const unsigned long long tag0 = xc.epoch << 16;
  // granule buffers of this chain: the one this part publishes into, the one its importer reads
  const size_t gstride = (size_t)e.elbTmax * NS * 16;  // bytes per part
  char* gbase = (char*)(xc.gran) + (size_t)c * PARTS * gstride;
  const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(gbase, 0, (int)(PARTS * gstride), 0x00020000);
  const int gout = part * (int)gstride, gin = ((part + PARTS - 1) % PARTS) * (int)gstride;
  for (int q = tid; q < T * NS; q += 64 * (WPC + 2)) Sl[q] = Sc[q];
  for (int q = tid; q < nc; q += 64 * (WPC + 2)) {
    const int t = cl[q];
    int m = 0;
    for (int a = 0; a < NS; ++a) m |= sN[t * NS + a] ? (1 << a) : 0;
    Tm[q] = t | (m << 16);
    int j = q;
    while (j + 1 < nc && cl[j + 1] <= t + p) ++j;
    reach[q] = j;
  }
  if (tid <= WPC) {
    const int g = part * WPC + tid;  // the importer's predecessor pass is gw - 1 of the part before
    prog[tid] = tid < WPC ? ((g < P) ? g * nc : done_all) : ((part * WPC - 1 + W) % W) * nc;
  }
  __syncthreads();
  if (wave == WPC + 1) {
    // ---- exporter: the cells of every month the last drawing wave (global wave gw_last) has drawn in a
    //      pass whose successor runs on the next part, in month order, up to 8 months per batch
    constexpr int KM = 8;
    const int k = lane / NS, a = lane - (lane / NS) * NS;
    const bool act = lane < KM * NS;
    bool stuck = false;
    for (int ne = part * WPC + WPC - 1; ne + 1 < P && !stuck; ne += W) {
      const unsigned long long tag = tag0 + (unsigned long long)(ne + 1);
      int it = 0;
      for (int m = 0; m < nc;) {
        const int pl = __hip_atomic_load(&prog[WPC - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int avail = pl >= done_all ? nc : min(nc, max(0, pl - ne * nc));
        const int cnt = min(avail - m, KM);
        if (cnt <= 0) {
          if (e.spec && (it & 63) == 63 && elb_ps_decision(e, c) == 1) {  // the PS branch accepted
            ne = P;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if (++it > (1 << 24)) {
            stuck = true;
            break;
          }
          continue;
        }
        it = 0;
        if (act && k < cnt) {
          const int t = Tm[m + k] & 0xffff;
          const unsigned long long vb = (unsigned long long)__double_as_longlong(Sl[t * NS + a]);
          const __attribute__((ext_vector_type(4))) unsigned g = {(unsigned)vb, (unsigned)(vb >> 32), (unsigned)tag,
                                                                   (unsigned)(tag >> 32)};
          __builtin_amdgcn_raw_buffer_store_b128(g, grs, gout + (t * NS + a) * 16, 0, 16);  // sc1
        }
        m += cnt;
      }
    }
    if (stuck && lane == 0) atomicOr(&cs.status[c], CCMM_STATUS_HANDOFF);
    __syncthreads();
    return;
  }
  if (wave == WPC) {
    // ---- importer: passes n' = gw - 1 (mod W) of the previous part's last wave, whose successor pass
    //      n' + 1 runs here; month by month in order, up to 8 months per round trip
    constexpr int KM = 8;
    const int k = lane / NS, a = lane - (lane / NS) * NS;
    const bool act = lane < KM * NS;
    bool stuck = false;
    for (int np = (part * WPC - 1 + W) % W; np + 1 < P && !stuck; np += W) {
      const unsigned long long want = tag0 + (unsigned long long)(np + 1);
      int it = 0;
      for (int m = 0; m < nc;) {
        const int mk = m + k;
        bool ok = true;
        double v = 0.0;
        int t = 0;
        if (act && mk < nc) {
          t = Tm[mk] & 0xffff;
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(grs, gin + (t * NS + a) * 16, 0, 16);  // sc1
          v = __hiloint2double((int)x[1], (int)x[0]);
          ok = ((unsigned long long)x[3] << 32 | x[2]) == want;
        }
        // months m .. m + cnt - 1 are complete (every cell tagged for pass np)
        const unsigned long long bad = __ballot(!ok);
        int cnt = KM;
#pragma unroll
        for (int kk = 0; kk < KM; ++kk)
          if (cnt == KM && ((bad >> (kk * NS)) & ((1ull << NS) - 1))) cnt = kk;
        cnt = min(cnt, nc - m);
        if (cnt == 0) {
          if (e.spec && (it & 63) == 63 && elb_ps_decision(e, c) == 1) {  // the PS branch accepted
            np = P;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if (++it > (1 << 24)) {
            stuck = true;
            break;
          }
          continue;
        }
        it = 0;
        if (act && k < cnt) Sl[t * NS + a] = v;
        wave_lds_sync();
        m += cnt;
        if (lane == 0)
          __hip_atomic_store(&prog[WPC], np * nc + m, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    if (lane == 0) __hip_atomic_store(&prog[WPC], done_all, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (stuck && lane == 0) atomicOr(&cs.status[c], CCMM_STATUS_HANDOFF);
    __syncthreads();
    return;
  }
  const int c0 = lane, c1 = lane + 64;
  const bool h0 = c0 < ncol, h1 = c1 < ncol;
  const int kk0 = c0 / NS, sp0 = c0 % NS, kk1 = c1 / NS, sp1 = c1 % NS;
  const int off0 = (kk0 < p) ? -(kk0 + 1) : (kk0 - p + 1);
  const int off1 = (kk1 < p) ? -(kk1 + 1) : (kk1 - p + 1);
  constexpr int kHd = NS + NS * (NS - 1) + 2 * NS;
  struct Rec {
    double hd[kHd], g0[NS], g1[NS];
  };
  const int c0l = h0 ? c0 : 0, c1l = h1 ? c1 : 0;
  auto load_rec = [&](int ci, Rec& r_) {
    const double* r = recs + (size_t)ci * e.condStride;
    for (int q = 0; q < kHd; ++q) r_.hd[q] = r[q];
    for (int a = 0; a < NS; ++a) {
      r_.g0[a] = r[head + c0l * NS + a];
      r_.g1[a] = r[head + c1l * NS + a];
    }
  };
  auto uniforms = [&](int n) {  // pass n's rand(Ns, elbT) (gibbsdrawShadowrates.m:173, page n)
    if (rng.crn) {
      for (int q = lane; q < T * NS; q += 64) {
        const double uu = rng.uniform(CCMM_RNG_ELB, (uint32_t)(q + T * NS * n));
        Ul[q] = uu;
        Zl[q] = elb_ppnd16(uu);
      }
    } else {
      const uint32_t base = (uint32_t)(T * NS * n);
      for (int q = 2 * lane; q < T * NS + 1; q += 128) {
        const uint32_t i0 = base + (uint32_t)q - ((base + (uint32_t)q) & 1u);
        const u32x4 r = rng.raw(CCMM_RNG_ELB, i0 >> 1);
        const int q0 = (int)(i0 - base), q1 = q0 + 1;
        const double u0 = u01(r.x, r.y), u1 = u01(r.z, r.w);
        if (q0 >= 0 && q0 < T * NS) {
          Ul[q0] = u0;
          Zl[q0] = elb_ppnd16(u0);
        }
        if (q1 >= 0 && q1 < T * NS) {
          Ul[q1] = u1;
          Zl[q1] = elb_ppnd16(u1);
        }
      }
    }
    wave_lds_sync();
  };
  int* pprog = &prog[wave == 0 ? WPC : wave - 1];  // the predecessor: local wave or the importer
  int n = gw;
  Rec rc, rn;
  load_rec(0, rc);
  int tm = Tm[0];
  bool stuck = false;
  int tmn = Tm[nc > 1 ? 1 : 0];
  bool aborted = false;  // spec mode: the PS branch accepted a proposal
  int dec = 0;           // spec mode: the decision loaded one month ago
  for (; n < P && !stuck && !aborted; n += W) {
    uniforms(n);
    for (int i = 0; i < nc; ++i) {
      const int ni = (i + 1 < nc) ? i + 1 : 0;
      const int nni = (ni + 1 < nc) ? ni + 1 : 0;
      const int tmnn = Tm[nni];
      load_rec(ni, rn);  // next month of this wave (month 0 of its next pass after the last)
      if (e.spec && (i & 3) == 0) {  // the PS decision, loaded after the record, read four months later
        if (dec == 1) {
          aborted = true;
          break;
        }
        dec = elb_ps_decision(e, c);
      }
      if (n > 0 && !ELB_ABL(256)) {  // (256: timing only, no predecessor wait)
        const int need = (n - 1) * nc + reach[i] + 1;
        int it = 0;
        while (__hip_atomic_load(pprog, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
          __builtin_amdgcn_s_sleep(1);
          if (++it > (1 << 24)) {
            stuck = true;
            break;
          }
        }
        if (stuck) break;
      }
      const int t = __builtin_amdgcn_readfirstlane(tm) & 0xffff, msk = __builtin_amdgcn_readfirstlane(tm) >> 16;
      double u[NS], zu[NS];
      for (int a = 0; a < NS; ++a) {
        u[a] = Ul[t * NS + a];
        zu[a] = Zl[t * NS + a];
      }
      const int tn0 = t + off0, tn1 = t + off1;
      const double v0 = (h0 && tn0 >= 0 && tn0 < T) ? Sl[tn0 * NS + sp0] : 0.0;
      const double v1 = (h1 && tn1 >= 0 && tn1 < T) ? Sl[tn1 * NS + sp1] : 0.0;
      double cur[NS];
      for (int a = 0; a < NS; ++a) cur[a] = Sl[t * NS + a];
      double sp[NS];
      for (int a = 0; a < NS; ++a) sp[a] = fma(h0 ? rc.g0[a] : 0.0, v0, (h1 ? rc.g1[a] : 0.0) * v1);
      if (ELB_ABL(1024)) {  // timing only: a second, discarded copy of the month sums on the path
        double sq[NS];
        for (int a = 0; a < NS; ++a) sq[a] = sp[a] * 1.0000001;
        wave_sum_dpp_n(sq);
        for (int a = 0; a < NS; ++a) asm volatile("" ::"v"(sq[a]));
      }
      wave_sum_dpp_n(sp);
      for (int a = 0; a < NS; ++a) sp[a] = rc.hd[a] + sp[a];
      const double* beta = rc.hd + NS;
      const double* so = beta + NS * (NS - 1);
      for (int a = 0; a < NS; ++a) {
        if (!((msk >> a) & 1)) continue;
        double mu = sp[a];
        int y = 0;
        for (int b = 0; b < NS; ++b) {
          if (b == a) continue;
          mu = fma(beta[a * (NS - 1) + y], cur[b] - sp[b], mu);
          ++y;
        }
        uint8_t fl = 0;
#ifdef CCMM_ABLATION
        if (ELB_ABL(4096) && lane == 0) {  // ub histogram of the draws (ablation build, ccmm_elb_ubhist)
          const double ub = (e.elb - mu) * fabs(so[NS + a]);
          const int bin = ub >= 9.0 ? 0 : ub >= 7.0 ? 1 : ub >= 5.0 ? 2 : ub >= 3.0 ? 3 : ub >= 1.0 ? 4 : ub >= -1.0 ? 5 : 6;
          atomicAdd(&g_elb_ubhist[bin], 1ull);
        }
#endif
        cur[a] = elb_trunc_normal_pz(mu, so[a], so[NS + a], e.elb, u[a], zu[a], fl);
        if (ELB_ABL(2048)) {  // timing only: a second, discarded draw on the path
          uint8_t f2 = 0;
          const double d2 = elb_trunc_normal_pz(mu * 1.0000001, so[a], so[NS + a], e.elb, u[a], zu[a], f2);
          asm volatile("" ::"v"(d2));
        }
        if (e.flags && lane == 0) e.flags[(((size_t)c * e.passes + n) * e.elbTmax + t) * NS + a] = fl;
      }
      for (int a = 0; a < NS; ++a) Sl[t * NS + a] = cur[a];
      rc = rn;
      tm = tmn;
      tmn = tmnn;
      if (lane == 0)
        __hip_atomic_store(&prog[wave], n * nc + i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  if (lane == 0) __hip_atomic_store(&prog[wave], done_all, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (stuck && lane == 0) atomicOr(&cs.status[c], CCMM_STATUS_HANDOFF);
  __syncthreads();
  // the part that ran the last pass holds the final draw of every censored cell
  double* dst = e.spec ? e.ScurSpec + (size_t)c * e.elbTmax * NS : Sc;  // (spec: k_elb_spec_select picks)
  if (((P - 1) % W) / WPC == part)
    for (int q = tid; q < T * NS; q += 64 * WPC) dst[q] = Sl[q];
}

// ---------------------------------------------------------------- Gibbs passes, eight per wave
// The wavefront of k_elb_gibbs_wf inside ONE wave: eight lanes per pass in flight ("octets": lane
// 8 w + j, pass slot w = 0..7 runs passes w, w + 8, ...), so the passes synchronise by cross-lane
// shuffles instead of workgroup barriers and each truncated-normal draw is evaluated on 8 lanes
// instead of 64 (the wave kernels are issue-bound on that redundancy from B = 256 up).  Lane j of an
// octet owns the eight tree leaves 8 j .. 8 j + 7 of the month's 2 p Ns neighbour columns (leaf
// l = fma(g_l, v_l, g_{l+64} v_{l+64})): its group sum ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7))
// and the xor-1 / xor-2 / xor-4 sums over the octet give exactly the pairwise tree of wave_sum_dpp
// over 64 lanes, so the draws, flags and states are bit-identical to k_elb_gibbs / k_elb_gibbs_wf.
// Wavefront rule as there: pass n may draw month i once pass n - 1 has drawn every month up to
// reach(i) (the predecessor octet's progress, read by one shuffle per step; within a step the eight
// passes touch disjoint cells of Sl).
template <int NS>
__global__ __launch_bounds__(64) void k_elb_gibbs_oct(Dims d, ElbDev e, ChainState cs, RngArgs ra) {
  constexpr int W = 8;
  extern __shared__ double sm[];
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int p = e.p;
  const int T = e.elbT[s], nc = e.ncens[s];
  if (nc == 0) return;
  if (e.psFlag && e.psFlag[c] > 0) return;  // a PS proposal was accepted (:453-454)
  const int lane = threadIdx.x;
  const int w = lane >> 3, j = lane & 7;
  const Rng rng = ra.make(c);
  const int ncol = 2 * p * NS;
  const int head = elb_cond_head(NS);
  double* Sl = sm;                                 // T x NS (t-major)
  int* Tm = (int*)(sm + (size_t)e.elbTmax * NS);   // t | (mask << 16)
  int* reach = Tm + e.elbTmax;
  double* Sc = e.Scur + (size_t)c * e.elbTmax * NS;
  const uint8_t* sN = e.sNaN + (size_t)s * e.elbTmax * NS;
  const int* cl = e.cens + (size_t)s * e.elbTmax;
  const double* recs = e.cond + (size_t)c * e.elbTmax * e.condStride;
  const int P = e.passes;
  const int done_all = P * nc;
  for (int q = lane; q < T * NS; q += 64) Sl[q] = Sc[q];
  for (int q = lane; q < nc; q += 64) {
    const int t = cl[q];
    int m = 0;
    for (int a = 0; a < NS; ++a) m |= sN[t * NS + a] ? (1 << a) : 0;
    Tm[q] = t | (m << 16);
    int jj = q;
    while (jj + 1 < nc && cl[jj + 1] <= t + p) ++jj;
    reach[q] = jj;
  }
  __syncthreads();
  // this lane's leaves: l = 8 j + m; column l (and l + 64) -> neighbour month offset and rate
  int off0[8], sp0[8], off1[8], sp1[8];
  bool h0[8], h1[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int c0 = 8 * j + m, c1 = c0 + 64;
    h0[m] = c0 < ncol;
    h1[m] = c1 < ncol;
    const int kk0 = c0 / NS, kk1 = c1 / NS;
    sp0[m] = c0 % NS;
    sp1[m] = c1 % NS;
    off0[m] = (kk0 < p) ? -(kk0 + 1) : (kk0 - p + 1);
    off1[m] = (kk1 < p) ? -(kk1 + 1) : (kk1 - p + 1);
  }
  const int pred = 8 * ((w + W - 1) % W) + j;
  int n = w, i = 0;
  int prog = (n < P) ? n * nc : done_all;
  // the uniforms of the slot's next month (rand(Ns, elbT) page n, gibbsdrawShadowrates.m:173) are
  // drawn one step ahead, so the generator stays off the month-to-month dependence chain
  // (no precomputed AS241 here, unlike the wave kernels: the eight passes of a wave draw different
  // months, so the fast path of elb_trunc_normal_pz would only help when all eight take it at once, and
  // the per-step precompute costs more issue than it saves; the full evaluation gives the same bits)
  auto draw_u = [&](int nn, int ii, double (&uu)[NS]) {
    const int tt = Tm[ii] & 0xffff;
#pragma unroll
    for (int a = 0; a < NS; ++a)
      uu[a] = ELB_ABL(2) ? 0.5 : rng.uniform(CCMM_RNG_ELB, (uint32_t)(tt * NS + a + T * NS * nn));
  };
  double ucur[NS];
  if (n < P) draw_u(n, 0, ucur);
  // exit condition every wave reaches: the wavefront needs at most P nc + W (nc + 1) steps
  const int max_steps = P * nc + W * (nc + 1) + 8;
  for (int step = 0; step < max_steps; ++step) {
    const int pp = __shfl(prog, pred);
    if (__ballot(prog < done_all) == 0) break;
    bool can = n < P;
    if (can && n > 0) can = pp >= (n - 1) * nc + reach[i] + 1;
    if (can) {
      const int tm = Tm[i];
      const int t = tm & 0xffff, msk = tm >> 16;
      const double* r = recs + (size_t)i * e.condStride;
      int nn = n, ni = i + 1;
      if (ni == nc) {
        ni = 0;
        nn = n + W;
      }
      double unext[NS];
      if (nn < P) draw_u(nn, ni, unext);
      double hd[NS + NS * (NS - 1) + 2 * NS];
#pragma unroll
      for (int q = 0; q < NS + NS * (NS - 1) + 2 * NS; ++q) hd[q] = r[q];
      double x[8][NS];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int c0 = 8 * j + m, c1 = c0 + 64;
        const int tn0 = t + off0[m], tn1 = t + off1[m];
        const double v0 = (h0[m] && tn0 >= 0 && tn0 < T) ? Sl[tn0 * NS + sp0[m]] : 0.0;
        const double v1 = (h1[m] && tn1 >= 0 && tn1 < T) ? Sl[tn1 * NS + sp1[m]] : 0.0;
#pragma unroll
        for (int a = 0; a < NS; ++a) {
          const double g0 = h0[m] ? r[head + c0 * NS + a] : 0.0;
          const double g1 = h1[m] ? r[head + c1 * NS + a] : 0.0;
          x[m][a] = fma(g0, v0, g1 * v1);
        }
      }
      double sp[NS];
#pragma unroll
      for (int a = 0; a < NS; ++a) {
        double v = ((x[0][a] + x[1][a]) + (x[2][a] + x[3][a])) + ((x[4][a] + x[5][a]) + (x[6][a] + x[7][a]));
        v += dpp_d<0xB1>(v);   // xor 1
        v += dpp_d<0x4E>(v);   // xor 2
        v += dpp_d<0x141>(v);  // row_half_mirror: xor 4 within the octet
        sp[a] = hd[a] + v;
      }
      // conditional draws in index order (gibbsdrawShadowrates.m:206-218)
      const double* beta = hd + NS;
      const double* so = beta + NS * (NS - 1);
      double cur[NS];
#pragma unroll
      for (int a = 0; a < NS; ++a) cur[a] = Sl[t * NS + a];
#pragma unroll
      for (int a = 0; a < NS; ++a) {
        if (!((msk >> a) & 1)) continue;
        double mu = sp[a];
        int y = 0;
#pragma unroll
        for (int b = 0; b < NS; ++b) {
          if (b == a) continue;
          mu = fma(beta[a * (NS - 1) + y], cur[b] - sp[b], mu);
          ++y;
        }
        uint8_t fl = 0;
        cur[a] = ELB_ABL(1) ? fmin(mu, e.elb) : elb_gibbs_trunc_normal(mu, so[a], so[NS + a], e.elb, ucur[a], fl);
        if (e.flags && j == 0) e.flags[(((size_t)c * e.passes + n) * e.elbTmax + t) * NS + a] = fl;
      }
      if (j == 0) {
#pragma unroll
        for (int a = 0; a < NS; ++a) Sl[t * NS + a] = cur[a];
      }
      n = nn;
      i = ni;
#pragma unroll
      for (int a = 0; a < NS; ++a) ucur[a] = unext[a];
    }
    prog = (n < P) ? n * nc + i : done_all;
  }
  if (prog < done_all && lane == 0) atomicOr(&cs.status[c], 32);  // hand-off step cap reached (ccmm.h bit 32; never expected)
  __syncthreads();
  for (int q = lane; q < T * NS; q += 64) Sc[q] = Sl[q];
}

// ---------------------------------------------------------------- speculative step: the sweep's draw
// after the PS branch and the speculative Gibbs passes: the accepted proposal (already in Scur, k_ps_apply)
// or, where the PS branch rejected (or had no proposals), the Gibbs draw
__global__ void k_elb_spec_select(ElbDev e, const int* slot, int B) {
  const int c = blockIdx.x;
  if (c >= B) return;
  const int s = slot[c];
  if (e.ncens[s] == 0 || e.psFlag[c] > 0) return;
  const size_t n = (size_t)e.elbT[s] * e.Ns;
  for (size_t q = threadIdx.x; q < n; q += blockDim.x)
    e.Scur[(size_t)c * e.elbTmax * e.Ns + q] = e.ScurSpec[(size_t)c * e.elbTmax * e.Ns + q];
}

// ---------------------------------------------------------------- rebuild X, Y (per chain)
// shadowYdata(p+elbT0+1:end, ndxS) = shadowrate'; X(t, 1+(l-1)N+s) = Y(t-l, s) (:501-509)
__global__ void k_elb_rebuild(Dims d, ElbDev e, XSel xs, ChainState cs, int xslab0, double* dpool,
                              int ldd, int drows, double* dcpool, int dcld, long long dcslab) {
  const int c = blockIdx.y;
  const int s = cs.slot[c];
  const int N = d.N, TP = d.TP, Ns = e.Ns, p = e.p;
  const int T0 = e.elbT0[s], T = e.elbT[s];
  double* Y = const_cast<double*>(xs.ypool) + (size_t)xs.yidx[c] * N * TP;
  double* X = const_cast<double*>(xs.pool) + (size_t)(xslab0 + c) * d.KP * TP;
  const double* Sc = e.Scur + (size_t)c * e.elbTmax * Ns;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;  // (l in 0..p, si, t)
  if (q >= T * Ns * (p + 1)) return;
  const int l = q % (p + 1);
  const int r = q / (p + 1);
  const int si = r % Ns, t = r / Ns;
  const double v = Sc[t * Ns + si];
  const int var = e.ndxS[si];
  if (l == 0) {
    Y[(size_t)var * TP + T0 + t] = v;
    // lag-structured twin of the chain's X/Y (ccmm_lag.hip): D(p + row, var) = Y(row, var)
    if (dpool) dpool[((size_t)(xslab0 + c) * drows + p + T0 + t) * ldd + var] = v;
    // column-major twin of the large path (ccmm_big.h ColX): D(p + row, var), column var
    if (dcpool) dcpool[(size_t)(xslab0 + c) * dcslab + (size_t)var * dcld + p + T0 + t] = v;
  } else {
    const int row = T0 + t + l;  // X(row, lag l of var) = Y(row - l, var)
    if (row < T0 + T) X[(size_t)(1 + (l - 1) * N + var) * TP + row] = v;
  }
}

// ---------------------------------------------------------------- draw store
// shadowrate_all(thisMCMCdraw, :, :) = shadowrate (:542); NaN beyond the vintage's elbT
__global__ void k_elb_store(ElbDev e, ChainState cs, double* out, int cap, int m) {
  const int c = blockIdx.x;
  const int T = e.elbT[cs.slot[c]];
  const int per = e.Ns * e.elbTmax;
  const double* Sc = e.Scur + (size_t)c * per;
  double* o = out + ((size_t)c * cap + m) * per;
  for (int q = threadIdx.x; q < per; q += blockDim.x) o[q] = (q / e.Ns < T) ? Sc[q] : __builtin_nan("");
}

// ---------------------------------------------------------------- instantiations launched by ccmm_abi.hip
#define CCMM_ELB_INST(NS)                                                                              \
  template __global__ void k_elb_cond<NS>(Dims, ElbDev, ChainState, int, int);                         \
  template __global__ void k_elb_gibbs<NS>(Dims, ElbDev, ChainState, RngArgs);                         \
  template __global__ void k_elb_gibbs_wf<NS, 4, false>(Dims, ElbDev, ChainState, RngArgs);            \
  template __global__ void k_elb_gibbs_wf<NS, 4, true>(Dims, ElbDev, ChainState, RngArgs);             \
  template __global__ void k_elb_gibbs_wf<NS, 8, false>(Dims, ElbDev, ChainState, RngArgs);            \
  template __global__ void k_elb_gibbs_wf<NS, 8, true>(Dims, ElbDev, ChainState, RngArgs);             \
  template __global__ void k_elb_gibbs_mp<NS, 4, 2>(Dims, ElbDev, ChainState, RngArgs, ElbXch);        \
  template __global__ void k_elb_gibbs_mp<NS, 2, 4>(Dims, ElbDev, ChainState, RngArgs, ElbXch);        \
  template __global__ void k_elb_gibbs_oct<NS>(Dims, ElbDev, ChainState, RngArgs);
CCMM_ELB_INST(1)
CCMM_ELB_INST(2)
CCMM_ELB_INST(3)
CCMM_ELB_INST(4)
CCMM_ELB_INST(5)
#undef CCMM_ELB_INST

}  // namespace ccmm
