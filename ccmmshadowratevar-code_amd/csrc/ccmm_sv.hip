// Latency-optimised SV precision sampler (same algorithm as k_sv_sample in
// ccmm_kernels.hip, see the derivation there) for a compile-time N <= 32.
//
// One wave per chain.  Every N x N operand a lane needs repeatedly lives in its
// registers with compile-time indices, so every dependent step of the three
// sequential recursions (block TRSM, block Cholesky, forward/backward
// substitution) is an in-register FMA fed by v_readlane broadcasts:
//   lane c (< N) holds  column c of Q            qc[.]
//                       column c of M_t          m[.]    (M_t = Ld_{t-1}^{-1} Q)
//                       row c of Ld_t            s[.]    (row layout Cholesky)
// The previous factor Ld_{t-1} is read by broadcast from LDS in the TRSM; the
// Schur complement S_t = P_tt - M_t'M_t is formed by all 64 lanes (4 entries
// each) through LDS.  The backward pass re-reads Ld_t (row and column of each
// lane) from HBM one step ahead of use.
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

template <int NN>
__global__ __launch_bounds__(64) void k_sv_fast(Dims d, const int* __restrict__ Tslot,
                                                const double* __restrict__ V0inv,
                                                const double* __restrict__ V0invm, ChainState cs,
                                                RngArgs ra) {
  constexpr int NE = NN * (NN + 1) / 2;
  constexpr int EPL = (NE + 63) / 64;  // S entries per lane
  __shared__ double Lp[NN * NN];   // Ld_{t-1}, row-major
  __shared__ double rLp[NN];       // 1 / diag(Ld_{t-1})
  __shared__ double Ml[NN * NN];   // M_t row-major [r][c]
  __shared__ double Sl[NN * NN];   // S_t lower, row-major
  __shared__ double Ql[NN * NN];   // Q row-major
  __shared__ double wl[NN];        // w_{t-1}
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int T = Tslot[s];
  const int TP = d.TP;
  const int lane = threadIdx.x;
  const bool act = lane < NN;
  const int ln = act ? lane : 0;
  const Rng rng = ra.make(c);
  const double* sq = cs.sqrtPHI + (size_t)c * NN * NN;  // column-major lower
  const double* obs = cs.svobs + (size_t)c * NN * TP;
  const double* ir = cs.svir + (size_t)c * NN * TP;
  double* Ldg = cs.svLd + (size_t)c * (TP + 1) * NN * NN;  // [t][r*NN + k]
  double* Wg = cs.svw + (size_t)c * (TP + 1) * NN;
  int bad = 0;

  // ---------------------------------------------------------------- Q = (sqrtPHI sqrtPHI')^-1
  double li[NN];  // column `lane` of Li = sqrtPHI^-1 (lower)
#pragma unroll
  for (int r = 0; r < NN; ++r) {
    double v = (r == ln) ? 1.0 : 0.0;
#pragma unroll
    for (int q = 0; q < r; ++q) v = fma(-sq[r + q * NN], li[q], v);
    li[r] = (r >= ln) ? v / sq[r + r * NN] : 0.0;
  }
  if (act) {
#pragma unroll
    for (int r = 0; r < NN; ++r) Ml[r * NN + lane] = li[r];
  }
  __syncthreads();
  double qc[NN];  // Q[:, lane] = Q[lane, :]
#pragma unroll
  for (int r = 0; r < NN; ++r) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < NN; ++q) v = fma(Ml[q * NN + r], li[q], v);
    qc[r] = v;
    if (act) Ql[r * NN + lane] = v;
  }
  // S-entry assignment: entry e = lane + 64 j  ->  (ea, eb), ea >= eb
  int ea[EPL], eb[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int e = lane + 64 * j;
    int a = 0;
    while ((a + 1) * (a + 2) / 2 <= e) ++a;
    ea[j] = (e < NE) ? a : -1;
    eb[j] = e - a * (a + 1) / 2;
  }

  // ---------------------------------------------------------------- right-looking Cholesky, row layout
  double s_[NN];
  double rps[NN];  // 1/diag, uniform
  auto chol_rows = [&]() {
#pragma unroll
    for (int q = 0; q < NN; ++q) {
      double dq = readlane_d(s_[q], q);
      if (!(dq > 0.0)) {
        bad = 1;
        dq = 1.0;
      }
      const double piv = sqrt(dq);
      const double rp = 1.0 / piv;
      rps[q] = rp;
      s_[q] = (lane == q) ? piv : s_[q] * rp;
#pragma unroll
      for (int k = q + 1; k < NN; ++k) {
        const double lkq = readlane_d(s_[q], k);
        s_[k] = fma(-s_[q], lkq, s_[k]);
      }
    }
  };
  // forward substitution L y = b, lane i holds b_i and row i of L in s_
  auto fwd_rows = [&](double b) {
#pragma unroll
    for (int k = 0; k < NN; ++k) {
      const double yk = readlane_d(b, k) * rps[k];
      b = (lane == k) ? yk : ((lane > k) ? fma(-s_[k], yk, b) : b);
    }
    return b;
  };

  // ---------------------------------------------------------------- t = 0
  {
    const double* Vi = V0inv + (size_t)s * NN * NN;
#pragma unroll
    for (int k = 0; k < NN; ++k) s_[k] = Vi[ln + k * NN] + qc[k];
    chol_rows();
    double w = fwd_rows(act ? V0invm[(size_t)s * NN + lane] : 0.0);
    if (act) {
#pragma unroll
      for (int k = 0; k < NN; ++k) {
        const double v = (k <= lane) ? s_[k] : 0.0;
        Lp[lane * NN + k] = v;
        Ldg[lane * NN + k] = v;
      }
      Wg[lane] = w;
      wl[lane] = w;
    }
    __syncthreads();
  }
  // fix rLp (avoid runtime register index): recompute from LDS
  if (act) rLp[lane] = 1.0 / Lp[lane * NN + lane];
  __syncthreads();

  // ---------------------------------------------------------------- forward recursion
  for (int t = 1; t <= T; ++t) {
    const double irv = act ? ir[(size_t)lane * TP + t - 1] : 0.0;
    const double bob = act ? obs[(size_t)lane * TP + t - 1] * irv : 0.0;
    // (1) M = Lp^-1 Q, column `lane`
    double m[NN];
#pragma unroll
    for (int r = 0; r < NN; ++r) m[r] = qc[r];
#pragma unroll
    for (int r = 0; r < NN; ++r) {
      m[r] *= rLp[r];
#pragma unroll
      for (int i = r + 1; i < NN; ++i) m[i] = fma(-Lp[i * NN + r], m[r], m[i]);
    }
    // b_t + M' w_{t-1}
    double bt = bob;
#pragma unroll
    for (int q = 0; q < NN; ++q) bt = fma(m[q], wl[q], bt);
    if (act) {
#pragma unroll
      for (int r = 0; r < NN; ++r) Ml[r * NN + lane] = m[r];
    }
    if (act) wl[lane] = irv;  // reuse wl to pass diag(R_t^-1)
    __syncthreads();
    // (2) S = qf Q + diag(ir) - M'M, lower entries spread over 64 lanes
    const double qf = (t == T) ? 1.0 : 2.0;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      if (ea[j] >= 0) {
        const int a = ea[j], b = eb[j];
        double v = qf * Ql[a * NN + b] + ((a == b) ? wl[a] : 0.0);
#pragma unroll
        for (int q = 0; q < NN; ++q) v = fma(-Ml[q * NN + a], Ml[q * NN + b], v);
        Sl[a * NN + b] = v;
      }
    }
    __syncthreads();
    // (3) Cholesky of S (row layout)
#pragma unroll
    for (int k = 0; k < NN; ++k) s_[k] = (k <= ln) ? Sl[ln * NN + k] : 0.0;
    chol_rows();
    // (4) w_t = Ld^-1 (b_t + M' w_{t-1})
    const double w = fwd_rows(bt);
    double* Ldt = Ldg + (size_t)t * NN * NN;
    if (act) {
#pragma unroll
      for (int k = 0; k < NN; ++k) {
        const double v = (k <= lane) ? s_[k] : 0.0;
        Lp[lane * NN + k] = v;
        Ldt[lane * NN + k] = v;
      }
      Wg[(size_t)t * NN + lane] = w;
      wl[lane] = w;
    }
    __syncthreads();
    if (act) rLp[lane] = 1.0 / Lp[lane * NN + lane];
    __syncthreads();
  }

  // ---------------------------------------------------------------- backward pass
  double* hout = cs.h + (size_t)c * NN * TP;
  double* eta = cs.eta + (size_t)c * NN * TP;
  double* sqh = cs.sqrtht + (size_t)c * NN * TP;
  double x = 0.0;  // lane r: x_{t+1}(r)
  double lr[NN], lc[NN];
  {
    const double* Ldt = Ldg + (size_t)T * NN * NN;
#pragma unroll
    for (int k = 0; k < NN; ++k) {
      lr[k] = (k <= ln) ? Ldt[ln * NN + k] : 0.0;
      lc[k] = (k >= ln) ? Ldt[k * NN + ln] : 0.0;
    }
  }
  for (int t = T; t >= 0; --t) {
    const double* Ldt = Ldg + (size_t)t * NN * NN;
    // prefetch the next (earlier) factor
    double nlr[NN], nlc[NN];
    if (t > 0) {
      const double* Ln = Ldg + (size_t)(t - 1) * NN * NN;
#pragma unroll
      for (int k = 0; k < NN; ++k) {
        nlr[k] = (k <= ln) ? Ln[ln * NN + k] : 0.0;
        nlc[k] = (k >= ln) ? Ln[k * NN + ln] : 0.0;
      }
    }
    double rd[NN];
#pragma unroll
    for (int k = 0; k < NN; ++k) rd[k] = 1.0 / Ldt[k * NN + k];
    double rr = act ? Wg[(size_t)t * NN + lane] + rng.normal(CCMM_RNG_SVZ, (uint32_t)(lane + NN * t))
                    : 0.0;
    if (t < T) {
      // g = Q x_{t+1}; g <- Ld_t^-1 g
      double g = 0.0;
#pragma unroll
      for (int q = 0; q < NN; ++q) g = fma(qc[q], readlane_d(x, q), g);
#pragma unroll
      for (int k = 0; k < NN; ++k) {
        const double gk = readlane_d(g, k) * rd[k];
        g = (lane == k) ? gk : ((lane > k) ? fma(-lr[k], gk, g) : g);
      }
      rr += g;
    }
    // x_t = Ld_t^-T rr
#pragma unroll
    for (int k = NN - 1; k >= 0; --k) {
      const double xk = readlane_d(rr, k) * rd[k];
      rr = (lane == k) ? xk : ((lane < k) ? fma(-lc[k], xk, rr) : rr);
    }
    if (act) {
      if (t < T) eta[(size_t)lane * TP + t] = x - rr;  // shock of t+1
      if (t >= 1) {
        hout[(size_t)lane * TP + t - 1] = rr;
        sqh[(size_t)lane * TP + t - 1] = exp(rr * 0.5);
      }
    }
    x = rr;
    if (t > 0) {
#pragma unroll
      for (int k = 0; k < NN; ++k) {
        lr[k] = nlr[k];
        lc[k] = nlc[k];
      }
    }
  }
  for (int q = lane; q < NN * (TP - T); q += 64) {
    const int r = q / (TP - T), t = T + q % (TP - T);
    hout[(size_t)r * TP + t] = 0.0;
    eta[(size_t)r * TP + t] = 0.0;
    sqh[(size_t)r * TP + t] = 1.0;
  }
  if (bad && lane == 0) atomicOr(&cs.status[c], 8);
}

}  // namespace ccmm
