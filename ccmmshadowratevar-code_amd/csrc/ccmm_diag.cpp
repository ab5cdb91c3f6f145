// Convergence diagnostics of the OOS drivers: psrf (DiagnosticsShadowrate.m:34-128, the same
// function as Diagnostics.m:28) and shadowratePSRF (goVARshadowrateBlockHybrid.m:322-325,
// goVARhybrid.m:322-323, goVARshadowrate.m:332-333).  Host code: the inputs are the kept shadow-rate
// draws the batch loop already holds on the host, a few MB per vintage.
#include <cmath>
#include <limits>
#include <string>
#include <vector>

#include "../../include/ccmm.h"

namespace ccmm {
void set_last_error(const std::string& msg);  // ccmm_abi.hip
}

namespace {

const double kNaN = std::numeric_limits<double>::quiet_NaN();

// R of one variable from its M sequences of length n: seq(t, i) = the t-th draw of sequence i.
// Statement order of DiagnosticsShadowrate.m:106-128.
template <class Seq>
double psrf_one(int n, int M, Seq seq) {
  std::vector<double> mean_i(M);
  double W = 0.0;
  for (int i = 0; i < M; ++i) {  // :108-113
    double s = 0.0;
    for (int t = 0; t < n; ++t) s += seq(t, i);
    const double mu = s / n;
    mean_i[i] = mu;
    double ss = 0.0;
    for (int t = 0; t < n; ++t) {
      const double x = seq(t, i) - mu;
      ss += x * x;
    }
    W += ss;
  }
  W = W / (double(n - 1) * M);
  double m = 0.0;  // :117
  for (int i = 0; i < M; ++i) m += mean_i[i];
  m /= M;
  double Bpn = 0.0;  // :118-122
  for (int i = 0; i < M; ++i) {
    const double x = mean_i[i] - m;
    Bpn += x * x;
  }
  Bpn = Bpn / (M - 1);
  const double S = double(n - 1) / n * W + Bpn;  // :125
  const double R = double(M + 1) / M * S / W - double(n - 1) / M / n;
  return std::sqrt(R);  // :128
}

}  // namespace

extern "C" int ccmm_psrf(int n, int D, int M, const double* X, double* R) {
  if (n < 1 || D < 0 || M < 1 || (D > 0 && (!X || !R))) {
    ccmm::set_last_error("ccmm_psrf: n >= 1, D >= 0, M >= 1 and X, R required");
    return CCMM_ERR_ARG;
  }
  if (M == 1) {  // one chain: first and last thirds (DiagnosticsShadowrate.m:82-91)
    const int m3 = n / 3;
    if (m3 < 1) {
      ccmm::set_last_error("ccmm_psrf: Too few samples");  // :103-105
      return CCMM_ERR_ARG;
    }
    for (int d = 0; d < D; ++d) {
      const double* x = X + size_t(d) * n;
      R[d] = psrf_one(m3, 2, [&](int t, int i) { return x[i == 0 ? t : n - m3 + t]; });
    }
    return CCMM_OK;
  }
  if (n < 2) {
    ccmm::set_last_error("ccmm_psrf: Too few samples");
    return CCMM_ERR_ARG;
  }
  for (int d = 0; d < D; ++d)
    R[d] = psrf_one(n, M, [&](int t, int i) { return X[(size_t(i) * D + d) * n + t]; });
  return CCMM_OK;
}

namespace {
// mean over the rate's months at the ELB of psrf(.) per cell: chains = false averages the reference's
// one-chain statistic (first / last thirds of each chain, DiagnosticsShadowrate.m:82-91) over the C
// chains; chains = true treats the C chains as the sequences of one psrf (M >= 2 draws each)
int shadow_psrf(int M, int Ns, int elbT, int ldT, int C, const double* draws, const uint8_t* mask, double* out,
                bool chains, const char* who) {
  if (M < 1 || Ns < 1 || elbT < 0 || ldT < elbT || C < 1 || !out || (elbT > 0 && (!draws || !mask))) {
    ccmm::set_last_error(std::string(who) + ": invalid arguments");
    return CCMM_ERR_ARG;
  }
  // psrf stops with 'Too few samples' (DiagnosticsShadowrate.m:103-105) when a sequence would be
  // empty; here the diagnostic is NaN instead, so a short run still returns its draws
  const bool too_few = chains ? (C < 2 || M < 2) : M / 3 < 1;
  for (int s = 0; s < Ns; ++s) {
    if (too_few) {
      out[s] = kNaN;
      continue;
    }
    // DiagnosticsShadowrate(shadowrate_all(:, s, ELBdummy(startELB:thisT, s)), s): the mean of
    // psrf over the cells of rate s at the ELB (NaN: mean of an empty row)
    double sum = 0.0;
    int cells = 0;
    for (int t = 0; t < elbT; ++t) {
      if (!mask[size_t(t) * Ns + s]) continue;
      // draws M x Ns x ldT x C: element (m, s, t, c)
      auto at = [&](int m, int c) { return draws[((size_t(c) * ldT + t) * Ns + s) * M + m]; };
      if (chains) {
        sum += psrf_one(M, C, [&](int k, int i) { return at(k, i); });
      } else {
        const int m3 = M / 3;
        double rc = 0.0;
        for (int c = 0; c < C; ++c) rc += psrf_one(m3, 2, [&](int k, int i) { return at(i == 0 ? k : M - m3 + k, c); });
        sum += rc / C;
      }
      ++cells;
    }
    out[s] = cells ? sum / cells : kNaN;
  }
  return CCMM_OK;
}
}  // namespace

extern "C" int ccmm_shadowrate_psrf(int M, int Ns, int elbT, int ldT, int C, const double* draws,
                                    const uint8_t* mask, double* out) {
  return shadow_psrf(M, Ns, elbT, ldT, C, draws, mask, out, false, "ccmm_shadowrate_psrf");
}

extern "C" int ccmm_shadowrate_psrf_chains(int M, int Ns, int elbT, int ldT, int C, const double* draws,
                                           const uint8_t* mask, double* out) {
  return shadow_psrf(M, Ns, elbT, ldT, C, draws, mask, out, true, "ccmm_shadowrate_psrf_chains");
}
