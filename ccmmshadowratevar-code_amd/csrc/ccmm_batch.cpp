// ccmm_run_batch (include/ccmm.h): the vintage loop of goVARshadowrateBlockHybrid.m:258-517
// (goVARhybrid.m:258, goVAR.m:242) as one device-resident chain set, composed from the public
// chain-set entry points.  Host code only; the sweeps, forecasts and summaries run on the device.
#include <algorithm>
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

struct BatchError {
  int rc;
};

void check(int rc) {
  if (rc < 0) throw BatchError{rc};
}

void arg(bool ok, const char* msg) {
  if (!ok) {
    ccmm::set_last_error(std::string("ccmm_run_batch: ") + msg);
    throw BatchError{CCMM_ERR_ARG};
  }
}

// log(mean(exp(x))) with the max shift of goVARshadowrateBlockHybrid.m:438-439
double logmeanexp(const std::vector<double>& x) {
  double m = -std::numeric_limits<double>::infinity();
  for (double v : x) {
    if (std::isnan(v)) return kNaN;  // mean(exp(x - m)) is NaN as soon as one score is
    m = std::max(m, v);
  }
  if (!std::isfinite(m)) return m;
  double s = 0.0;
  for (double v : x) s += std::exp(v - m);
  return std::log(s / double(x.size())) + m;
}

struct ChainSet {
  ccmm_chains* h = nullptr;
  ~ChainSet() {
    if (h) ccmm_chains_destroy(h);
  }
};

struct Runner {
  const ccmm_batch_config& cf;
  const ccmm_vintage* vin;
  int V, N, p, K, Ns, C, H, Nd, Ny;
  bool shadow, hybrid;
  int elbTall;  // max elbT over all V vintages (output layout)
  int warn = 0;  // CCMM_WARN_MVNCDF from a forecast record

  Runner(const ccmm_batch_config& c, int V_, const ccmm_vintage* v) : cf(c), vin(v), V(V_) {
    N = cf.N;
    p = cf.p;
    shadow = cf.model == CCMM_MODEL_BLOCKHYBRID || cf.model == CCMM_MODEL_HYBRID;
    hybrid = cf.model == CCMM_MODEL_HYBRID;
    Ns = shadow ? cf.Ns : 0;
    K = N * p + 1 + (hybrid ? Ns * p : 0);
    C = cf.nchains;
    H = cf.H;
    Nd = cf.MCMCdraws > 0 ? cf.fcstNdraws / cf.MCMCdraws : 0;
    Ny = 0;  // counted in validate(), once ndxYields is known to be non-NULL
    elbTall = 0;
    for (int v = 0; v < V; ++v)
      if (shadow) elbTall = std::max(elbTall, vin[v].T - vin[v].elbT0);
  }

  void fcst_rc(int rc) {
    check(rc);
    if (rc == CCMM_WARN_MVNCDF) warn = rc;
  }

  void validate() {
    arg(cf.model == CCMM_MODEL_LINEAR || shadow, "model must be linear, block hybrid or hybrid");
    arg(N >= 1 && p >= 1 && C >= 1 && V >= 0, "N, p, nchains must be positive");
    arg(cf.MCMCdraws >= 1 && cf.burnin >= 0, "MCMCdraws >= 1, burnin >= 0");
    arg(cf.fcstNdraws >= cf.MCMCdraws && cf.fcstNdraws % cf.MCMCdraws == 0,
        "fcstNdraws must be multiple of MCMCdraws");  // goVARshadowrateBlockHybrid.m:123-126
    arg(H >= 1 && cf.ndxYields, "H >= 1 and ndxYields required");
    for (int i = 0; i < N; ++i) Ny += cf.ndxYields[i] != 0;
    arg(!shadow || (Ns >= 1 && cf.ndxS), "shadow-rate models need Ns >= 1 and ndxS");
    arg(!hybrid || !cf.actual_block, "actual_block must be NULL for the hybrid model");
    arg(cf.model != CCMM_MODEL_BLOCKHYBRID || cf.actual_block, "block hybrid needs actual_block");
    arg(!cf.postprocess || cf.nq == 0 || cf.pct, "pct required for nq > 0");
    for (int v = 0; v < V; ++v) {
      const ccmm_vintage& u = vin[v];
      arg(u.T > p && u.Y && u.X && u.iVdiag && u.iVb && u.sPHI && u.h0mean && u.h0vcvsqrt && u.PAI0 &&
              u.sqrtht0 && u.yrealized,
          "vintage arrays missing");
      arg(!shadow || (u.elbT0 >= 0 && u.elbT0 <= u.T && (u.elbT0 == u.T || u.sNaN)),
          "vintage ELB window invalid");
    }
  }

  void fill_nan(ccmm_batch_out* o, int v) {
    auto nanfill = [](double* a, size_t n, int v) {
      if (a) std::fill(a + size_t(v) * n, a + size_t(v + 1) * n, kNaN);
    };
    size_t NH = size_t(N) * H, KN = size_t(K) * N, nq = cf.nq;
    nanfill(o->logscore, 4, v);
    nanfill(o->fcstYhat, NH, v);
    nanfill(o->fcstShadowYhat, NH, v);
    nanfill(o->PAImean, KN, v);
    nanfill(o->PAIstdev, KN, v);
    nanfill(o->shadowrate_all, size_t(cf.MCMCdraws) * Ns * elbTall * C, v);
    if (o->countELBaccept) o->countELBaccept[v] = -1;
    nanfill(o->fcstYmedian, NH, v);
    nanfill(o->fcstYcrps, NH, v);
    nanfill(o->fcstYquantiles, NH * nq, v);
    nanfill(o->fcstYcummedian, NH, v);
    nanfill(o->fcstYcumcrps, NH, v);
    nanfill(o->fcstYcumquantiles, NH * nq, v);
    nanfill(o->fcstShadowYmedian, size_t(Ny) * H, v);
    nanfill(o->fcstShadowYquantiles, size_t(Ny) * H * nq, v);
    nanfill(o->PAImedian, KN, v);
    nanfill(o->PAIquantiles, KN * nq, v);
    nanfill(o->scoreDraws, size_t(cf.fcstNdraws) * C * 4, v);
    nanfill(o->shadowratePSRF, size_t(Ns), v);
    nanfill(o->shadowratePSRFchains, size_t(Ns), v);
  }

  // One chain set over the vintages `vs` (indices into vin) on attempt `attempt`; writes the
  // outputs of every vintage whose chains all finished unflagged and returns the others.
  std::vector<int> run(ccmm_ctx* ctx, const std::vector<int>& vs, int attempt, ccmm_batch_out* o) {
    const int nv = int(vs.size());
    const int B = C * nv;
    const int M = cf.MCMCdraws;
    int Tmax = 0, elbTmax = 0;
    for (int v : vs) {
      Tmax = std::max(Tmax, vin[v].T);
      if (shadow) elbTmax = std::max(elbTmax, vin[v].T - vin[v].elbT0);
    }
    const int chunk = std::max(1, std::min(cf.chunk > 0 ? cf.chunk : 50, M));
    ccmm_chain_config cc{};
    cc.model = cf.model;
    cc.N = N;
    cc.p = p;
    cc.K = K;
    cc.T = Tmax;
    cc.B = B;
    cc.ndata = nv;
    cc.dPHI = N + 3;  // mcmcVAR.m:164
    cc.rng_crn = 0;
    cc.store_capacity = cf.postprocess ? M : chunk;
    cc.logy2offset = 1e-3;
    cc.seed = cf.seed;
    cc.Ns = Ns;
    cc.elbTmax = shadow ? std::max(elbTmax, 1) : 0;
    cc.elb_gibbsburn = cf.gibbsburn;
    cc.elb = cf.elb;
    ChainSet cs;
    cs.h = ccmm_chains_create(ctx, &cc);
    if (!cs.h) throw BatchError{CCMM_ERR_ARG};
    ccmm_chains* ch = cs.h;
    for (int s = 0; s < nv; ++s) {
      const ccmm_vintage& u = vin[vs[s]];
      check(ccmm_chains_set_data(ch, s, u.T, u.Y, u.X, u.iVdiag, u.iVb, u.sPHI, u.h0mean, u.h0vcvsqrt));
    }
    if (shadow) check(ccmm_chains_set_elb_model(ch, cf.ndxS, hybrid ? nullptr : cf.actual_block));
    check(ccmm_chains_set_fcst(ch, H, Nd, cf.ndxYields, cf.postprocess ? 1 : 0));
    std::vector<int> slots(B);
    for (int b = 0; b < B; ++b) slots[b] = b / C;
    check(ccmm_chains_set_slots(ch, slots.data()));
    // PREVdraw at m == 0 (mcmcVARshadowrateBlockHybrid.m:308-317), replicated over the chains
    std::vector<double> PAI(size_t(K) * N * B), A(size_t(N) * N * B, 0.0), sq(size_t(Tmax) * N * B, 1.0),
        hh(size_t(Tmax) * N * B, 0.0), sP(size_t(N) * N * B, 0.0);
    for (int s = 0; s < nv; ++s) {
      const ccmm_vintage& u = vin[vs[s]];
      if (shadow) check(ccmm_chains_set_elb_slot(ch, s, u.elbT0, u.sNaN));
      check(ccmm_chains_set_fcst_slot(ch, s, u.yrealized));  // yrealized(:, 1)
      for (int c = 0; c < C; ++c) {
        const size_t b = size_t(s) * C + c;
        std::copy(u.PAI0, u.PAI0 + size_t(K) * N, PAI.begin() + b * K * N);
        for (int i = 0; i < N; ++i) {
          A[b * N * N + size_t(i) * N + i] = 1.0;
          sP[b * N * N + size_t(i) * N + i] = 0.01;
          for (int t = 0; t < u.T; ++t) {
            const double v = u.sqrtht0[size_t(i) * u.T + t];
            sq[b * Tmax * N + size_t(i) * Tmax + t] = v;
            hh[b * Tmax * N + size_t(i) * Tmax + t] = u.h0init ? u.h0init[size_t(i) * u.T + t] : 2.0 * std::log(v);
          }
        }
      }
    }
    check(ccmm_chains_set_state(ch, PAI.data(), A.data(), sq.data(), hh.data(), sP.data()));
    std::vector<uint32_t> ids(B);
    for (int s = 0; s < nv; ++s)
      for (int c = 0; c < C; ++c)
        ids[size_t(s) * C + c] = uint32_t(vin[vs[s]].unit) * uint32_t(C) + uint32_t(c) +
                                 uint32_t(attempt) * 1000003u;
    check(ccmm_chains_set_rng_ids(ch, ids.data()));
    const bool ps = shadow && cf.Nproposals > 0;
    if (ps)  // block hybrid: m >= MCMCburnin * .5 (:435); hybrid: every sweep (mcmcVARhybridGibbs.m:458)
      check(ccmm_chains_set_elb_ps(ch, cf.Nproposals, hybrid ? 1 : std::max(1, (cf.burnin + 1) / 2)));

    for (int done = 0; done < cf.burnin;) {
      const int n = std::min(chunk, cf.burnin - done);
      check(ccmm_chains_sweep(ch, n, nullptr, 0));
      done += n;
    }
    // kept sweeps
    const size_t KN = size_t(K) * N, NH = size_t(N) * H;
    std::vector<double> scores(size_t(Nd) * M * 4 * B);
    std::vector<double> fYsum(NH * B, 0.0), fYcsum(NH * B, 0.0), Psum, P2sum;
    std::vector<double> shadowd;  // M x Ns x elbTmax x B
    const int eT = cc.elbTmax;
    if (shadow && (o->shadowrate_all || o->shadowratePSRF || o->shadowratePSRFchains)) shadowd.assign(size_t(M) * Ns * eT * B, kNaN);
    if (!cf.postprocess) {
      Psum.assign(KN * B, 0.0);
      P2sum.assign(KN * B, 0.0);
    }
    std::vector<double> sc, fy, fyc, sd;
    for (int done = 0; done < M;) {
      const int n = std::min(chunk, M - done);
      check(ccmm_chains_sweep(ch, n, nullptr, 1));
      if (!cf.postprocess) {
        sc.assign(size_t(Nd) * n * 4 * B, 0.0);
        fy.assign(NH * B, 0.0);
        fyc.assign(NH * B, 0.0);
        fcst_rc(ccmm_chains_get_fcst(ch, sc.data(), fy.data(), fyc.data(), nullptr, nullptr, nullptr));
        if (!shadowd.empty()) sd.assign(size_t(n) * Ns * eT * B, 0.0);
        // PAI sums over the draws on the device (running, in draw order: the host loop's order and
        // rounding), so the draws themselves never cross PCIe
        check(ccmm_chains_pai_moments(ch, done == 0, nullptr, nullptr));
        check(ccmm_chains_get_draws(ch, nullptr, nullptr, nullptr, nullptr, sd.empty() ? nullptr : sd.data()));
        for (size_t i = 0; i < NH * B; ++i) {
          fYsum[i] += fy[i];
          fYcsum[i] += fyc[i];
        }
        // scores Nd x n x 4 x B into Nd x M x 4 x B at draw offset `done`
        for (size_t kb = 0; kb < size_t(4) * B; ++kb)
          std::copy(sc.begin() + kb * Nd * n, sc.begin() + (kb + 1) * Nd * n,
                    scores.begin() + kb * Nd * M + size_t(done) * Nd);
        if (!shadowd.empty())  // n x (Ns eT B) into M x (Ns eT B)
          for (size_t e = 0; e < size_t(Ns) * eT * B; ++e)
            for (int m = 0; m < n; ++m) shadowd[e * M + done + m] = sd[e * n + m];
      }
      done += n;
    }
    if (!cf.postprocess) check(ccmm_chains_pai_moments(ch, 0, Psum.data(), P2sum.data()));
    std::vector<int> status(B, 0), ca(B, 0), cb(B, 0);
    check(ccmm_chains_get_status(ch, status.data()));
    if (ps) check(ccmm_chains_get_ps(ch, ca.data(), cb.data(), nullptr));
    std::vector<int> failed;
    std::vector<char> ok(nv, 1);
    for (int s = 0; s < nv; ++s)
      for (int c = 0; c < C; ++c)
        if (status[size_t(s) * C + c] & ~CCMM_STATUS_INFO) ok[s] = 0;  // bits 1, 64: informational (valid draws)

    const size_t nq = size_t(cf.nq);
    if (cf.postprocess) {
      // goVARshadowrateBlockHybrid.m:349-480 on the device, per vintage (data slot)
      std::vector<double> mean, med, qs, sdv, crps, ycr(NH);
      std::vector<uint8_t> rows(cf.ndxYields, cf.ndxYields + N);
      for (int s = 0; s < nv; ++s) {
        if (!ok[s]) continue;
        const int v = vs[s];
        const ccmm_vintage& u = vin[v];
        auto sl = [v](double* a, size_t n) { return a ? a + size_t(v) * n : nullptr; };
        // fcstYdraws (source 1) against yrealized
        check(ccmm_chains_summaries(ch, 1, s, nullptr, nullptr, u.yrealized, cf.nq, cf.pct, nullptr,
                                    sl(o->fcstYmedian, NH), sl(o->fcstYquantiles, NH * nq), nullptr,
                                    sl(o->fcstYcrps, NH)));
        // ycumdraws against the cumulated realized values (:353)
        std::copy(u.yrealized, u.yrealized + NH, ycr.begin());
        if (cf.cumcode)
          for (int i = 0; i < N; ++i)
            if (cf.cumcode[i])
              for (int h = 1; h < H; ++h) ycr[size_t(h) * N + i] += ycr[size_t(h - 1) * N + i];
        check(ccmm_chains_summaries(ch, 1, s, nullptr, cf.cumcode, ycr.data(), cf.nq, cf.pct, nullptr,
                                    sl(o->fcstYcummedian, NH), sl(o->fcstYcumquantiles, NH * nq), nullptr,
                                    sl(o->fcstYcumcrps, NH)));
        // fcstShadowYdraws (source 0, ndxYIELDS rows)
        if (Ny > 0)
          check(ccmm_chains_summaries(ch, 0, s, rows.data(), nullptr, nullptr, cf.nq, cf.pct, nullptr,
                                      sl(o->fcstShadowYmedian, size_t(Ny) * H),
                                      sl(o->fcstShadowYquantiles, size_t(Ny) * H * nq), nullptr, nullptr));
        // PAI_all (source 2)
        check(ccmm_chains_summaries(ch, 2, s, nullptr, nullptr, nullptr, cf.nq, cf.pct, sl(o->PAImean, KN),
                                    sl(o->PAImedian, KN), sl(o->PAIquantiles, KN * nq), sl(o->PAIstdev, KN),
                                    nullptr));
      }
      fcst_rc(ccmm_chains_get_fcst(ch, scores.data(), fYsum.data(), fYcsum.data(), nullptr, nullptr, nullptr));
      if (!shadowd.empty())
        check(ccmm_chains_get_draws(ch, nullptr, nullptr, nullptr, nullptr, shadowd.data()));
    }

    // per-vintage results (:437-456)
    const size_t nk = size_t(M) * C;
    std::vector<double> x;
    for (int s = 0; s < nv; ++s) {
      const int v = vs[s];
      if (!ok[s]) {
        failed.push_back(v);
        continue;
      }
      for (int k = 0; k < 4; ++k) {
        x.clear();
        for (int c = 0; c < C; ++c) {
          const size_t b = size_t(s) * C + c;
          const double* src = scores.data() + (b * 4 + k) * Nd * M;
          x.insert(x.end(), src, src + size_t(Nd) * M);
        }
        if (o->logscore) o->logscore[size_t(v) * 4 + k] = logmeanexp(x);
        if (o->scoreDraws)
          std::copy(x.begin(), x.end(), o->scoreDraws + (size_t(v) * 4 + k) * Nd * M * C);
      }
      for (size_t e = 0; e < NH; ++e) {
        double a = 0.0, bsum = 0.0;
        for (int c = 0; c < C; ++c) {
          const size_t b = size_t(s) * C + c;
          a += fYcsum[b * NH + e];
          bsum += fYsum[b * NH + e];
        }
        if (o->fcstYhat) o->fcstYhat[size_t(v) * NH + e] = a / double(nk * Nd);
        if (o->fcstShadowYhat) o->fcstShadowYhat[size_t(v) * NH + e] = bsum / double(nk * Nd);
      }
      if (!cf.postprocess)
        for (size_t e = 0; e < KN; ++e) {
          double a = 0.0, a2 = 0.0;
          for (int c = 0; c < C; ++c) {
            a += Psum[(size_t(s) * C + c) * KN + e];
            a2 += P2sum[(size_t(s) * C + c) * KN + e];
          }
          const double mu = a / double(nk);
          if (o->PAImean) o->PAImean[size_t(v) * KN + e] = mu;
          if (o->PAIstdev) o->PAIstdev[size_t(v) * KN + e] = std::sqrt(std::max(a2 / double(nk) - mu * mu, 0.0));
        }
      if (o->countELBaccept) {
        int n = 0;
        for (int c = 0; c < C; ++c) n += ca[size_t(s) * C + c] + cb[size_t(s) * C + c];
        o->countELBaccept[v] = ps ? n : -1;
      }
      if (o->shadowrate_all && Ns > 0) {
        // M x Ns x eT (chain set) -> M x Ns x elbTall (output), NaN beyond the set's window
        double* dst = o->shadowrate_all + size_t(v) * M * Ns * elbTall * C;
        for (int c = 0; c < C; ++c)
          for (int t = 0; t < elbTall; ++t)
            for (int j = 0; j < Ns; ++j)
              for (int m = 0; m < M; ++m) {
                const size_t b = size_t(s) * C + c;
                dst[((size_t(c) * elbTall + t) * Ns + j) * M + m] =
                    t < eT ? shadowd[((b * eT + t) * Ns + j) * M + m] : kNaN;
              }
      }
      if (o->shadowratePSRF && Ns > 0) {
        // goVARshadowrateBlockHybrid.m:322-325: per shadow rate, psrf over its censored months
        const ccmm_vintage& u = vin[v];
        check(ccmm_shadowrate_psrf(M, Ns, u.T - u.elbT0, eT, C, shadowd.data() + size_t(s) * C * M * Ns * eT,
                                   u.sNaN, o->shadowratePSRF + size_t(v) * Ns));
      }
      if (o->shadowratePSRFchains && Ns > 0) {  // the across-chains form (no reference counterpart)
        const ccmm_vintage& u = vin[v];
        check(ccmm_shadowrate_psrf_chains(M, Ns, u.T - u.elbT0, eT, C,
                                          shadowd.data() + size_t(s) * C * M * Ns * eT, u.sNaN,
                                          o->shadowratePSRFchains + size_t(v) * Ns));
      }
      if (o->attempts) o->attempts[v] = attempt + 1;
    }
    return failed;
  }
};

}  // namespace

extern "C" int ccmm_run_batch(ccmm_ctx* ctx, const ccmm_batch_config* cfg, int V, const ccmm_vintage* vintages,
                              ccmm_batch_out* out) {
  try {
    if (!ctx || !cfg || !out || (V > 0 && !vintages)) {
      ccmm::set_last_error("ccmm_run_batch: null argument");
      return CCMM_ERR_ARG;
    }
    Runner r(*cfg, V, vintages);
    r.validate();
    std::vector<int> todo(V);
    for (int v = 0; v < V; ++v) todo[v] = v;
    for (int attempt = 0; !todo.empty(); ++attempt) {
      std::vector<int> failed = r.run(ctx, todo, attempt, out);
      if (failed.empty()) break;
      if (attempt >= cfg->max_retries) {  // give up: NaN outputs for the unit
        for (int v : failed) {
          r.fill_nan(out, v);
          if (out->attempts) out->attempts[v] = attempt + 2;
        }
        break;
      }
      todo = failed;
    }
    const int rc = ccmm_synchronize(ctx);
    return rc != 0 ? rc : r.warn;
  } catch (const BatchError& e) {
    return e.rc;
  } catch (const std::exception& e) {
    ccmm::set_last_error(std::string("ccmm_run_batch: ") + e.what());
    return CCMM_ERR_HIP;
  }
}
