// C-ABI implementation of libccmm (include/ccmm.h): contexts, device-resident
// chain sets and the block-level drop-ins.  Host code only: the kernels are defined in their own
// translation units (ccmm_kernels / ccmm_gram_chol / ccmm_cta_solve / ccmm_elb / ccmm_ps / ccmm_fcst /
// ccmm_lag / ccmm_svpart / ccmm_big / ccmm_bign / ccmm_post / ccmm_girf) and declared in their headers.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <atomic>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "ccmm_sweep.h"
#include "ccmm_elb.h"
#include "ccmm_fcst.h"
#include "ccmm_lag.h"
#include "ccmm_svpart.h"
#include "ccmm_big.h"
#include "ccmm_bign.h"
#include "ccmm_post.h"
#include "ccmm_girf.h"
#include <cstdlib>

using namespace ccmm;

namespace {

thread_local std::string g_err;

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct ArgError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHECK(x)                                                                        \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess)                                                                  \
      throw HipError(std::string(#x) + ": " + hipGetErrorString(e_) + " (" __FILE__ ":" + \
                     std::to_string(__LINE__) + ")");                                      \
  } while (0)

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const ArgError& e) {
    g_err = e.what();
    return CCMM_ERR_ARG;
  } catch (const HipError& e) {
    g_err = e.what();
    return CCMM_ERR_HIP;
  } catch (const std::exception& e) {
    g_err = e.what();
    return CCMM_ERR_HIP;
  }
}

void require(bool ok, const char* msg) {
  if (!ok) throw ArgError(msg);
}

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    if (count <= n && p) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (count == 0) return;
    HIPCHECK(hipMalloc(&p, count * sizeof(T)));
    n = count;
    // debug: CCMM_POISON=1 fills new allocations with 0xFF bytes (NaN doubles) to expose
    // reads of never-written device memory
#ifdef CCMM_ABLATION
    static const bool poison = std::getenv("CCMM_POISON") != nullptr;
    if (poison) HIPCHECK(hipMemset(p, 0xFF, count * sizeof(T)));
#endif
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};

// small dense host helpers (N <= 128): lower Cholesky and SPD inverse, column-major
void host_chol(std::vector<double>& A, int n) {
  for (int j = 0; j < n; ++j) {
    double s = A[j + j * n];
    for (int k = 0; k < j; ++k) s -= A[j + k * n] * A[j + k * n];
    if (!(s > 0)) throw ArgError("matrix not positive definite");
    const double d = std::sqrt(s);
    A[j + j * n] = d;
    for (int i = j + 1; i < n; ++i) {
      double v = A[i + j * n];
      for (int k = 0; k < j; ++k) v -= A[i + k * n] * A[j + k * n];
      A[i + j * n] = v / d;
    }
    for (int i = 0; i < j; ++i) A[i + j * n] = 0.0;
  }
}

std::vector<double> host_spd_inverse(const std::vector<double>& A, int n) {
  std::vector<double> L = A;
  host_chol(L, n);
  std::vector<double> inv(n * n, 0.0);
  for (int col = 0; col < n; ++col) {
    std::vector<double> x(n, 0.0);
    for (int i = 0; i < n; ++i) {  // L y = e_col
      double v = (i == col) ? 1.0 : 0.0;
      for (int k = 0; k < i; ++k) v -= L[i + k * n] * x[k];
      x[i] = v / L[i + i * n];
    }
    for (int i = n - 1; i >= 0; --i) {  // L' z = y
      double v = x[i];
      for (int k = i + 1; k < n; ++k) v -= L[k + i * n] * x[k];
      x[i] = v / L[i + i * n];
    }
    for (int i = 0; i < n; ++i) inv[i + col * n] = x[i];
  }
  return inv;
}

}  // namespace

// Gauss-Legendre nodes/weights by Newton on P_n (host, once); negative half
static GLNodes make_gl_nodes() {
  GLNodes g{};
  const int ns[3] = {6, 12, 20};
  for (int r = 0; r < 3; ++r) {
    const int n = ns[r];
    for (int i = 0; i < n / 2; ++i) {
      double x = -std::cos(M_PI * (i + 0.75) / (n + 0.5));
      double dp = 0.0;
      for (int it = 0; it < 100; ++it) {
        double p0 = 1.0, p1 = x;
        for (int k = 2; k <= n; ++k) {
          const double p2 = ((2.0 * k - 1.0) * x * p1 - (k - 1.0) * p0) / k;
          p0 = p1;
          p1 = p2;
        }
        dp = n * (x * p1 - p0) / (x * x - 1.0);
        const double dx = p1 / dp;
        x -= dx;
        if (std::fabs(dx) < 1e-17) break;
      }
      g.x[r][i] = x;
      g.w[r][i] = 2.0 / ((1.0 - x * x) * dp * dp);
    }
  }
  return g;
}

struct ccmm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  Options opt;  // inherited by the chain sets created on it and used by the block-level drop-ins
};

enum KernelId {
  KID_RESID,
  KID_WEIGHTS,
  KID_SOLVE,
  KID_ASTEP,
  KID_SVMIX,
  KID_SVSAMPLE,
  KID_PHIGEN,
  KID_PHI,
  KID_STORE,
  KID_GRAMCHOL,
  KID_ELBPREP,
  KID_ELBCOND,
  KID_ELBGIBBS,
  KID_ELBREBUILD,
  KID_GRAMLAG,
  KID_SOLVELAG,
  KID_FCST,
  KID_GRAMBIG,
  KID_CHOLBIG,
  KID_SOLVEBIG,
  KID_ASTEPBIG,
  KID_SVBIG,
  KID_PHIBIG,
  KID_PSCHOL,
  KID_PSPROP,
  KID_COUNT
};
static const char* kKernelNames[KID_COUNT] = {"k_resid", "k_cta_weights",
                                              "k_cta_solve", "k_astep", "k_sv_mix", "k_sv_part",
                                              "k_phi_gen", "k_phi", "k_store", "k_gram_chol",
                                              "k_elb_prep", "k_elb_cond", "k_elb_gibbs",
                                              "k_elb_rebuild", "k_gram_chol_lag",
                                              "k_cta_solve_lag", "k_fcst",
                                              "k_gram_big", "k_chol_big", "k_cta_solve_big",
                                              "k_astep_big", "k_sv_big", "k_phi_big",
                                              "k_ps_chol", "k_ps_prop"};

// MFMA phase lock: chain sets given the same id (ccmm_chains_set_mfma_lock) on one device
// serialise their CTA Gram + Cholesky phase through a cross-stream event, so the groups fall
// out of step and one group's per-chain sequential blocks (CTA solve, SV, ELB Gibbs) run
// beside another group's MFMA phase instead of all groups contending for the CUs at once.
struct PhaseLock {
  std::mutex m;
  hipEvent_t last = nullptr;  // event recorded after the latest enqueued locked phase
};

static PhaseLock& phase_lock(int device, int id) {
  static std::mutex gm;
  static std::map<std::pair<int, int>, std::unique_ptr<PhaseLock>> locks;
  std::lock_guard<std::mutex> g(gm);
  auto& p = locks[{device, id}];
  if (!p) p.reset(new PhaseLock);
  return *p;
}

// the predictive-density kernels of one kept draw per chain (ccmm_fcst.hip): the paths (one
// single-wave workgroup per (draw, chain); job Nd = the linear model's mean path) then the scores
static void launch_fcst(hipStream_t st, FcstArgs& a, double* sv1, bool reg_opt) {
  const bool reg = fcst_reg_path(a.N, a.p, a.bh) && reg_opt;
  a.hc = fcst_chunk(a.N, a.Kx, a.p, a.H, reg);
  a.sv1 = sv1;
  const size_t lp = fcst_paths_lds_doubles(a.N, a.Kx, a.p, a.hc, reg) * sizeof(double);
  const size_t ls = fcst_scores_lds_doubles(a.N) * sizeof(double);
  if (lp > 160 * 1024) throw std::runtime_error("forecast state does not fit LDS");
  const int njobs = a.bh ? a.Nd : a.Nd + 1;
  const bool even = reg && a.N % 2 == 0 && a.N < kFcstRegN;
  const void* kf = even ? (const void*)k_fcst<kFcstRegN - 1>
                        : reg ? (const void*)k_fcst<kFcstRegN> : (const void*)k_fcst<0>;
  HIPCHECK(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lp));
  if (even)
    hipLaunchKernelGGL(k_fcst<kFcstRegN - 1>, dim3(njobs, a.B), dim3(64), lp, st, a);
  else if (reg)
    hipLaunchKernelGGL(k_fcst<kFcstRegN>, dim3(njobs, a.B), dim3(64), lp, st, a);
  else
    hipLaunchKernelGGL(k_fcst<0>, dim3(njobs, a.B), dim3(64), lp, st, a);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipFuncSetAttribute((const void*)k_fcst_scores, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ls));
  hipLaunchKernelGGL(k_fcst_scores, dim3(a.Nd, a.B), dim3(64), ls, st, a);
  HIPCHECK(hipGetLastError());
}

struct ccmm_chains {
  ccmm_ctx* ctx = nullptr;
  ccmm_chain_config cfg{};
  Dims d{};
  int nslabX = 0, nslabY = 0;
  // per-slot data
  std::vector<int> hT;
  DBuf<int> Tslot, slot, xidx, yidx, status;
  DBuf<double> Xpool, Ypool, iVdiag, iVb, sPHI, V0inv, V0invm;
  // chain state
  DBuf<double> PAI, A, invA, sqrtht, h, h0, sqrtPHI, PHI, E, logy2, eta, svobs, svir, W, ih2;
  DBuf<int8_t> kai;
  DBuf<double> G, rdiag, svLd, svw, svSep, svG, Zphi;
  DBuf<double> crn;
  // storage of kept draws
  DBuf<double> sPAI, sPHI_, sInvA, sSqrtht, sShadow;
  DBuf<double> solveXch;  // k_cta_solve_lag split: X'v half partials (SolveXch)
  DBuf<uint64_t> solveFlag;
  uint64_t solve_epoch = 0;
  Options opt;  // kernel forms and schedules (ccmm_chains_set_option), from the context at create
  DBuf<double> paiMom;  // running PAI sums | sums of squares (ccmm_chains_pai_moments)
  int mom_done = 0;     // stored draws already added to paiMom
  // block-hybrid ELB model (mcmcVARshadowrateBlockHybrid.m): X/Y slabs 0..ndata-1 hold
  // the vintages' actual data, slabs ndata + c the chain's shadow-rate data
  bool bh = false;
  // hybrid model (mcmcVARhybridGibbs.m): same chain layout as bh, one design per chain
  // (CTA, no actual-rate block), trailing columns = censored actual-rate lags
  bool hybrid = false;
  bool fcst_bh = false;  // block-hybrid companion in the predictive density (k_fcst a.bh)
  bool have_elb_model = false;
  std::vector<bool> have_elb_slot;
  std::vector<int> hNdxS, hElbT0, hElbT;
  std::vector<uint8_t> hActual;
  DBuf<int> dNdxS, dElbT0, dElbT, dNcens, dCens;
  DBuf<uint8_t> dActual, dSNaN;
  DBuf<double> ePhi, eY0, eYt, eEt, eCond, eScur;
  std::vector<std::vector<uint8_t>> hSNaN;  // per slot, elbTmax x Ns (t-major)
  // acceptance-sampling branch (ccmm_ps.hip): ps_np proposals per sweep from sweep
  // m = ps_from_m on (1-based, m = sweep + 1; the reference: m >= MCMCburnin/2, :435)
  int ps_np = 0, ps_from_m = -1, psW = 0, ps_nmax = 0;
  bool ps_dirty = true;
  DBuf<double> eEtPS, psL, psY;
  DBuf<int> psCell, psN, psAcc, psFlag, psCount, sAccept;
  int stored = 0;
  uint32_t sweep = 0;
  // predictive density of every stored sweep (mcmcVAR.m:298-381,
  // mcmcVARshadowrateBlockHybrid.m:550-669), kept on the device
  bool have_fcst = false;
  int fH = 0, fNd = 0, fKeep = 0, fstored = 0, fldXj = 0;
  DBuf<uint8_t> fYields, fRecFloor;
  bool have_rec_floor = false;
  std::vector<bool> have_fcst_slot;
  DBuf<double> fYreal, fXj, fY, fYc, fYhat, fSc, fYsum, fYcsum, fYhatsum, fScStore, fPaths, fPathsC, fSv1;
  DBuf<int> fStatus;
  // Philox stream ids (counter word 1) per chain; default the chain index
  bool have_ids = false;
  DBuf<uint32_t> rngIds;
  bool resid_valid = false;
  bool have_state = false;
  // timing-only ablation of k_gram_chol (results invalid): 1 = no SYRK, 2 = no Cholesky
  int gc_mode = env_ablation("CCMM_GC_MODE", 0);
  std::vector<bool> have_slot;
  // lag-structured design (ccmm_lag.hip): D slabs parallel to the X slabs
  bool lag_capable = false;
  int lagNT = 0, ldd = 0, drows = 0;
  std::vector<bool> slot_lag;
  DBuf<double> Dpool;
  // large path: column-major lag twin of every X slab (ccmm_big.h ColX), when each slab's X is
  // [1, lags 1..p of N (+ Ns) data columns]; k_elb_rebuild keeps the chains' twins current
  bool colx_capable = false;
  std::vector<bool> slot_colx;
  DBuf<double> Dcpool;
  DBuf<int> dXoff;
  int dcld = 0, dcext = 0;
  size_t dcslab = 0;
  DBuf<int> dColmap, astepTab;
  // large-system CTA (ccmm_big.hip): K > 256 or N > 32, or option large_path
  bool big = false;
  int nGroups = 0;
  DBuf<int4> bigGroups;
  DBuf<double> Ubuf, Dinv, bigW, bigScr;
  // profiling
  bool profiling = false;
  struct Ev {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Ev> pending;
  std::vector<hipEvent_t> evpool;
  double kms[KID_COUNT] = {};
  int64_t kcount[KID_COUNT] = {};

  int mfma_lock = 0;
  hipEvent_t mfma_ev = nullptr;

  ~ccmm_chains() {
    if (evFcstFork) {
      (void)hipEventDestroy(evFcstFork);
      (void)hipEventDestroy(evFcstDone);
    }
    if (aux2) {
      (void)hipStreamSynchronize(aux2);
      (void)hipEventDestroy(evSpec);
      (void)hipEventDestroy(evSpecJoin);
      (void)hipStreamDestroy(aux2);
    }
    if (aux) {
      (void)hipStreamSynchronize(aux);
      (void)hipEventDestroy(evFork);
      (void)hipEventDestroy(evJoin);
      (void)hipStreamDestroy(aux);
    }
    if (mfma_ev) {
      PhaseLock& L = phase_lock(ctx->device, mfma_lock);
      std::lock_guard<std::mutex> g(L.m);
      if (L.last == mfma_ev) L.last = nullptr;
      (void)hipEventDestroy(mfma_ev);
    }
    for (auto& e : pending) {
      evpool.push_back(e.a);
      evpool.push_back(e.b);
    }
    for (auto e : evpool) (void)hipEventDestroy(e);
  }

  hipEvent_t get_event() {
    if (!evpool.empty()) {
      hipEvent_t e = evpool.back();
      evpool.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e));
    return e;
  }

  template <class L>
  void launch(int kid, L&& fn, hipStream_t on = nullptr) {
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t st = on ? on : ctx->stream;
    if (profiling) {
      a = get_event();
      b = get_event();
      HIPCHECK(hipEventRecord(a, st));
    }
    fn();
    HIPCHECK(hipGetLastError());
    if (profiling) {
      HIPCHECK(hipEventRecord(b, st));
      pending.push_back({kid, a, b});
    }
  }

  // auxiliary stream of the sweep: the inverse-Wishart block runs on it beside the ELB step, which
  // reads none of its inputs or outputs (mcmcVARshadowrateBlockHybrid.m:386-392 vs :395-520); the
  // main stream waits for it before the draw store, the forecasts and the next sweep's SV block
  hipStream_t aux = nullptr;
  hipEvent_t evFork = nullptr, evJoin = nullptr;
  void ensure_aux() {
    if (aux) return;
    HIPCHECK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    HIPCHECK(hipEventCreateWithFlags(&evFork, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&evJoin, hipEventDisableTiming));
  }

  void collect_profile() {
    if (pending.empty()) return;
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    for (auto& e : pending) {
      float ms = 0.f;
      HIPCHECK(hipEventElapsedTime(&ms, e.a, e.b));
      kms[e.kid] += ms;
      kcount[e.kid] += 1;
      evpool.push_back(e.a);
      evpool.push_back(e.b);
    }
    pending.clear();
  }

  ChainState view() {
    ChainState cs;
    cs.slot = slot.p;
    cs.PAI = PAI.p;
    cs.A = A.p;
    cs.invA = invA.p;
    cs.sqrtht = sqrtht.p;
    cs.h = h.p;
    cs.sqrtPHI = sqrtPHI.p;
    cs.PHI = PHI.p;
    cs.E = E.p;
    cs.logy2 = logy2.p;
    cs.eta = eta.p;
    cs.svobs = svobs.p;
    cs.svir = svir.p;
    cs.kai = kai.p;
    cs.W = W.p;
    cs.ih2 = ih2.p;
    cs.G = G.p;
    cs.svLd = svLd.p;
    cs.svw = svw.p;
    cs.Zphi = Zphi.p;
    cs.status = status.p;
    cs.Aelb = aswitch ? AelbD.p : nullptr;
    cs.atELB = aswitch ? atELBD.p : nullptr;
    return cs;
  }
  // CTAsysAswitching (block-level drop-in only): second A matrix for the months at the ELB
  bool aswitch = false;
  DBuf<double> AelbD;
  DBuf<uint8_t> atELBD;
  XSel xsel() const { return XSel{Xpool.p, xidx.p, Ypool.p, yidx.p}; }

  int64_t crn_off[kRngBlocks] = {};
  int64_t crn_len = 0;

  void init(ccmm_ctx* c, const ccmm_chain_config& cf, int nX, int nY) {
    ctx = c;
    cfg = cf;
    opt = c->opt;
    bh = cf.model == CCMM_MODEL_BLOCKHYBRID || cf.model == CCMM_MODEL_HYBRID || cf.model == CCMM_MODEL_SHADOWRATE;
    // mcmcVARshadowrate.m: the ELB step of the block hybrid, one shadow-rate design for every
    // equation (no actual-rate block), the linear model's predictive density (:536-641)
    fcst_bh = bh && cf.model != CCMM_MODEL_SHADOWRATE;
    hybrid = cf.model == CCMM_MODEL_HYBRID;
    if (bh) {
      require(cf.Ns >= 1 && cf.Ns <= kElbNsMax, "Ns must be in [1, 5]");
      require(cf.elbTmax >= 0 && cf.elbTmax <= cf.T, "elbTmax must be in [0, T]");
      require(cf.elbTmax < 65536, "elbTmax must be < 65536");  // k_elb_gibbs month list
      require(cf.elb_gibbsburn >= 0, "elb_gibbsburn must be >= 0");
      require(2 * cf.p * cf.Ns <= kElbColMax, "2 p Ns must be <= 128");
      require(cf.p >= 1, "p must be >= 1");
    }
    require(cf.N >= 1 && cf.N <= kBigMaxN, "N must be in [1, 128]");
    if (hybrid)  // [1, lags of the N variables, lags of the Ns actual rates] (mcmcVARhybridGibbs.m:84)
      require(cf.K == cf.N * cf.p + 1 + cf.Ns * cf.p, "hybrid model: K must equal N*p+1+Ns*p");
    else
      require(cf.K == cf.N * cf.p + 1 || cf.p == 0, "K must equal N*p+1");
    require(cf.K >= 1 && cf.K <= 1536, "K must be in [1, 1536]");
    require(cf.T >= 2 && cf.B >= 1 && cf.ndata >= 1, "bad T/B/ndata");
    d.N = cf.N;
    d.p = cf.p;
    d.K = cf.K;
    d.KP = round_up(cf.K, kTile);
    d.TP = round_up(cf.T, kTChunk);
    d.B = cf.B;
    d.nmat = cf.B * cf.N;
    require(d.KP <= kBigMaxKP, "this build supports K <= 1536");
    // KP > 256: the register-tiled fused Gram + Cholesky (k_gram_chol) stops at 16 tiles; the
    // large path takes every larger system (the hybrid model, K = 277, included)
    big = d.KP > 256 || cf.N > kMaxNSmall || opt[OPT_LARGE_PATH] != 0;
    nslabX = nX;
    nslabY = nY;
    const size_t B = cf.B, N = cf.N, KP = d.KP, TP = d.TP;
    hT.assign(cf.ndata, cf.T);
    have_slot.assign(cf.ndata, false);
    Tslot.alloc(cf.ndata);
    slot.alloc(B);
    xidx.alloc(B * N);
    yidx.alloc(B);
    status.alloc(B);
    Xpool.alloc((size_t)nX * KP * TP);
    Ypool.alloc((size_t)nY * N * TP);
    HIPCHECK(hipMemsetAsync(Xpool.p, 0, Xpool.n * sizeof(double), ctx->stream));
    HIPCHECK(hipMemsetAsync(Ypool.p, 0, Ypool.n * sizeof(double), ctx->stream));
    init_lag(nX);
    init_colx();
    iVdiag.alloc((size_t)cf.ndata * N * KP);
    iVb.alloc((size_t)cf.ndata * N * KP);
    sPHI.alloc((size_t)cf.ndata * N * N);
    V0inv.alloc((size_t)cf.ndata * N * N);
    V0invm.alloc((size_t)cf.ndata * N);
    PAI.alloc(B * N * KP);
    HIPCHECK(hipMemsetAsync(PAI.p, 0, PAI.n * sizeof(double), ctx->stream));
    A.alloc(B * N * N);
    invA.alloc(B * N * N);
    sqrtht.alloc(B * N * TP);
    h.alloc(B * N * TP);
    h0.alloc(B * N);
    sqrtPHI.alloc(B * N * N);
    PHI.alloc(B * N * N);
    E.alloc(B * N * TP);
    logy2.alloc(B * N * TP);
    eta.alloc(B * N * TP);
    svobs.alloc(B * N * TP);
    svir.alloc(B * N * TP);
    kai.alloc(B * N * TP);
    W.alloc(B * N * TP);
    ih2.alloc(B * N * TP);
    std::vector<int> zeros(cf.ndata, cf.T);
    HIPCHECK(hipMemcpyAsync(Tslot.p, zeros.data(), cf.ndata * sizeof(int), hipMemcpyHostToDevice,
                            ctx->stream));
    if (bh) init_elb();
    std::vector<int> sl(B, 0);
    set_slots(sl.data());
    HIPCHECK(hipMemsetAsync(status.p, 0, B * sizeof(int), ctx->stream));
    layout_crn();
  }

  // CRN layout (blocks in CCMM_RNG_* order, sizes from Tmax); the predictive-density
  // block (mcmcVAR.m:302,306) is appended once ccmm_chains_set_fcst configured it
  void layout_crn() {
    const ccmm_chain_config& cf = cfg;
    const int64_t N = cf.N;
    int64_t o = 0;
    const int64_t T = cf.T;
    crn_off[CCMM_RNG_PAI] = o;
    o += (int64_t)cf.K * N;
    crn_off[CCMM_RNG_A] = o;
    o += (int64_t)N * (N - 1) / 2;
    crn_off[CCMM_RNG_SVU] = o;
    o += (int64_t)N * T;
    crn_off[CCMM_RNG_SVZ] = o;
    o += (int64_t)N * (T + 1);
    crn_off[CCMM_RNG_PHI] = o;
    o += (int64_t)N * (T + cf.dPHI);
    if (bh) {
      crn_off[CCMM_RNG_ELB] = o;
      o += (int64_t)cf.Ns * cf.elbTmax * (cf.elb_gibbsburn + 1);
    }
    if (have_fcst) {
      crn_off[CCMM_RNG_FCST] = o;
      o += 2 * N * fH * fNd;
    }
    if (bh && ps_np > 0) {  // randn(nmiss, Nproposals), column-major with leading dimension nmiss
      crn_off[CCMM_RNG_PS] = o;
      o += (int64_t)cf.Ns * cf.elbTmax * ps_np;
    }
    crn_len = o;
  }

  // The lag path needs X = [1, lags 1..p of the N variables] (mcmcVAR.m:62-72), a
  // supported tile count and D + weights resident in one CU's LDS.
  void init_lag(int nX) {
    slot_lag.assign(cfg.ndata, false);
    lag_capable = false;
    if (cfg.p < 1 || cfg.K != cfg.N * cfg.p + 1) return;
    const int N = cfg.N;
    lagNT = (N * cfg.p + 15) / 16;
    ldd = (N % 2 == 0) ? N + 1 : N + 2;  // odd stride, spare zero column N
    drows = cfg.T + cfg.p + 4;  // SYRK k-steps read up to row T + p + 2
    const size_t lds_max = 160 * 1024;
    if (!lag_supported_nt(lagNT) || N > 32 || 16 * lagNT + 1 > d.KP ||
        gl_lds_bytes(lagNT, drows, ldd, d.TP) > lds_max ||
        sl_lds_bytes(lagNT, drows, ldd, d.TP, N <= 8 ? 8 : (N <= 20 ? 20 : 32)) > lds_max)
      return;
    lag_capable = true;
    Dpool.alloc((size_t)nX * drows * ldd);
    HIPCHECK(hipMemsetAsync(Dpool.p, 0, Dpool.n * sizeof(double), ctx->stream));
    std::vector<int> cm(16 * lagNT);
    for (int a = 0; a < 16 * lagNT; ++a) {
      if (a < N * cfg.p) {
        const int l = a / N + 1, k = a % N;
        cm[a] = (cfg.p - l) * ldd + k;
      } else {
        cm[a] = N;  // spare zero column of row t
      }
    }
    dColmap.alloc(cm.size());
    HIPCHECK(hipMemcpy(dColmap.p, cm.data(), cm.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  // the lag twin of the large path: columns 0..N-1 the data, N..N+Ns-1 the hybrid's actual-rate
  // columns (mcmcVARhybridGibbs.m:77-84), then a column of ones (the intercept) and a zero column
  // (padded coefficients); row p + t = month t, rows 0..p-1 the presample
  void init_colx() {
    if (colx_capable || !big || cfg.p < 1) return;
    slot_colx.assign(cfg.ndata, false);
    const int N = cfg.N, p = cfg.p, ex = hybrid ? cfg.Ns : 0;
    if (cfg.K != N * p + 1 + ex * p) return;
    dcext = ex;
    dcld = round_up(d.TP + p, 8);
    dcslab = (size_t)(N + ex + 2) * dcld;
    Dcpool.alloc((size_t)nslabX * dcslab);
    HIPCHECK(hipMemsetAsync(Dcpool.p, 0, Dcpool.n * sizeof(double), ctx->stream));
    std::vector<int> off(d.KP);
    for (int a = 0; a < d.KP; ++a) {
      if (a == 0) {
        off[a] = (N + ex) * dcld;
      } else if (a >= cfg.K) {
        off[a] = (N + ex + 1) * dcld;
      } else if (a - 1 < N * p) {
        const int b = a - 1, l = b / N + 1, k = b % N;
        off[a] = k * dcld + p - l;
      } else {
        const int b = a - 1 - N * p, l = b / ex + 1, si = b % ex;
        off[a] = (N + si) * dcld + p - l;
      }
    }
    dXoff.alloc(d.KP);
    HIPCHECK(hipMemcpy(dXoff.p, off.data(), off.size() * sizeof(int), hipMemcpyHostToDevice));
    colx_capable = true;
  }
  // a slot's twin from its X (T x K): column k's rows from the lag-1 column one month later and the
  // presample from X's first row; exact check against every entry of X
  void try_upload_Dc(int slot, int T, const double* X) {
    if (!colx_capable) return;
    slot_colx[slot] = false;
    const int N = cfg.N, p = cfg.p, K = cfg.K, ex = dcext, nc = N + ex;
    std::vector<double> D(dcslab, 0.0);
    std::vector<int> off(K);
    HIPCHECK(hipMemcpy(off.data(), dXoff.p, K * sizeof(int), hipMemcpyDeviceToHost));
    auto colk = [&](int k, int l) { return k < N ? 1 + (l - 1) * N + k : 1 + N * p + (l - 1) * ex + (k - N); };
    for (int k = 0; k < nc; ++k) {
      for (int l = 1; l <= p; ++l) D[(size_t)k * dcld + p - l] = X[(size_t)colk(k, l) * T];  // rows 0..p-1
      for (int t = 1; t < T; ++t) D[(size_t)k * dcld + p + t - 1] = X[(size_t)colk(k, 1) * T + t];
    }
    for (int t = 0; t < d.TP + p; ++t) D[(size_t)nc * dcld + t] = 1.0;
    for (int a = 0; a < K; ++a)
      for (int t = 0; t < T; ++t)
        if (X[(size_t)a * T + t] != D[(size_t)off[a] + t]) return;
    HIPCHECK(hipMemcpy(Dcpool.p + (size_t)slot * dcslab, D.data(), D.size() * sizeof(double), hipMemcpyHostToDevice));
    slot_colx[slot] = true;
  }
  ColX colx() const {
    bool on = colx_capable && opt[OPT_BIG_LAGX];
    for (int s = 0; on && s < cfg.ndata; ++s) on = slot_colx[s];
    return on ? ColX{Dcpool.p, dXoff.p, (long long)dcslab, dcld, (int)(dcslab / dcld)} : ColX{nullptr, nullptr, 0, 0, 0};
  }
  bool lag_active() const {
    if (!lag_capable || !opt[OPT_LAG]) return false;
    for (int s = 0; s < cfg.ndata; ++s)
      if (!slot_lag[s]) return false;
    return true;
  }
  int lag_mode = env_ablation("CCMM_LAG_MODE", 0);
  // phase skips (timing only) and bit 128 (full-row block factors, same draws): ablation build only
  int sv_mode = env_ablation("CCMM_SV_MODE", 0);
  // timing-only ablation of k_elb_gibbs (results invalid): 1 no truncnorm, 2 no uniforms
  int elb_mode = env_ablation("CCMM_ELB_MODE", 0);
  LagSel lagsel() const { return LagSel{Dpool.p, xidx.p, dColmap.p, ldd, drows, cfg.p, lag_mode}; }
  // D (rows x ldd) of a slot from its X (T x K) and Y (T x N): rows 0..p-1 from the
  // lags of X's first row, rows p.. = Y.  Exact check that X is that lag design.
  void try_upload_D(int slot, int T, const double* Y, const double* X) {
    slot_lag[slot] = false;
    if (!lag_capable) return;
    const int N = cfg.N, p = cfg.p, K = cfg.K;
    std::vector<double> D((size_t)drows * ldd, 0.0);
    for (int l = 1; l <= p; ++l)
      for (int k = 0; k < N; ++k) D[(size_t)(p - l) * ldd + k] = X[(size_t)(1 + (l - 1) * N + k) * T];
    for (int t = 0; t < T; ++t)
      for (int k = 0; k < N; ++k) D[(size_t)(t + p) * ldd + k] = Y[(size_t)k * T + t];
    for (int t = 0; t < T; ++t) {
      if (X[t] != 1.0) return;
      for (int a = 0; a < K - 1; ++a) {
        const int l = a / N + 1, k = a % N;
        if (X[(size_t)(1 + a) * T + t] != D[(size_t)(t + p - l) * ldd + k]) return;
      }
    }
    HIPCHECK(hipMemcpy(Dpool.p + (size_t)slot * drows * ldd, D.data(), D.size() * sizeof(double),
                       hipMemcpyHostToDevice));
    slot_lag[slot] = true;
  }

  void init_elb() {
    const size_t B = cfg.B, N = cfg.N, Ns = cfg.Ns, ET = std::max(cfg.elbTmax, 1), nd = cfg.ndata;
    have_elb_slot.assign(nd, false);
    hSNaN.assign(nd, std::vector<uint8_t>((size_t)ET * Ns, 0));
    hNdxS.assign(Ns, 0);
    hActual.assign(N, 1);
    hElbT0.assign(nd, cfg.T);
    hElbT.assign(nd, 0);
    dNdxS.alloc(Ns);
    dActual.alloc(N);
    dElbT0.alloc(nd);
    dElbT.alloc(nd);
    dNcens.alloc(nd);
    dCens.alloc(nd * ET);
    dSNaN.alloc(nd * ET * Ns);
    HIPCHECK(hipMemset(dElbT.p, 0, nd * sizeof(int)));
    HIPCHECK(hipMemset(dNcens.p, 0, nd * sizeof(int)));
    HIPCHECK(hipMemset(dSNaN.p, 0, dSNaN.n));
    ePhi.alloc(B * N * N * cfg.p);
    eY0.alloc(B * ET * N);
    eYt.alloc(B * ET * N);
    eEt.alloc(B * ET * N);
    eCond.alloc(B * ET * (size_t)elb_cond_stride(cfg.Ns, cfg.p, ps_np > 0));
    eScur.alloc(B * ET * Ns);
    HIPCHECK(hipMemset(eScur.p, 0, eScur.n * sizeof(double)));
  }

  const double* elb_yhat = nullptr;  // ccmm_gibbs_shadowrates: explicit YHAT0
  int elb_b3 = 0;                    // ccmm_gibbs_shadowrates_b3: no Y0 path, intercept in the state
  const double* elb_Amon = nullptr;  // ccmm_gibbs_shadowrates_b3: per-month structural matrices
  int elb_Afull = 0;                 // ccmm_gibbs_shadowrates*: A = inverse of a general impact matrix
  uint8_t* elb_flags = nullptr;      // drawTruncNormal branch flags of the last ELB step (or nullptr)
  DBuf<uint8_t> dElbFlags;
  ElbDev elb_view() const {
    ElbDev e{};
    e.Ns = cfg.Ns;
    e.p = cfg.p;
    e.elbTmax = std::max(cfg.elbTmax, 1);
    e.passes = cfg.elb_gibbsburn + 1;
    e.elb = cfg.elb;
    e.ndxS = dNdxS.p;
    e.actual = dActual.p;
    e.elbT0 = dElbT0.p;
    e.elbT = dElbT.p;
    e.sNaN = dSNaN.p;
    e.ncens = dNcens.p;
    e.cens = dCens.p;
    e.Xactual = Xpool.p;
    e.Phi = ePhi.p;
    e.Y0 = eY0.p;
    e.Yt = eYt.p;
    e.Et = eEt.p;
    e.cond = eCond.p;
    e.Scur = eScur.p;
    e.condStride = elb_cond_stride(cfg.Ns, cfg.p, ps_np > 0);
    e.kshadow = cfg.N * cfg.p + 1;
    e.K = cfg.K;
    e.mode = elb_mode;
    e.yhat = elb_yhat;
    e.flags = elb_flags;
    e.ps = 0;
    e.EtPS = eEtPS.p;
    e.psFlag = nullptr;
    e.b3 = elb_b3;
    e.Amon = elb_Amon;
    e.Afull = elb_Afull;
    e.spec = 0;
    e.psState = nullptr;
    e.psEpoch = 0;
    e.ScurSpec = nullptr;
    return e;
  }

  void set_elb_model(const int* ndxS, const uint8_t* actual) {
    const int N = cfg.N, Ns = cfg.Ns;
    for (int a = 0; a < Ns; ++a) {
      require(ndxS[a] >= 0 && ndxS[a] < N, "ndxS out of range");
      require(!actual[ndxS[a]], "a shadow-rate variable cannot be in the actual-rate block");
      if (a) require(ndxS[a] > ndxS[a - 1], "ndxS must be strictly increasing");
      hNdxS[a] = ndxS[a];
    }
    for (int i = 0; i < N; ++i) hActual[i] = actual[i] ? 1 : 0;
    HIPCHECK(hipMemcpy(dNdxS.p, hNdxS.data(), Ns * sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dActual.p, hActual.data(), N, hipMemcpyHostToDevice));
    have_elb_model = true;
    std::vector<int> sl(cfg.B);
    HIPCHECK(hipMemcpy(sl.data(), slot.p, cfg.B * sizeof(int), hipMemcpyDeviceToHost));
    set_slots(sl.data());
  }

  void set_elb_slot(int s, int elbT0, const uint8_t* sNaN) {
    const int Ns = cfg.Ns, ET = std::max(cfg.elbTmax, 1);
    const int T = hT[s];
    require(elbT0 >= 0, "elbT0 must be >= 0");
    const int elbT = std::max(0, T - elbT0);
    require(elbT <= cfg.elbTmax, "T - elbT0 exceeds elbTmax");
    std::vector<uint8_t> m((size_t)ET * Ns, 0);
    std::vector<int> cl(ET, 0);
    int nc = 0;
    for (int t = 0; t < elbT; ++t) {
      bool any = false;
      for (int a = 0; a < Ns; ++a) {
        const uint8_t v = sNaN[a + (size_t)Ns * t] ? 1 : 0;  // Ns x elbT column-major
        m[(size_t)t * Ns + a] = v;
        any |= v != 0;
      }
      if (any) cl[nc++] = t;
    }
    hElbT0[s] = elbT0;
    hElbT[s] = elbT;
    hSNaN[s] = m;
    ps_dirty = true;
    HIPCHECK(hipMemcpy(dSNaN.p + (size_t)s * ET * Ns, m.data(), m.size(), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dCens.p + (size_t)s * ET, cl.data(), ET * sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dNcens.p + s, &nc, sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dElbT0.p + s, &elbT0, sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dElbT.p + s, &elbT, sizeof(int), hipMemcpyHostToDevice));
    have_elb_slot[s] = true;
  }

  // PREVdraw.X = X0, PREVdraw.Y = Y0 (mcmcVARshadowrateBlockHybrid.m:310-316)
  void reset_chain_slabs() {
    if (!bh) return;
    std::vector<int> sl(cfg.B);
    HIPCHECK(hipMemcpy(sl.data(), slot.p, cfg.B * sizeof(int), hipMemcpyDeviceToHost));
    const size_t xs = (size_t)d.KP * d.TP, ys = (size_t)d.N * d.TP;
    for (int c = 0; c < cfg.B; ++c) {
      HIPCHECK(hipMemcpyAsync(Xpool.p + (size_t)(cfg.ndata + c) * xs, Xpool.p + (size_t)sl[c] * xs,
                              xs * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
      HIPCHECK(hipMemcpyAsync(Ypool.p + (size_t)(cfg.ndata + c) * ys, Ypool.p + (size_t)sl[c] * ys,
                              ys * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
      if (colx_capable)
        HIPCHECK(hipMemcpyAsync(Dcpool.p + (size_t)(cfg.ndata + c) * dcslab, Dcpool.p + (size_t)sl[c] * dcslab,
                                dcslab * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
      if (lag_capable) {
        const size_t ds = (size_t)drows * ldd;
        HIPCHECK(hipMemcpyAsync(Dpool.p + (size_t)(cfg.ndata + c) * ds, Dpool.p + (size_t)sl[c] * ds,
                                ds * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
      }
    }
    HIPCHECK(hipStreamSynchronize(ctx->stream));
  }

  // default index maps for the sweep-level linear model: X/Y slab = data slot
  void set_slots(const int* sl) {
    const int B = cfg.B, N = cfg.N;
    std::vector<int> xi((size_t)B * N), yi(B);
    for (int c = 0; c < B; ++c) {
      require(sl[c] >= 0 && sl[c] < cfg.ndata, "slot out of range");
      if (bh) {  // CTAsys designs: actual-rate block on the vintage's X, shadow block on the chain's
        yi[c] = cfg.ndata + c;
        for (int j = 0; j < N; ++j)
          xi[(size_t)c * N + j] = hActual[j] ? sl[c] : cfg.ndata + c;
      } else {
        yi[c] = sl[c];
        for (int j = 0; j < N; ++j) xi[(size_t)c * N + j] = sl[c];
      }
    }
    HIPCHECK(hipMemcpyAsync(slot.p, sl, B * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    HIPCHECK(hipMemcpyAsync(xidx.p, xi.data(), xi.size() * sizeof(int), hipMemcpyHostToDevice,
                            ctx->stream));
    build_groups(xi);
    HIPCHECK(hipMemcpyAsync(yidx.p, yi.data(), yi.size() * sizeof(int), hipMemcpyHostToDevice,
                            ctx->stream));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    resid_valid = false;
  }

  // systems of a chain that share one X slab, four per Gram workgroup (ccmm_big.hip)
  void build_groups(const std::vector<int>& xi) {
    const int B = cfg.B, N = cfg.N;
    if (big) {
      std::vector<int4> g;
      for (int c = 0; c < B; ++c) {
        std::vector<bool> done(N, false);
        for (int j = 0; j < N; ++j) {
          if (done[j]) continue;
          int m[4] = {-1, -1, -1, -1}, n = 0;
          for (int q = j; q < N && n < 4; ++q)
            if (!done[q] && xi[(size_t)c * N + q] == xi[(size_t)c * N + j]) {
              m[n++] = c * N + q;
              done[q] = true;
            }
          g.push_back(int4{m[0], m[1], m[2], m[3]});
        }
      }
      nGroups = (int)g.size();
      bigGroups.alloc(g.size());
      HIPCHECK(hipMemcpy(bigGroups.p, g.data(), g.size() * sizeof(int4), hipMemcpyHostToDevice));
    }
  }

  void upload_X(int slab, int T, const double* X) {  // X: T x K column-major
    const int K = d.K, KP = d.KP, TP = d.TP;
    std::vector<double> buf((size_t)KP * TP, 0.0);
    for (int a = 0; a < K; ++a)
      for (int t = 0; t < T; ++t) buf[(size_t)a * TP + t] = X[(size_t)a * T + t];
    HIPCHECK(hipMemcpy(Xpool.p + (size_t)slab * KP * TP, buf.data(), buf.size() * sizeof(double),
                       hipMemcpyHostToDevice));
  }
  void upload_TN(double* dst, int nmat, int T, const double* src, double pad) {
    // nmat matrices of T x N (column-major) -> [m][N][TP]
    const int N = d.N, TP = d.TP;
    std::vector<double> buf((size_t)nmat * N * TP, pad);
    for (int m = 0; m < nmat; ++m)
      for (int i = 0; i < N; ++i)
        for (int t = 0; t < T; ++t)
          buf[((size_t)m * N + i) * TP + t] = src[((size_t)m * N + i) * T + t];
    HIPCHECK(hipMemcpy(dst, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  void download_TN(const double* srcd, int nmat, int T, double* dst) {
    const int N = d.N, TP = d.TP;
    std::vector<double> buf((size_t)nmat * N * TP);
    HIPCHECK(hipMemcpy(buf.data(), srcd, buf.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int m = 0; m < nmat; ++m)
      for (int i = 0; i < N; ++i)
        for (int t = 0; t < T; ++t)
          dst[((size_t)m * N + i) * T + t] = buf[((size_t)m * N + i) * TP + t];
  }
  void upload_KN(double* dst, int nmat, const double* src, double pad) {
    const int N = d.N, K = d.K, KP = d.KP;
    std::vector<double> buf((size_t)nmat * N * KP, pad);
    for (int m = 0; m < nmat; ++m)
      for (int j = 0; j < N; ++j)
        for (int a = 0; a < K; ++a)
          buf[((size_t)m * N + j) * KP + a] = src[((size_t)m * N + j) * K + a];
    HIPCHECK(hipMemcpy(dst, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  void download_KN(const double* srcd, int nmat, double* dst) {
    const int N = d.N, K = d.K, KP = d.KP;
    std::vector<double> buf((size_t)nmat * N * KP);
    HIPCHECK(hipMemcpy(buf.data(), srcd, buf.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int m = 0; m < nmat; ++m)
      for (int j = 0; j < N; ++j)
        for (int a = 0; a < K; ++a)
          dst[((size_t)m * N + j) * K + a] = buf[((size_t)m * N + j) * KP + a];
  }

  void set_slot_prior(int s, const double* iVd, const double* ivb, const double* sP,
                      const double* h0mean, const double* h0vcvsqrt) {
    const int N = d.N;
    upload_KN(iVdiag.p + (size_t)s * N * d.KP, 1, iVd, 1.0);
    upload_KN(iVb.p + (size_t)s * N * d.KP, 1, ivb, 0.0);
    HIPCHECK(hipMemcpy(sPHI.p + (size_t)s * N * N, sP, N * N * sizeof(double), hipMemcpyHostToDevice));
    set_slot_h0(s, h0mean, h0vcvsqrt);
  }
  void set_slot_h0(int s, const double* h0mean, const double* h0vcvsqrt) {
    const int N = d.N;
    std::vector<double> V0(N * N, 0.0);
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        double v = 0;
        for (int k = 0; k < N; ++k) v += h0vcvsqrt[i + k * N] * h0vcvsqrt[j + k * N];
        V0[i + j * N] = v;
      }
    std::vector<double> Vi = host_spd_inverse(V0, N);
    std::vector<double> m(N, 0.0);
    for (int i = 0; i < N; ++i)
      for (int k = 0; k < N; ++k) m[i] += Vi[i + k * N] * h0mean[k];
    HIPCHECK(hipMemcpy(V0inv.p + (size_t)s * N * N, Vi.data(), N * N * sizeof(double),
                       hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(V0invm.p + (size_t)s * N, m.data(), N * sizeof(double), hipMemcpyHostToDevice));
  }
  void set_T(int s, int T) {
    require(T >= 2 && T <= cfg.T, "slot T out of range");
    hT[s] = T;
    HIPCHECK(hipMemcpy(Tslot.p + s, &T, sizeof(int), hipMemcpyHostToDevice));
  }

  // ---------------------------------------------------------- kernel launches
  RngArgs rng_args(const double* dcrn, int64_t stride) const {
    RngArgs ra{};
    ra.crn = dcrn;
    ra.crn_chain_stride = stride;
    ra.seed = cfg.seed;
    ra.sweep = sweep;
    ra.ids = have_ids ? rngIds.p : nullptr;
    for (int i = 0; i < kRngBlocks; ++i) ra.off[i] = crn_off[i];
    return ra;
  }

  void ensure_cta() {
    if (!G.p) {
      G.alloc((size_t)d.nmat * d.KP * d.KP);
      // the fused NT = 18 path (256 < K <= 288, KP = 320) never writes rows / columns past 288:
      // they stay zero for k_cta_solve2's 64-row blocks
      HIPCHECK(hipMemsetAsync(G.p, 0, G.n * sizeof(double), ctx->stream));
    }
    rdiag.alloc((size_t)d.nmat * d.KP);
  }
  static constexpr int kResidMultiMinB = 16;
  void run_resid() {
    ChainState cs = view();
    const int nb = d.N <= 8 ? 8 : (d.N <= 20 ? 20 : 32);
    const size_t lds = (size_t)d.K * nb * sizeof(double);
    launch(KID_RESID, [&] {
      // one pass per design slab (k_resid_multi) once the chains fill the chip; at small B the per-equation
      // kernel's B N TP / 256 workgroups keep the slab loads in flight (0.12 -> ~0.01 ms at B = 1): the same
      // fma order per equation, so E is bit-identical either way
      if (d.N <= 32 && lds <= 64 * 1024 && d.B > kResidMultiMinB) {
        const dim3 g((d.TP + 255) / 256, d.B);
        if (nb == 8) hipLaunchKernelGGL(k_resid_multi<8>, g, dim3(256), lds, ctx->stream, d, Tslot.p, xsel(), cs);
        else if (nb == 20) hipLaunchKernelGGL(k_resid_multi<20>, g, dim3(256), lds, ctx->stream, d, Tslot.p, xsel(), cs);
        else hipLaunchKernelGGL(k_resid_multi<32>, g, dim3(256), lds, ctx->stream, d, Tslot.p, xsel(), cs);
      } else {
        hipLaunchKernelGGL(k_resid, dim3((d.TP + 255) / 256, d.N, d.B), dim3(256), 0, ctx->stream, d,
                           Tslot.p, xsel(), cs);
      }
    });
    resid_valid = true;
  }

  void run_cta(const RngArgs& ra) {
    ensure_cta();
    ChainState cs = view();
    if (!resid_valid) run_resid();
    if (big) {
      run_cta_big(ra, cs);
      return;
    }
    if (lag_active()) {
      run_cta_lag(ra, cs);
      return;
    }
    // generic design (KP <= 256): the register-tiled fused Gram + Cholesky, then the per-chain solve
    const int fnt = d.KP / 16;
    launch(KID_WEIGHTS, [&] {
      hipLaunchKernelGGL(k_cta_weights, dim3((d.TP + 255) / 256, d.N, d.B), dim3(256), 0,
                         ctx->stream, d, Tslot.p, cs, 1);
    });
    const size_t lds = (size_t)std::max(2 * kGcTC * gc_ldz(fnt), (fnt + 1) * 16 * kGcLdp) * sizeof(double);
    launch(KID_GRAMCHOL, [&] {
      switch (fnt) {
#define CASE_GC(NT)                                                                           \
  case NT:                                                                                    \
    HIPCHECK(hipFuncSetAttribute((const void*)k_gram_chol<NT>,                                \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));      \
    hipLaunchKernelGGL(k_gram_chol<NT>, dim3(d.nmat), dim3(512), lds, ctx->stream, d, Tslot.p, \
                       xsel(), cs, iVdiag.p, rdiag.p, gc_mode);                               \
    break;
        CASE_GC(4)
        CASE_GC(8)
        CASE_GC(12)
        CASE_GC(16)
#undef CASE_GC
        default:
          throw ArgError("k_gram_chol: unsupported KP");
      }
    });
    const size_t lds_solve2 =
        (size_t)(d.TP + 2 * d.KP + 64 * kSolveLd + 2 * d.N * d.N) * sizeof(double);
    join_fcst();  // the previous kept sweep's predictive density reads PAI
    launch(KID_SOLVE, [&] {
      if (d.N <= 8)
        hipLaunchKernelGGL(k_cta_solve2<8>, dim3(d.B), dim3(256), lds_solve2, ctx->stream, d,
                           Tslot.p, iVb.p, xsel(), cs, rdiag.p, ra);
      else if (d.N <= 20)
        hipLaunchKernelGGL(k_cta_solve2<20>, dim3(d.B), dim3(256), lds_solve2, ctx->stream, d,
                           Tslot.p, iVb.p, xsel(), cs, rdiag.p, ra);
      else
        hipLaunchKernelGGL(k_cta_solve2<32>, dim3(d.B), dim3(256), lds_solve2, ctx->stream, d,
                           Tslot.p, iVb.p, xsel(), cs, rdiag.p, ra);
    });
  }

  // large-N blocks (N > 32; ccmm_bign.hip)
  void run_astep_big(const RngArgs& ra) {
    const size_t np = (size_t)bign_astep_npad(d);
    bigW.alloc((size_t)d.B * (d.N - 1) * np * np);
    ChainState cs = view();
    launch(KID_ASTEPBIG, [&] {
      HIPCHECK(bign_launch_astep(ctx->stream, d, Tslot.p, cs, ra, cfg.logy2offset, bigW.p));
    });
  }
  void run_sv_big(const RngArgs& ra) {
    bigScr.alloc((size_t)d.B * bign_sv_scratch(d));
    ChainState cs = view();
    launch(KID_SVMIX, [&] {
      hipLaunchKernelGGL(k_sv_mix, dim3((d.N * d.TP + 255) / 256, d.B), dim3(256), 0, ctx->stream,
                         d, Tslot.p, cs, ra);
    });
    launch(KID_SVBIG, [&] {
      HIPCHECK(bign_launch_sv(ctx->stream, d, Tslot.p, V0inv.p, V0invm.p, cs, ra, bigScr.p));
    });
  }
  void run_phi_big(const RngArgs& ra) {
    Zphi.alloc((size_t)d.B * d.N * (d.TP + cfg.dPHI));
    bigScr.alloc((size_t)d.B * bign_sv_scratch(d));  // >= 3 N^2 per chain
    ChainState cs = view();
    launch(KID_PHIGEN, [&] {
      hipLaunchKernelGGL(k_phi_gen, dim3((d.N * (d.TP + cfg.dPHI) + 255) / 256, d.B), dim3(256), 0,
                         ctx->stream, d, Tslot.p, cfg.dPHI, cs, ra);
    });
    launch(KID_PHIBIG, [&] {
      HIPCHECK(bign_launch_phi(ctx->stream, d, Tslot.p, cfg.dPHI, sPHI.p, cs, bigScr.p));
    });
  }

  // CTA for large systems (ccmm_big.hip): weights -> multi-equation MFMA Gram -> per-system
  // blocked Cholesky -> per-chain sequential solve
  int big_mask = env_ablation("CCMM_BIG_MASK", 7);
  void run_cta_big(const RngArgs& ra, const ChainState& cs) {
    Ubuf.alloc((size_t)d.B * d.N * d.TP);
    Dinv.alloc((size_t)d.nmat * d.KP * 64);
    std::unique_lock<std::mutex> lk;
    PhaseLock* L = nullptr;
    if (mfma_lock > 0) {
      L = &phase_lock(ctx->device, mfma_lock);
      lk = std::unique_lock<std::mutex>(L->m);
      if (L->last) HIPCHECK(hipStreamWaitEvent(ctx->stream, L->last, 0));
      if (!mfma_ev) HIPCHECK(hipEventCreateWithFlags(&mfma_ev, hipEventDisableTiming));
    }
    launch(KID_WEIGHTS, [&] {
      hipLaunchKernelGGL(k_cta_weights, dim3((d.TP + 255) / 256, d.N, d.B), dim3(256), 0,
                         ctx->stream, d, Tslot.p, cs, 0);
    });
    launch(KID_GRAMBIG, [&] {
      HIPCHECK(big_launch_cta(ctx->stream, d, Tslot.p, slot.p, iVdiag.p, iVb.p, xsel(), cs, bigGroups.p,
                              nGroups, rdiag.p, ra, Ubuf.p, Dinv.p, 1 & big_mask, colx()));
    });
    launch(KID_CHOLBIG, [&] {
      HIPCHECK(big_launch_cta(ctx->stream, d, Tslot.p, slot.p, iVdiag.p, iVb.p, xsel(), cs, bigGroups.p,
                              nGroups, rdiag.p, ra, Ubuf.p, Dinv.p, 2 & big_mask, colx()));
    });
    if (L) {
      HIPCHECK(hipEventRecord(mfma_ev, ctx->stream));
      L->last = mfma_ev;
      lk.unlock();
    }
    join_fcst();  // the previous kept sweep's predictive density reads PAI
    launch(KID_SOLVEBIG, [&] {
      HIPCHECK(big_launch_cta(ctx->stream, d, Tslot.p, slot.p, iVdiag.p, iVb.p, xsel(), cs, bigGroups.p,
                              nGroups, rdiag.p, ra, Ubuf.p, Dinv.p, 4 & big_mask, colx()));
    });
  }

  // Parity export: the lag path's weighted Gram of every (chain, equation) system at the current
  // state, [c b'; b M] (K x K, without the prior), decoded from the kernel's tile slots
  void export_cta_gram(double* out) {
    require(lag_active(), "ccmm_chains_get_cta_gram: the lag-structured CTA path is not active");
    ensure_cta();
    ChainState cs = view();
    hipLaunchKernelGGL(k_cta_weights, dim3((d.TP + 255) / 256, d.N, d.B), dim3(256), 0, ctx->stream, d,
                       Tslot.p, cs, 1);
    HIPCHECK(hipGetLastError());
    LagSel ls = lagsel();
    ls.mode = 8;
    const size_t lds_g = gl_lds_bytes(lagNT, drows, ldd, d.TP);
    HIPCHECK(lag_launch_gram(lagNT, ctx->stream, lds_g, d, Tslot.p, ls, cs, iVdiag.p));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    const int NT = lagNT, NTILE = gl_ntile(NT), K = d.K, KL = K - 1;
    std::vector<double> o((size_t)gl_out_len(NT));
    for (int mat = 0; mat < d.nmat; ++mat) {
      HIPCHECK(hipMemcpy(o.data(), G.p + (size_t)mat * d.KP * d.KP, o.size() * sizeof(double),
                         hipMemcpyDeviceToHost));
      double* Gm = out + (size_t)mat * K * K;
      Gm[0] = o[(size_t)NTILE * 256];
      for (int a = 0; a < KL; ++a) Gm[1 + a] = Gm[(size_t)(1 + a) * K] = o[(size_t)NTILE * 256 + 1 + a];
      for (int gi = 0; gi < NTILE; ++gi) {
        const int ti = gl_ti(NT, gi), tj = gl_tj(NT, gi);
        for (int r = 0; r < 4; ++r)
          for (int lane = 0; lane < 64; ++lane) {
            const int row = 16 * tj + (lane >> 4) + 4 * r, col = 16 * ti + (lane & 15);  // upper tile (tj, ti)
            if (row < KL && col < KL) {
              const double v = o[(size_t)gi * 256 + 64 * r + lane];
              Gm[(size_t)(1 + row) + (size_t)(1 + col) * K] = v;
              Gm[(size_t)(1 + col) + (size_t)(1 + row) * K] = v;
            }
          }
      }
    }
  }

  // Parity export: the lag path's factor record of every (chain, equation) system at the current
  // state as k_gram_chol_lag writes it (gl_out_len(NT) doubles per system: the factor tiles in
  // slot layout, then [1 / L00, L(1 + a, 0)])
  void export_cta_factor(double* out) {
    require(lag_active(), "ccmm_chains_get_cta_factor: the lag-structured CTA path is not active");
    ensure_cta();
    ChainState cs = view();
    hipLaunchKernelGGL(k_cta_weights, dim3((d.TP + 255) / 256, d.N, d.B), dim3(256), 0, ctx->stream, d,
                       Tslot.p, cs, 1);
    HIPCHECK(hipGetLastError());
    const LagSel ls = lagsel();
    const size_t lds_g = gl_lds_bytes(lagNT, drows, ldd, d.TP);
    HIPCHECK(lag_launch_gram(lagNT, ctx->stream, lds_g, d, Tslot.p, ls, cs, iVdiag.p));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    const size_t n = (size_t)gl_out_len(lagNT);
    for (int mat = 0; mat < d.nmat; ++mat)
      HIPCHECK(hipMemcpy(out + (size_t)mat * n, G.p + (size_t)mat * d.KP * d.KP, n * sizeof(double),
                         hipMemcpyDeviceToHost));
  }

  // k_cta_solve_lag on two workgroups per chain (bit-identical draws; the halves spin on each other's
  // X'v partials): only when all 2B workgroups can be resident at once, so no half waits on a partner
  // that cannot start (auto: also B <= kSolveSplitMaxB, where the split pays)
  int split_resident = -1;
  bool solve_split_ok() {
    const int o = opt[OPT_SOLVE_SPLIT];
    if (o == 0 || (o < 0 && d.B > kSolveSplitMaxB)) return false;
    if (split_resident < 0) {
      const int nmax = d.N <= 8 ? 8 : (d.N <= 20 ? 20 : 32);
      split_resident = lag_solve_resident(lagNT, nmax, sl_lds_bytes(lagNT, drows, ldd, d.TP, nmax), opt[OPT_SOLVE_ASYNC]);
    }
    return 2 * d.B <= split_resident;
  }

  // CTA on the lag structure: sqrt weights -> Gram + Cholesky + inverse -> sequential solve
  void run_cta_lag(const RngArgs& ra, const ChainState& cs) {
    launch(KID_WEIGHTS, [&] {
      hipLaunchKernelGGL(k_cta_weights, dim3((d.TP + 255) / 256, d.N, d.B), dim3(256), 0,
                         ctx->stream, d, Tslot.p, cs, 1);
    });
    const LagSel ls = lagsel();
    const size_t lds_g = gl_lds_bytes(lagNT, drows, ldd, d.TP);
    const int nmax = d.N <= 8 ? 8 : (d.N <= 20 ? 20 : 32);
    const size_t lds_s = sl_lds_bytes(lagNT, drows, ldd, d.TP, nmax);
    std::unique_lock<std::mutex> lk;
    PhaseLock* L = nullptr;
    if (mfma_lock > 0) {  // same phase lock as run_cta_big
      L = &phase_lock(ctx->device, mfma_lock);
      lk = std::unique_lock<std::mutex>(L->m);
      if (L->last) HIPCHECK(hipStreamWaitEvent(ctx->stream, L->last, 0));
      if (!mfma_ev) HIPCHECK(hipEventCreateWithFlags(&mfma_ev, hipEventDisableTiming));
    }
    launch(KID_GRAMLAG, [&] {
      HIPCHECK(lag_launch_gram(lagNT, ctx->stream, lds_g, d, Tslot.p, ls, cs, iVdiag.p));
    });
    if (L) {
      HIPCHECK(hipEventRecord(mfma_ev, ctx->stream));
      L->last = mfma_ev;
      lk.unlock();
    }
    SolveXch xc{nullptr, nullptr, 0};
    if (solve_split_ok()) {
      if (!solveFlag.p) {
        solveXch.alloc((size_t)d.B * 2 * 2 * 256);
        solveFlag.alloc((size_t)d.B * 2);
        HIPCHECK(hipMemsetAsync(solveFlag.p, 0, (size_t)d.B * 2 * sizeof(uint64_t), ctx->stream));
      }
      xc = SolveXch{solveXch.p, (unsigned long long*)solveFlag.p, ++solve_epoch};
    }
    join_fcst();  // the previous kept sweep's predictive density reads PAI
    launch(KID_SOLVELAG, [&] {
      HIPCHECK(lag_launch_solve(lagNT, nmax, opt[OPT_SOLVE_ASYNC], ctx->stream, lds_s, d, Tslot.p, iVb.p, xsel(), ls,
                                cs, ra, xc));
    });
  }

  void run_astep(const RngArgs& ra) {
    if (d.N > kMaxNSmall) {
      run_astep_big(ra);
      return;
    }
    ChainState cs = view();
    const int N = d.N;
    const int total = (N - 1) * N * (N + 1) / 6 + N * (N - 1) / 2 + 8;
    size_t lds = (size_t)(total + N * N) * sizeof(double);
    // stage the chain's residuals in LDS when they fit (N = 20, T = 750: 138 KB in all)
    int es_off = -1;
    const size_t staged = lds + (size_t)N * d.TP * sizeof(double);
    if (staged <= 160 * 1024) {
      es_off = total + N * N;
      lds = staged;
    }
    // k_astep_w (wave-parallel factorisations, the default) or the one-thread-per-regression
    // k_astep (option astep_serial); same draws up to summation order inside the factorisation
    // (identical update order, fma placement as written)
    const bool v1 = opt[OPT_ASTEP_SERIAL] != 0;
    const void* fn = v1 ? (const void*)k_astep : (N <= 20 ? (const void*)k_astep_w<20> : (const void*)k_astep_w<32>);
    if (lds > 64 * 1024) HIPCHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (!astepTab.p) {  // the 4 x 4 Gram tiles (ii, A, B) of astep_gram_tiles, largest ii first
      std::vector<int> tab(1, 0);
      for (int ii = N - 1; ii >= 1; --ii)
        for (int A = 0; 4 * A <= ii; ++A)
          for (int Bk = 0; Bk <= A && 4 * Bk < ii; ++Bk) tab.push_back(ii << 16 | A << 8 | Bk);
      tab[0] = (int)tab.size() - 1;
      astepTab.alloc(tab.size());
      HIPCHECK(hipMemcpy(astepTab.p, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    launch(KID_ASTEP, [&] {
      if (v1)
        hipLaunchKernelGGL(k_astep, dim3(d.B), dim3(256), lds, ctx->stream, d, Tslot.p, cs, ra,
                           cfg.logy2offset, es_off, astepTab.p);
      else if (N <= 20)
        hipLaunchKernelGGL(k_astep_w<20>, dim3(d.B), dim3(512), lds, ctx->stream, d, Tslot.p, cs, ra,
                           cfg.logy2offset, es_off, astepTab.p);
      else
        hipLaunchKernelGGL(k_astep_w<32>, dim3(d.B), dim3(512), lds, ctx->stream, d, Tslot.p, cs, ra,
                           cfg.logy2offset, es_off, astepTab.p);
    });
  }

  // SV scratch of the partitioned sampler (ccmm_svpart.hip): block factors C_t, w_t,
  // separator records, fill vectors g_t; matrices padded to the bucket size NN
  void ensure_sv() {
    const size_t NN = sv_bucket(d.N);
    svLd.alloc((size_t)d.B * (d.TP + 1) * NN * NN);
    svw.alloc((size_t)d.B * (d.TP + 1) * NN);
    svSep.alloc((size_t)d.B * sv_sep_len(d.N));
    svG.alloc((size_t)2 * d.B * (d.TP + 1) * NN);  // fill vectors g | SV normals z
  }

  void run_sv(const RngArgs& ra) {
    if (d.N > kMaxNSmall) {
      run_sv_big(ra);
      return;
    }
    ensure_sv();
    ChainState cs = view();
    launch(KID_SVMIX, [&] {
      hipLaunchKernelGGL(k_sv_mix, dim3((d.N * d.TP + 255) / 256, d.B), dim3(256), 0, ctx->stream,
                         d, Tslot.p, cs, ra);
    });
    launch(KID_SVSAMPLE, [&] {
      HIPCHECK(sv_launch_part(d.N, ctx->stream, d, Tslot.p, V0inv.p, V0invm.p, cs, ra, svSep.p, svG.p, sv_mode,
                                opt[OPT_SV_NWG], opt[OPT_SV_MFMA] != 0));
    });
  }

  void run_phi(const RngArgs& ra, hipStream_t on = nullptr) {
    if (d.N > kMaxNSmall) {
      run_phi_big(ra);
      return;
    }
    hipStream_t st = on ? on : ctx->stream;
    Zphi.alloc((size_t)d.B * d.N * (d.TP + cfg.dPHI));
    ChainState cs = view();
    launch(KID_PHIGEN, [&] {
      hipLaunchKernelGGL(k_phi_gen, dim3((d.N * (d.TP + cfg.dPHI) + 255) / 256, d.B), dim3(256), 0,
                         st, d, Tslot.p, cfg.dPHI, cs, ra);
    }, st);
    size_t lds = (size_t)(4 * d.N * (d.N + 1)) * sizeof(double);
    const size_t staged = lds + (size_t)d.N * (d.TP + 1) * sizeof(double);
    // bit 0: eta staged in LDS; bit 1: then Z in the same region (k_phi)
    const size_t staged_z = lds + (size_t)d.N * std::max(d.TP + 1, d.TP + cfg.dPHI) * sizeof(double);
    const int stage_eta = staged_z <= 160 * 1024 ? 3 : (staged <= 160 * 1024 ? 1 : 0);
    if (stage_eta) {
      lds = (stage_eta & 2) ? staged_z : staged;
      if (lds > 64 * 1024)
        HIPCHECK(hipFuncSetAttribute((const void*)k_phi, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
    }
    launch(KID_PHI, [&] {
      hipLaunchKernelGGL(k_phi, dim3(d.B), dim3(256), lds, st, d, Tslot.p, cfg.dPHI, sPHI.p, cs, stage_eta);
    }, st);
  }

  void run_store() {
    if (cfg.store_capacity <= 0) return;
    if (stored >= cfg.store_capacity) throw ArgError("draw store full: call ccmm_chains_get_draws");
    const size_t B = d.B, N = d.N, K = d.K, cap = cfg.store_capacity;
    sPAI.alloc(B * cap * K * N);
    sPHI_.alloc(B * cap * N * (N + 1) / 2);
    sInvA.alloc(B * cap * N * N);
    sSqrtht.alloc(B * cap * (size_t)cfg.T * N);
    Store st{sPAI.p, sPHI_.p, sInvA.p, sSqrtht.p, cfg.store_capacity, stored, cfg.T};
    ChainState cs = view();
    launch(KID_STORE, [&] {
      hipLaunchKernelGGL(k_store, dim3(64, d.B), dim3(256), 0, ctx->stream, d, cs, st);
    });
    if (bh && cfg.elbTmax > 0) {
      sShadow.alloc(B * cap * cfg.Ns * cfg.elbTmax);
      ElbDev e = elb_view();
      launch(KID_STORE, [&] {
        hipLaunchKernelGGL(k_elb_store, dim3(d.B), dim3(256), 0, ctx->stream, e, cs, sShadow.p,
                           cfg.store_capacity, stored);
      });
      if (keep_first) {  // missingrate_all (mcmcVARshadowrate.m:498)
        sMissing.alloc(B * cap * cfg.Ns * cfg.elbTmax);
        ElbDev e2 = elb_view();
        launch(KID_STORE, [&] {
          hipLaunchKernelGGL(k_ps_first_store, dim3(d.B), dim3(256), 0, ctx->stream,
                             (last_ps && psFirst.p) ? psFirst.p : nullptr, e2.elbT, cs.slot, sMissing.p,
                             cfg.Ns * cfg.elbTmax, cfg.Ns, cfg.store_capacity, stored);
        });
      }
      if (ps_np > 0) {  // stackAccept (:457): ndxAccept of the stored sweep, 0 = none / Gibbs
        sAccept.alloc(B * cap);
        launch(KID_STORE, [&] {
          hipLaunchKernelGGL(k_ps_store, dim3((d.B + 255) / 256), dim3(256), 0, ctx->stream,
                             last_ps ? psFlag.p : nullptr, sAccept.p, d.B, cfg.store_capacity, stored);
        });
      }
    }
    ++stored;
  }

  // ---------------------------------------------------------------- PS branch
  void set_elb_ps(int np, int from_m) {
    require(np >= 0 && np <= (1 << 20), "Nproposals must be in [0, 2^20]");
    const int old = ps_np;
    ps_np = np;
    ps_from_m = np > 0 ? from_m : -1;
    if ((old > 0) != (np > 0) && cfg.elbTmax > 0) {
      const size_t B = cfg.B, ET = std::max(cfg.elbTmax, 1);
      eCond.alloc(B * ET * (size_t)elb_cond_stride(cfg.Ns, cfg.p, np > 0));
    }
    ps_dirty = true;
    layout_crn();
  }
  // band width of the censored-cell precision and the largest cell count over the slots
  void ps_layout() {
    if (!ps_dirty) return;
    const int Ns = cfg.Ns, p = cfg.p, ET = std::max(cfg.elbTmax, 1);
    int wmax = 1, nmax = 1;
    for (int sl = 0; sl < cfg.ndata; ++sl) {
      if (!have_elb_slot[sl]) continue;
      std::vector<int> tcell;  // month of every censored cell, in cell order
      for (int t = 0; t < hElbT[sl]; ++t)
        for (int a = 0; a < Ns; ++a)
          if (hSNaN[sl][(size_t)t * Ns + a]) tcell.push_back(t);
      const int n = (int)tcell.size();
      nmax = std::max(nmax, n);
      int first = 0;  // first cell within p months before the current one
      for (int i = 0; i < n; ++i) {
        while (tcell[first] < tcell[i] - p) ++first;
        wmax = std::max(wmax, i - first + 1);
      }
    }
    require(wmax <= kPsWMax, "PS branch: censored-cell band width exceeds 80 (Ns (p + 1) too large)");
    psW = wmax <= 16 ? 16 : wmax <= 32 ? 32 : wmax <= 48 ? 48 : wmax <= 64 ? 64 : 80;
    ps_nmax = nmax;
    const size_t B = cfg.B;
    eEtPS.alloc(B * ET * cfg.N);
    psL.alloc(B * (size_t)nmax * psW);
    psY.alloc(B * (size_t)nmax);
    psCell.alloc(B * (size_t)nmax);
    psN.alloc(B);
    psFlag.alloc(B);
    HIPCHECK(hipMemset(psFlag.p, 0, B * sizeof(int)));
    if (!psAcc.p) {
      psAcc.alloc(B);
      std::vector<int> big(B, INT_MAX);
      HIPCHECK(hipMemcpy(psAcc.p, big.data(), B * sizeof(int), hipMemcpyHostToDevice));
    }
    if (!psCount.p) {
      psCount.alloc(2 * B);
      HIPCHECK(hipMemset(psCount.p, 0, 2 * B * sizeof(int)));
    }
    ps_dirty = false;
  }
  bool ps_active() const { return ps_np > 0 && ps_from_m > 0 && (int64_t)sweep + 1 >= ps_from_m; }
  PsDev ps_view() const {
    PsDev ps{};
    ps.nmax = ps_nmax;
    ps.W = psW;
    ps.NP = ps_np;
    ps.elb = cfg.elb;
    ps.L = psL.p;
    ps.ybar = psY.p;
    ps.cell = psCell.p;
    ps.n = psN.p;
    ps.acc = psAcc.p;
    ps.flag = psFlag.p;
    ps.count = psCount.p;
    ps.per = cfg.Ns * std::max(cfg.elbTmax, 1);
    ps.first = keep_first ? psFirst.p : nullptr;
    ps.state = psState.p;
    ps.epoch = ps_epoch;
    return ps;
  }
  // missingrate_all (mcmcVARshadowrate.m:435, 498; mcmcVARhybridGibbs.m:486): keep proposal 1 of
  // every PS sweep in the draw store (ccmm_chains_keep_missingrate)
  bool keep_first = false;
  DBuf<double> psFirst, sMissing;
  int last_ps = 0;  // whether the last ELB step ran the PS branch (draw store bookkeeping)

  void run_ps(const RngArgs& ra, ElbDev& e, bool kept) {
    ChainState cs = view();
    if (keep_first) psFirst.alloc((size_t)d.B * cfg.Ns * std::max(cfg.elbTmax, 1));
    const PsDev ps = ps_view();
    // option ps_chol_lds: the first-generation k_ps_chol (LDS window) for every band width (same factor)
    if (psW <= 64 && !opt[OPT_PS_CHOL_LDS]) {  // register-window factorisation, one wave per chain (k_ps_chol_w)
      const size_t lds = ps_chol_w_lds_bytes(psW, std::max(cfg.elbTmax, 1), ps_nmax);
      require(lds <= 160 * 1024, "PS branch: cell list does not fit LDS");
      launch(KID_PSCHOL, [&] {
        switch (psW) {
#define CASE_PSC(W)                                                                                              \
  case W:                                                                                                        \
    HIPCHECK(hipFuncSetAttribute((const void*)k_ps_chol_w<W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    hipLaunchKernelGGL(k_ps_chol_w<W>, dim3(d.B), dim3(64), lds, ctx->stream, d, e, ps, cs);                  \
    break;
          CASE_PSC(16)
          CASE_PSC(32)
          CASE_PSC(48)
          CASE_PSC(64)
#undef CASE_PSC
          default:
            throw ArgError("PS band width");
        }
      });
    } else {
      const size_t lds = (size_t)(psW * psW + 2 * psW) * sizeof(double) + (size_t)ps_nmax * sizeof(int);
      require(lds <= 160 * 1024, "PS branch: cell list does not fit LDS");
      launch(KID_PSCHOL, [&] {
        HIPCHECK(hipFuncSetAttribute((const void*)k_ps_chol, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k_ps_chol, dim3(d.B), dim3(128), lds, ctx->stream, d, e, ps, cs);
      });
    }
    if (ps.first) {  // proposal 1's uncensored cells are the window's data (the chain's current Y)
      HIPCHECK(hipMemcpyAsync(psFirst.p, e.Scur, (size_t)d.B * ps.per * sizeof(double), hipMemcpyDeviceToDevice,
                              ctx->stream));
    }
    launch(KID_PSPROP, [&] {
      const dim3 g((ps_np + 255) / 256, d.B);
      switch (psW) {
#define CASE_PSW(W)                                                                                   \
  case W:                                                                                             \
    hipLaunchKernelGGL(k_ps_prop<W>, g, dim3(256), 0, ctx->stream, e, ps, ra);                        \
    hipLaunchKernelGGL(k_ps_apply<W>, dim3(d.B), dim3(64), (size_t)ps_nmax * sizeof(double), ctx->stream, e, \
                       ps, ra, kept ? 1 : 0);                                                           \
    break;
        CASE_PSW(16)
        CASE_PSW(32)
        CASE_PSW(48)
        CASE_PSW(64)
        CASE_PSW(80)
#undef CASE_PSW
        default:
          throw ArgError("PS band width");
      }
    });
    e.psFlag = psFlag.p;
  }

  void run_elb(const RngArgs& ra, bool kept) {
    if (cfg.elbTmax <= 0) return;
    ChainState cs = view();
    ElbDev e = elb_view();
    const bool ps = ps_active();
    last_ps = ps ? 1 : 0;
    if (ps) {
      ps_layout();
      e = elb_view();
      e.ps = 1;
    }
    const int N = d.N, p = cfg.p, Ns = cfg.Ns, Np = N * p;
    // Φ staged in LDS when it fits (N = 20, p = 12: 40 KB); N = 120 reads it from e.Phi
    // and Yb - yhat, Yb too (2 elbTmax N doubles: 52 KB at elbT = 165) when they fit beside it
    size_t lds_prep = (size_t)(2 + Np + N * (Np + 1)) * sizeof(double);
    int phi_lds = lds_prep <= 160 * 1024 ? 1 : 0;
    if (!phi_lds) lds_prep = (size_t)(2 + Np) * sizeof(double);
    const size_t lds_zy = lds_prep + (size_t)2 * cfg.elbTmax * N * sizeof(double);
    if (phi_lds && lds_zy <= 160 * 1024) {
      phi_lds |= 2;
      lds_prep = lds_zy;
    }
    // small batches: the window's residual rows over several workgroups per chain (Yb / Z in LDS)
    int prep_rows = 0, prep_wg = 1;
    if ((phi_lds & 2) && d.B < 128) {
      const int per = std::max(1, 256 / d.B);
      prep_rows = std::max(16, (cfg.elbTmax + per - 1) / per);
      prep_wg = (cfg.elbTmax + prep_rows - 1) / prep_rows;
    }
    launch(KID_ELBPREP, [&] {
      HIPCHECK(hipFuncSetAttribute((const void*)k_elb_prep, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds_prep));
      hipLaunchKernelGGL(k_elb_prep, dim3(d.B, prep_wg), dim3(kElbPrepThreads), lds_prep, ctx->stream, d, e, xsel(),
                         cs, phi_lds, prep_rows);
    });
    // W_k of kb lags at once (all p + 1 when they fit beside the rest; k_elb_cond)
    const size_t lds_cond0 =
        (size_t)((p + 1) * Ns * N + (1 + 2 * p * Ns) * Ns + 2 * Ns * Ns + N * p * Ns) * sizeof(double);
    int kb_cond = p + 1;
    while (kb_cond > 1 && lds_cond0 + (size_t)kb_cond * N * Ns * sizeof(double) > 96 * 1024) --kb_cond;
    size_t lds_cond = lds_cond0 + (size_t)kb_cond * N * Ns * sizeof(double);
    const int a_lds = (lds_cond + (size_t)N * N * sizeof(double) <= 64 * 1024) ? 1 : 0;
    if (a_lds) lds_cond += (size_t)N * N * sizeof(double);
    // two waves per censored month (BH N = 20: k_elb_cond 1.30 -> 1.13 ms at B = 256); four when the
    // month's staging fills a CU's LDS (N > 64)
    const int nth_cond = (N > 64) ? 256 : 128;
    launch(KID_ELBCOND, [&] {
      switch (Ns) {
#define CASE_NSC(NS)                                                                                 \
  case NS:                                                                                           \
    HIPCHECK(hipFuncSetAttribute((const void*)k_elb_cond<NS>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                 (int)lds_cond));                                                    \
    hipLaunchKernelGGL(k_elb_cond<NS>, dim3(e.elbTmax, d.B), dim3(nth_cond), lds_cond, ctx->stream, d, e, cs, a_lds, \
                       kb_cond);                                                                        \
    break;
        CASE_NSC(1)
        CASE_NSC(2)
        CASE_NSC(3)
        CASE_NSC(4)
        CASE_NSC(5)
#undef CASE_NSC
        default:
          throw ArgError("Ns must be in [1, 5]");
      }
    });
    // Gibbs passes: elb_waves passes in flight (k_elb_gibbs_wf, bit-identical draws), or the
    // one-wave sequential kernel (option elb_waves = 1)
    auto gibbs_lds = [&](int w) {  // shadow rates | per pass: uniforms and their elb_ppnd16 | month tables
      return w == 1 ? (size_t)3 * e.elbTmax * Ns * sizeof(double) + (size_t)e.elbTmax * sizeof(int)
                    : (size_t)(1 + 2 * w) * e.elbTmax * Ns * sizeof(double) + (size_t)2 * e.elbTmax * sizeof(int) +
                          (size_t)(2 * w + 1) * sizeof(int);
    };
    int W = opt[OPT_ELB_WAVES] <= 1 ? 1 : (opt[OPT_ELB_WAVES] < 8 ? 4 : 8);
    while (W > 1 && gibbs_lds(W) > 160 * 1024) W = (W == 8) ? 4 : 1;  // long ELB windows
    const size_t lds_gibbs = gibbs_lds(W);
    // eight passes in flight inside one wave (k_elb_gibbs_oct, bit-identical draws): the default;
    // option elb_oct = 0 selects the wave kernels
    const size_t lds_oct = (size_t)e.elbTmax * Ns * sizeof(double) + (size_t)2 * e.elbTmax * sizeof(int);
    // (the per-chain wave kernels keep shorter months at B < kElbOctMinB: one wave per chain cannot
    // fill the chip there, and a month costs the octet kernel more latency)
    const int elb_oct = opt[OPT_ELB_OCT];
    const bool use_oct = elb_oct && lds_oct <= 160 * 1024 && (elb_oct == 2 || d.B >= kElbOctMinB);
    // speculative Gibbs step (option elb_spec, small B): the asynchronous wave kernels start beside the PS
    // branch on a stream of their own and stop once it accepts; the draw is kept only for a rejected PS
    // (the reference's order and draws: PS first, the Gibbs draw the fallback, :438-466)
    const bool spec = ps && opt[OPT_ELB_SPEC] && d.B <= kElbMpMaxB && !use_oct && W > 1 && opt[OPT_ELB_ASYNC] &&
                      elb_flags == nullptr;
    hipStream_t gst = ctx->stream;
    if (spec) {
      if (!aux2) {
        HIPCHECK(hipStreamCreateWithFlags(&aux2, hipStreamNonBlocking));
        HIPCHECK(hipEventCreateWithFlags(&evSpec, hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&evSpecJoin, hipEventDisableTiming));
      }
      if (!psState.p) {
        psState.alloc(d.B);
        HIPCHECK(hipMemsetAsync(psState.p, 0, d.B * sizeof(unsigned long long), ctx->stream));
      }
      HIPCHECK(hipEventRecord(evSpec, ctx->stream));
      HIPCHECK(hipStreamWaitEvent(aux2, evSpec, 0));
      gst = aux2;
      eScurSpec.alloc(eScur.n);
      e.spec = 1;
      e.psState = psState.p;
      e.psEpoch = ++ps_epoch;
      e.ScurSpec = eScurSpec.p;
    } else if (ps) {
      run_ps(ra, e, kept);
    }
    if (use_oct) {
      launch(KID_ELBGIBBS, [&] {
        switch (Ns) {
#define CASE_NSO(NS)                                                                                           \
  case NS:                                                                                                     \
    HIPCHECK(hipFuncSetAttribute((const void*)k_elb_gibbs_oct<NS>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                 (int)lds_oct));                                                               \
    hipLaunchKernelGGL(k_elb_gibbs_oct<NS>, dim3(d.B), dim3(64), lds_oct, gst, d, e, cs, ra);                   \
    break;
          CASE_NSO(1)
          CASE_NSO(2)
          CASE_NSO(3)
          CASE_NSO(4)
          CASE_NSO(5)
#undef CASE_NSO
          default:
            throw ArgError("Ns must be in [1, 5]");
        }
      }, gst);
    } else if (elb_parts(W) > 1) {
      // the wavefront over 2 or 4 CUs per chain (k_elb_gibbs_mp, bit-identical draws)
      const int parts = elb_parts(W), wpc = 8 / parts;
      elbXch.alloc((size_t)d.B * parts * e.elbTmax * Ns * 2);
      if (elbXchZeroed != elbXch.p) {  // tags start at zero (tags of a launch are >= 2^16)
        HIPCHECK(hipMemsetAsync(elbXch.p, 0, elbXch.n * sizeof(double), ctx->stream));
        elbXchZeroed = elbXch.p;
      }
      const ElbXch xc{elbXch.p, ++elb_epoch};
      const size_t lds_mp = (size_t)(1 + 2 * wpc) * e.elbTmax * Ns * sizeof(double) +
                            (size_t)2 * e.elbTmax * sizeof(int) + (size_t)(wpc + 2) * sizeof(int);
      launch(KID_ELBGIBBS, [&] {
#define GIBBS_MP(NS, WPC_, PT)                                                                                  \
  do {                                                                                                        \
    HIPCHECK(hipFuncSetAttribute((const void*)k_elb_gibbs_mp<NS, WPC_, PT>,                                   \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_mp));                   \
    hipLaunchKernelGGL((k_elb_gibbs_mp<NS, WPC_, PT>), dim3(d.B, PT), dim3(64 * (WPC_ + 2)), lds_mp, gst,       \
                       d, e, cs, ra, xc);                                                                     \
  } while (0)
#define CASE_MP(NS)                    \
  case NS:                             \
    if (parts == 2)                    \
      GIBBS_MP(NS, 4, 2);              \
    else                               \
      GIBBS_MP(NS, 2, 4);              \
    break;
        switch (Ns) {
          CASE_MP(1)
          CASE_MP(2)
          CASE_MP(3)
          CASE_MP(4)
          CASE_MP(5)
          default:
            throw ArgError("Ns must be in [1, 5]");
        }
#undef CASE_MP
#undef GIBBS_MP
      }, gst);
    } else
    launch(KID_ELBGIBBS, [&] {
#define GIBBS_KA(NS, WW, AS)                                                                                \
  do {                                                                                                      \
    HIPCHECK(hipFuncSetAttribute((const void*)k_elb_gibbs_wf<NS, WW, AS>,                                   \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_gibbs));              \
    hipLaunchKernelGGL((k_elb_gibbs_wf<NS, WW, AS>), dim3(d.B), dim3(64 * WW), lds_gibbs, gst, d, e,         \
                       cs, ra);                                                                             \
  } while (0)
#define GIBBS_K(NS, WW)            \
  do {                             \
    if (opt[OPT_ELB_ASYNC])        \
      GIBBS_KA(NS, WW, true);      \
    else                           \
      GIBBS_KA(NS, WW, false);     \
  } while (0)
#define CASE_NS(NS)                                                                            \
  case NS:                                                                                     \
    if (W == 1) {                                                                              \
      HIPCHECK(hipFuncSetAttribute((const void*)k_elb_gibbs<NS>,                               \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_gibbs)); \
      hipLaunchKernelGGL(k_elb_gibbs<NS>, dim3(d.B), dim3(64), lds_gibbs, gst, d, e, cs, ra);         \
    } else if (W == 4) {                                                                       \
      GIBBS_K(NS, 4);                                                                          \
    } else {                                                                                   \
      GIBBS_K(NS, 8);                                                                          \
    }                                                                                          \
    break;
      switch (Ns) {
        CASE_NS(1)
        CASE_NS(2)
        CASE_NS(3)
        CASE_NS(4)
        CASE_NS(5)
        default:
          throw ArgError("Ns must be in [1, 5]");
      }
#undef CASE_NS
#undef GIBBS_K
#undef GIBBS_KA
    }, gst);
    if (spec) {  // the PS branch beside the Gibbs passes; k_ps_apply posts the decision they wait on
      ElbDev ep = e;
      ep.spec = 0;
      run_ps(ra, ep, kept);
      HIPCHECK(hipEventRecord(evSpecJoin, aux2));
      HIPCHECK(hipStreamWaitEvent(ctx->stream, evSpecJoin, 0));
      ep.spec = 1;  // (ep.psFlag: set by run_ps)
      hipLaunchKernelGGL(k_elb_spec_select, dim3(d.B), dim3(256), 0, ctx->stream, ep, slot.p, d.B);
      HIPCHECK(hipGetLastError());
    }
    const int nrb = e.elbTmax * Ns * (p + 1);
    launch(KID_ELBREBUILD, [&] {
      hipLaunchKernelGGL(k_elb_rebuild, dim3((nrb + 255) / 256, d.B), dim3(256), 0, ctx->stream, d, e,
                         xsel(), cs, cfg.ndata, lag_capable ? Dpool.p : nullptr, ldd, drows,
                         colx_capable ? Dcpool.p : nullptr, dcld, (long long)dcslab);
    });
    resid_valid = false;  // X, Y changed: RESID is recomputed before the next CTA
  }

  // workgroups (CUs) per chain of the ELB wavefront: k_elb_gibbs_mp spreads the W = 8 passes in flight
  // over 2 (or 4) CUs at small B, one drawing wave per SIMD, when every chain's parts can be resident
  // together (option elb_parts; auto: 2 for B <= kElbMpMaxB)
  DBuf<double> elbXch;
  hipStream_t aux2 = nullptr;  // the speculative Gibbs step's stream
  hipEvent_t evSpec = nullptr, evSpecJoin = nullptr;
  DBuf<unsigned long long> psState;  // PS decision per chain: ps_epoch << 1 | accepted (k_ps_apply)
  DBuf<double> eScurSpec;            // the speculative Gibbs draw (k_elb_spec_select)
  unsigned long long ps_epoch = 0;
  const double* elbXchZeroed = nullptr;
  unsigned long long elb_epoch = 0;
  int elb_parts(int W) {
    const int o = opt[OPT_ELB_PARTS];
    if (W != 8 || !opt[OPT_ELB_ASYNC] || o == 1 || cfg.elb_gibbsburn + 1 >= 65535) return 1;
    const int parts = o == 0 ? (d.B <= kElbMpMaxB ? 2 : 1) : (o >= 4 ? 4 : 2);
    if (parts == 1) return 1;
    int cus = 0;
    HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    // one workgroup of <= 384 threads per part, <= 110 KB of LDS: at least one per CU is resident
    return (d.B * parts <= cus) ? parts : 1;
  }

  void set_fcst(int H, int Nd, const uint8_t* ndxYields, int keep) {
    const int N = cfg.N, p = cfg.p;
    require(cfg.p >= 1 && (cfg.K == N * p + 1 || (hybrid && cfg.K == N * p + 1 + cfg.Ns * p)),
            "predictive density needs K = N*p + 1 (hybrid: + Ns*p)");
    require(!hybrid || cfg.Ns <= kElbNsMax, "hybrid predictive density: Ns <= 5");
    require(N <= kFcstMaxN, "predictive density supports N <= 32");
    require(H >= 1 && Nd >= 1, "H and Nd must be >= 1");
    require(cfg.store_capacity > 0, "predictive density needs store_capacity > 0 (one record per kept draw)");
    int nwx = 0;
    for (int i = 0; i < N; ++i) nwx += ndxYields[i] ? 0 : 1;
    require(nwx > 0 && nwx < N, "need at least one macro series and one yield");
    if (bh && !hybrid)
      for (int i = 0; i < N; ++i)
        require(!(hActual[i] && ndxYields[i]), "a yield cannot be in the actual-rate block");
    if (hybrid)
      for (int a = 0; a < cfg.Ns; ++a)
        require(ndxYields[hNdxS[a]], "the shadow-rate variables must be yields (ndxYIELDS)");
    fH = H;
    fNd = Nd;
    fKeep = keep ? 1 : 0;
    fldXj = cfg.K + N * p;
    const size_t B = cfg.B, HN = (size_t)H * N, cap = cfg.store_capacity;
    fYields.alloc(N);
    HIPCHECK(hipMemcpy(fYields.p, ndxYields, N, hipMemcpyHostToDevice));
    fYreal.alloc((size_t)cfg.ndata * N);
    std::vector<double> nan((size_t)cfg.ndata * N, std::nan(""));
    HIPCHECK(hipMemcpy(fYreal.p, nan.data(), nan.size() * sizeof(double), hipMemcpyHostToDevice));
    have_fcst_slot.assign(cfg.ndata, false);
    fXj.alloc(B * fldXj);
    fY.alloc(B * Nd * HN);
    fYc.alloc(B * Nd * HN);
    fYhat.alloc(B * HN);
    fSc.alloc(B * Nd * 4);
    fStatus.alloc(B);
    fYsum.alloc(B * HN);
    fYcsum.alloc(B * HN);
    fYhatsum.alloc(B * HN);
    fScStore.alloc(B * cap * Nd * 4);
    if (fKeep) {
      fPaths.alloc(B * cap * Nd * HN);
      fPathsC.alloc(B * cap * Nd * HN);
    }
    require(fcst_paths_lds_doubles(N, cfg.K, p, fcst_chunk(N, cfg.K, p, H)) * sizeof(double) <= 160 * 1024,
            "forecast state does not fit LDS");
    fSv1.alloc(B * Nd * N);
    have_fcst = true;
    reset_fcst();
    layout_crn();
  }
  void reset_fcst() {
    const size_t HN = (size_t)fH * cfg.N, B = cfg.B;
    HIPCHECK(hipMemsetAsync(fYsum.p, 0, B * HN * sizeof(double), ctx->stream));
    HIPCHECK(hipMemsetAsync(fYcsum.p, 0, B * HN * sizeof(double), ctx->stream));
    HIPCHECK(hipMemsetAsync(fYhatsum.p, 0, B * HN * sizeof(double), ctx->stream));
    HIPCHECK(hipMemsetAsync(fStatus.p, 0, B * sizeof(int), ctx->stream));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    fstored = 0;
  }

  // ---------------------------------------------------------------- post-processing
  // summaries over the kept draws of the chains of one data slot (ccmm_post.hip)
  DBuf<double> postA, postB, postOut;
  DBuf<char> postWs;
  DBuf<int> postRows;
  DBuf<uint8_t> postCum, postFlo;
  void summaries(int source, int sl, const uint8_t* rows, const uint8_t* cumcode, const uint8_t* flo, double fl,
                 const double* realized, int nq, const double* pct, double* mean, double* median, double* quant,
                 double* sdev, double* crps) {
    require(sl >= 0 && sl < cfg.ndata, "slot out of range");
    require(nq >= 0 && (nq == 0 || pct), "bad quantile list");
    std::vector<int> hs(cfg.B);
    HIPCHECK(hipMemcpy(hs.data(), slot.p, cfg.B * sizeof(int), hipMemcpyDeviceToHost));
    int c0 = -1, C = 0;
    for (int c = 0; c < cfg.B; ++c)
      if (hs[c] == sl) {
        if (c0 < 0) c0 = c;
        require(c == c0 + C, "the chains of the slot must be contiguous");
        ++C;
      }
    require(C > 0, "no chain bound to the slot");
    const int N = cfg.N, K = cfg.K;
    int S = 0, n = 0;
    if (source == 0 || source == 1) {
      require(have_fcst && fKeep, "forecast paths were not kept (ccmm_chains_set_fcst keep_paths)");
      require(fstored > 0, "no forecast records");
      std::vector<int> rl;
      for (int i = 0; i < N; ++i)
        if (!rows || rows[i]) rl.push_back(i);
      require(!rl.empty(), "no rows selected");
      S = (int)rl.size() * fH;
      n = C * fstored * fNd;
      postRows.alloc(rl.size());
      HIPCHECK(hipMemcpy(postRows.p, rl.data(), rl.size() * sizeof(int), hipMemcpyHostToDevice));
      if (cumcode) {
        postCum.alloc(N);
        HIPCHECK(hipMemcpy(postCum.p, cumcode, N, hipMemcpyHostToDevice));
      }
      if (flo) {
        postFlo.alloc(N);
        HIPCHECK(hipMemcpy(postFlo.p, flo, N, hipMemcpyHostToDevice));
      }
      postA.alloc((size_t)S * n);
      HIPCHECK(post_gather_fcst(ctx->stream, source == 0 ? fPaths.p : fPathsC.p, c0, C, fstored, fNd, fH, N,
                                cfg.store_capacity, postRows.p, (int)rl.size(), cumcode ? postCum.p : nullptr,
                                flo ? postFlo.p : nullptr, fl, postA.p));
    } else if (source == 2) {
      require(stored > 0 && sPAI.p, "no stored draws");
      require(!flo, "a floor applies to forecast paths only");
      S = K * N;
      n = C * stored;
      postA.alloc((size_t)S * n);
      HIPCHECK(post_gather_pai(ctx->stream, sPAI.p, c0, C, stored, cfg.store_capacity, K * N, postA.p));
    } else {
      throw ArgError("source must be 0 (paths), 1 (censored paths) or 2 (PAI draws)");
    }
    postB.alloc((size_t)S * n);
    const size_t wb = post_workspace_bytes(S, n);
    postWs.alloc(wb);
    // device scratch: pct | realized | mean | median | sd | crps | quantiles
    postOut.alloc((size_t)nq + (size_t)S * (5 + nq));
    double* dp = postOut.p;
    double* dr = dp + nq;
    double* dm = dr + S;
    double* dmed = dm + S;
    double* dsd = dmed + S;
    double* dcr = dsd + S;
    double* dq = dcr + S;
    if (nq) HIPCHECK(hipMemcpy(dp, pct, nq * sizeof(double), hipMemcpyHostToDevice));
    if (realized) HIPCHECK(hipMemcpy(dr, realized, S * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(post_summaries(ctx->stream, S, n, postA.p, postB.p, postWs.p, wb, realized ? dr : nullptr, nq, dp,
                            dm, dmed, nq ? dq : nullptr, dsd, crps ? dcr : nullptr));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    auto get = [&](double* dst, const double* src, size_t cnt) {
      if (dst) HIPCHECK(hipMemcpy(dst, src, cnt * sizeof(double), hipMemcpyDeviceToHost));
    };
    get(mean, dm, S);
    get(median, dmed, S);
    get(sdev, dsd, S);
    get(crps, dcr, S);
    get(quant, dq, (size_t)S * nq);
  }

  // the predictive density of a kept sweep on the auxiliary stream (option fcst_overlap, N <= 32): it reads
  // the sweep's PAI, invA, h, sqrtPHI and the chain's Y, which the next sweep first rewrites in its CTA
  // solve (PAI), so it runs beside the next sweep's residual, weights and Gram + Cholesky; join_fcst()
  // orders the solve (and the end of every ccmm_chains_sweep call) after it.  Same kernels, same inputs.
  bool fcst_pending = false;
  hipEvent_t evFcstFork = nullptr, evFcstDone = nullptr;
  void join_fcst() {
    if (!fcst_pending) return;
    HIPCHECK(hipStreamWaitEvent(ctx->stream, evFcstDone, 0));
    fcst_pending = false;
  }

  void run_fcst(const RngArgs& ra) {
    if (fstored >= cfg.store_capacity) throw ArgError("forecast store full: call ccmm_chains_get_fcst");
    hipStream_t fst = ctx->stream;
    // (small B only: with the chip full of the next sweep's Gram + Cholesky the overlap buys nothing)
    const bool overlap = opt[OPT_FCST_OVERLAP] != 0 && d.N <= kMaxNSmall && d.B <= kElbMpMaxB;
    if (overlap) {
      ensure_aux();
      if (!evFcstFork) {
        HIPCHECK(hipEventCreateWithFlags(&evFcstFork, hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&evFcstDone, hipEventDisableTiming));
      }
      HIPCHECK(hipEventRecord(evFcstFork, ctx->stream));
      HIPCHECK(hipStreamWaitEvent(aux, evFcstFork, 0));
      fst = aux;
    }
    static const GLNodes gl = make_gl_nodes();
    const int N = d.N, B = d.B, H = fH, Nd = fNd;
    ChainState cs = view();
    FcstArgs a{};
    a.B = B; a.N = N; a.p = cfg.p; a.H = H; a.Nd = Nd;
    a.bh = hybrid ? 2 : (fcst_bh ? 1 : 0);
    a.K = N * cfg.p + 1;
    a.Kx = cfg.K;
    a.Ns = hybrid ? cfg.Ns : 0;
    a.ndxS = hybrid ? dNdxS.p : nullptr;
    a.PAI = PAI.p; a.ldPAI = d.KP; a.invA = invA.p; a.logSV = h.p; a.ldSV = d.TP;
    a.svT = Tslot.p; a.slot = slot.p; a.sqrtPHI = sqrtPHI.p; a.Xj = fXj.p; a.ldXj = fldXj;
    a.yreal = fYreal.p; a.ldY = N; a.ndxYields = fYields.p; a.actual = fcst_bh ? dActual.p : nullptr;
    a.recFloor = have_rec_floor ? fRecFloor.p : nullptr;
    a.elb = cfg.elb;
    if (ra.crn) {
      a.svz = ra.crn + ra.off[CCMM_RNG_FCST];
      a.z = a.svz + (size_t)N * H * Nd;
      a.crnStride = ra.crn_chain_stride;
    }
    a.seed = cfg.seed; a.sweep = ra.sweep; a.ids = ra.ids;
    a.fY = fY.p; a.fYc = fYc.p; a.yhat = fYhat.p; a.scores = fSc.p; a.status = fStatus.p;
    a.gl = gl;
    a.mode = env_ablation("CCMM_FCST_MODE", 0);  // timing-only: 1 no scores, 2 no horizons
    const XSel xs = xsel();
    launch(KID_FCST, [&] {
      hipLaunchKernelGGL(k_fcst_jumpoff, dim3(B), dim3(256), 0, fst, N, cfg.p, N * cfg.p + 1, d.TP,
                         Tslot.p, slot.p, xs.ypool, xs.yidx, fldXj, fXj.p, hybrid ? cfg.Ns : 0,
                         hybrid ? dNdxS.p : nullptr, cfg.elb);
      launch_fcst(fst, a, fSv1.p, opt[OPT_FCST_REG] != 0);
      hipLaunchKernelGGL(k_fcst_accum, dim3(B), dim3(256), 0, fst, N, H, Nd,
                         cfg.store_capacity, fstored, fY.p, fYc.p, (fcst_bh || hybrid) ? nullptr : fYhat.p, fSc.p,
                         fYsum.p, fYcsum.p, fYhatsum.p, fScStore.p, fKeep ? fPaths.p : nullptr,
                         fKeep ? fPathsC.p : nullptr);
    }, fst);
    (void)cs;
    ++fstored;
    if (overlap) {
      HIPCHECK(hipEventRecord(evFcstDone, aux));
      fcst_pending = true;
    }
  }

  // ---------------------------------------------------------------- QR fallback
  // CTA.m:80-92: a chain whose coefficient block met a non-positive Cholesky pivot
  // (status bit 2) is redrawn on the host (host_cta_chain: Cholesky, or the Householder QR
  // of Kailath's array where it fails) from the same previous draw and normals; status
  // bit 2 is then replaced by bit 1 ("QR fallback used", informational).  Option force_qr routes
  // every chain through the host QR branch (tests); qr_fallback = 0 disables the check.
  DBuf<double> paiPrev, zHost;
  int64_t qr_count = 0;

  void snapshot_pai() {
    if (!opt[OPT_QR_FALLBACK]) return;
    paiPrev.alloc(PAI.n);
    HIPCHECK(hipMemcpyAsync(paiPrev.p, PAI.p, PAI.n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
  }

  // returns the chains redrawn
  int cta_fallback(const RngArgs& ra) {
    if (!opt[OPT_QR_FALLBACK]) return 0;
    const bool force_qr = opt[OPT_FORCE_QR] != 0;
    const int B = d.B, N = d.N, K = d.K, KP = d.KP, TP = d.TP;
    std::vector<int> st(B);
    HIPCHECK(hipMemcpyAsync(st.data(), status.p, B * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    std::vector<int> bad;
    for (int c = 0; c < B; ++c)
      if (force_qr || (st[c] & 2)) bad.push_back(c);
    if (bad.empty()) return 0;
    auto dl = [&](const auto* src, size_t n, auto& dst) {
      dst.resize(n);
      HIPCHECK(hipMemcpy(dst.data(), src, n * sizeof(dst[0]), hipMemcpyDeviceToHost));
    };
    std::vector<int> hslot, hT, hxi, hyi;
    dl(slot.p, (size_t)B, hslot);
    dl(Tslot.p, (size_t)cfg.ndata, hT);
    dl(xidx.p, (size_t)B * N, hxi);
    dl(yidx.p, (size_t)B, hyi);
    zHost.alloc((size_t)K * N);
    // inputs of every flagged chain to the host, the redraws in parallel, PAI back
    struct Job {
      int c, T, fl = 0;
      std::vector<double> Y, A, Ae, sh, ivd, ivb, pai, z;
      std::vector<uint8_t> at;
      std::vector<std::vector<double>> X;
      std::vector<const double*> Xs;
    };
    std::vector<Job> jobs(bad.size());
    for (size_t q = 0; q < bad.size(); ++q) {
      Job& jb = jobs[q];
      const int c = bad[q], s = hslot[c];
      jb.c = c;
      jb.T = hT[s];
      dl(Ypool.p + (size_t)hyi[c] * N * TP, (size_t)N * TP, jb.Y);
      dl(A.p + (size_t)c * N * N, (size_t)N * N, jb.A);
      if (aswitch) {
        dl(AelbD.p + (size_t)c * N * N, (size_t)N * N, jb.Ae);
        dl(atELBD.p + (size_t)c * TP, (size_t)TP, jb.at);
      }
      dl(sqrtht.p + (size_t)c * N * TP, (size_t)N * TP, jb.sh);
      dl(iVdiag.p + (size_t)s * N * KP, (size_t)N * KP, jb.ivd);
      dl(iVb.p + (size_t)s * N * KP, (size_t)N * KP, jb.ivb);
      dl(paiPrev.p + (size_t)c * N * KP, (size_t)N * KP, jb.pai);
      hipLaunchKernelGGL(k_rng_normals, dim3((K * N + 255) / 256), dim3(256), 0, ctx->stream, ra, c,
                         (int)CCMM_RNG_PAI, K * N, zHost.p);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipStreamSynchronize(ctx->stream));
      dl(zHost.p, (size_t)K * N, jb.z);
      jb.X.assign(N, {});
      jb.Xs.assign(N, nullptr);
      for (int j = 0; j < N; ++j) {
        int first = j;  // equations sharing a slab share the download
        for (int r = 0; r < j; ++r)
          if (hxi[(size_t)c * N + r] == hxi[(size_t)c * N + j]) {
            first = r;
            break;
          }
        if (first == j) dl(Xpool.p + (size_t)hxi[(size_t)c * N + j] * KP * TP, (size_t)KP * TP, jb.X[j]);
      }
      for (int j = 0; j < N; ++j) {
        int first = j;
        for (int r = 0; r < j; ++r)
          if (hxi[(size_t)c * N + r] == hxi[(size_t)c * N + j]) {
            first = r;
            break;
          }
        jb.Xs[j] = jb.X[first].data();
      }
    }
    {
      std::atomic<size_t> next{0};
      auto work = [&] {
        for (size_t q; (q = next++) < jobs.size();) {
          Job& jb = jobs[q];
          jb.fl = host_cta_chain(N, K, jb.T, jb.Y.data(), TP, jb.Xs.data(), TP, jb.A.data(), jb.sh.data(), TP,
                                 jb.ivd.data(), jb.ivb.data(), KP, jb.pai.data(), jb.z.data(), force_qr,
                                 aswitch ? jb.Ae.data() : nullptr, aswitch ? jb.at.data() : nullptr);
        }
      };
      const unsigned nth = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16u);
      std::vector<std::thread> th;
      for (unsigned i = 1; i < std::min<size_t>(nth, jobs.size()); ++i) th.emplace_back(work);
      work();
      for (auto& t : th) t.join();
    }
    for (Job& jb : jobs) {
      HIPCHECK(hipMemcpy(PAI.p + (size_t)jb.c * N * KP, jb.pai.data(), (size_t)N * KP * sizeof(double),
                         hipMemcpyHostToDevice));
      st[jb.c] = (st[jb.c] & ~2) | ((jb.fl & 1) ? 1 : 0) | ((jb.fl & 2) ? 2 : 0);
      qr_count += (jb.fl & 1) ? 1 : 0;
    }
    HIPCHECK(hipMemcpy(status.p, st.data(), B * sizeof(int), hipMemcpyHostToDevice));
    run_resid();  // RESID of the redrawn coefficients for the A-step
    return (int)bad.size();
  }

  void sweep_once(const double* dcrn, int64_t stride, bool store) {
    const RngArgs ra = rng_args(dcrn, stride);
    snapshot_pai();
    run_cta(ra);
    cta_fallback(ra);
    run_astep(ra);
    run_sv(ra);
    // block hybrid, N <= 32: the PHI block on the auxiliary stream beside the ELB step (the ELB kernels
    // read PAI, A, invA, sqrtht and the chain's data; PHI reads eta and writes sqrtPHI / PHI / Zphi)
    const bool fork = bh && cfg.elbTmax > 0 && d.N <= kMaxNSmall && opt[OPT_PHI_OVERLAP];
    if (fork) {
      ensure_aux();
      HIPCHECK(hipEventRecord(evFork, ctx->stream));
      HIPCHECK(hipStreamWaitEvent(aux, evFork, 0));
      run_phi(ra, aux);
      HIPCHECK(hipEventRecord(evJoin, aux));
      run_elb(ra, store);
      HIPCHECK(hipStreamWaitEvent(ctx->stream, evJoin, 0));
    } else {
      run_phi(ra);
      if (bh) run_elb(ra, store);
    }
    if (store) run_store();
    if (store && have_fcst) run_fcst(ra);
    ++sweep;
  }

  int check_status() {
    std::vector<int> st(d.B);
    HIPCHECK(hipMemcpy(st.data(), status.p, d.B * sizeof(int), hipMemcpyDeviceToHost));
    int any = 0;
    for (int v : st) any |= v & ~CCMM_STATUS_INFO;  // bits 1, 64: informational (valid draws)
    if (any) {
      HIPCHECK(hipMemset(status.p, 0, d.B * sizeof(int)));
      g_err = "non positive-definite matrix in a Gibbs block (status bits " + std::to_string(any) + ")";
      return CCMM_ERR_NOTSPD;
    }
    return CCMM_OK;
  }
};

namespace ccmm {
// error message of the next ccmm_last_error() on this thread (host modules outside this unit)
void set_last_error(const std::string& msg) { g_err = msg; }
}  // namespace ccmm

// ============================================================== C ABI
// ---------------------------------------------------------------- environment switches
namespace {
// timing-only ablations (results invalid), with the selector bits a default build still honours
struct AblationVar {
  const char* name;
  int keep_mask;
};
const AblationVar kAblationVars[] = {
    {"CCMM_CHOL_SKIP", 0},  {"CCMM_SOLVE_SKIP", 0}, {"CCMM_SV_SKIP", 0},  {"CCMM_GC_MODE", 0},
    {"CCMM_LAG_MODE", 0},   {"CCMM_BIG_MASK", 0},   {"CCMM_ELB_MODE", 0}, {"CCMM_SV_MODE", 0},
    {"CCMM_FCST_MODE", 0},  {"CCMM_POISON", 0},
};
// an ablation variable is "ignored" when it is set and a bit outside its keep_mask is non-zero
bool ablation_ignored(const AblationVar& v) {
#ifdef CCMM_ABLATION
  (void)v;
  return false;
#else
  const char* e = std::getenv(v.name);
  return e && (std::atoi(e) & ~v.keep_mask) != 0;
#endif
}
// an option's variable is "ignored" by a default build whenever it is set
bool option_env_ignored(int i) {
#ifdef CCMM_ABLATION
  (void)i;
  return false;
#else
  return std::getenv(kOptDesc[i].env) != nullptr;
#endif
}
// switches of kernels that no longer exist (round 5 and before): read by no build
const char* const kRetiredVars[] = {"CCMM_OLD_SOLVE", "CCMM_OLD_CHOL", "CCMM_GC18", "CCMM_NO_LAG",
                                    "CCMM_NO_QR_FALLBACK", "CCMM_SOLVE_WAVES"};
std::string ignored_list() {
  std::string out;
  for (const auto& v : kAblationVars)
    if (ablation_ignored(v)) out += (out.empty() ? "" : ",") + std::string(v.name);
  for (const char* r : kRetiredVars)
    if (std::getenv(r)) out += (out.empty() ? "" : ",") + std::string(r);
  for (int i = 0; i < kOptCount; ++i)
    if (option_env_ignored(i)) out += (out.empty() ? "" : ",") + std::string(kOptDesc[i].env);
  return out;
}
}  // namespace

const ccmm::OptDesc ccmm::kOptDesc[ccmm::kOptCount] = {
    {"solve_split", "CCMM_SOLVE_SPLIT", -1, -1, 1},
    {"solve_async", "CCMM_SOLVE_ASYNC", 1, 0, 1},
    {"sv_nwg", "CCMM_SV_NWG", 0, 0, 4},
    {"elb_waves", "CCMM_ELB_WAVES", 8, 1, 8},
    {"elb_oct", "CCMM_ELB_OCT", 1, 0, 2},
    {"elb_async", "CCMM_ELB_ASYNC", 1, 0, 1},
    {"elb_parts", "CCMM_ELB_PARTS", 0, 0, 4},
    {"elb_spec", "CCMM_ELB_SPEC", 0, 0, 1},
    {"fcst_reg", "CCMM_FCST_REG", 1, 0, 1},
    {"fcst_overlap", "CCMM_FCST_OVERLAP", 1, 0, 1},
    {"phi_overlap", "CCMM_PHI_OVERLAP", 1, 0, 1},
    {"qr_fallback", "CCMM_QR_FALLBACK", 1, 0, 1},
    {"big_lagx", "CCMM_BIG_LAGX", 1, 0, 1},
    {"lag", "CCMM_LAG", 1, 0, 1},
    {"large_path", "CCMM_FORCE_BIG", 0, 0, 1},
    {"astep_serial", "CCMM_ASTEP_V1", 0, 0, 1},
    {"ps_chol_lds", "CCMM_PS_CHOL_V1", 0, 0, 1},
    {"sv_mfma", "CCMM_SV_MFMA", 1, 0, 1},
    {"force_qr", "CCMM_FORCE_QR", 0, 0, 1},
    {"girf_generic", "CCMM_GIRF_GENERIC", 0, 0, 1},
};

ccmm::Options::Options() {
  for (int i = 0; i < kOptCount; ++i) {
    v[i] = kOptDesc[i].dflt;
#ifdef CCMM_ABLATION
    if (const char* e = std::getenv(kOptDesc[i].env)) v[i] = std::max(kOptDesc[i].lo, std::min(kOptDesc[i].hi, std::atoi(e)));
#endif
  }
}

int ccmm::option_id(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < kOptCount; ++i)
    if (std::strcmp(name, kOptDesc[i].name) == 0) return i;
  return -1;
}

int ccmm::env_ablation(const char* name, int off, int keep_mask) {
  const char* e = std::getenv(name);
  if (!e) return off;
#ifdef CCMM_ABLATION
  (void)keep_mask;
  return std::atoi(e);
#else
  return (off & ~keep_mask) | (std::atoi(e) & keep_mask);
#endif
}

extern "C" {

int ccmm_abi_version(void) { return CCMM_ABI_VERSION; }
const char* ccmm_last_error(void) { return g_err.c_str(); }

int ccmm_ablation_build(void) {
#ifdef CCMM_ABLATION
  return 1;
#else
  return 0;
#endif
}

int ccmm_env_ignored(char* buf, int len) {
  const std::string l = ignored_list();
  if (buf && len > 0) {
    const size_t n = std::min((size_t)len - 1, l.size());
    std::memcpy(buf, l.data(), n);
    buf[n] = 0;
  }
  int count = l.empty() ? 0 : 1;
  for (char ch : l) count += ch == ',' ? 1 : 0;
  return count;
}

int ccmm_option_count(void) { return kOptCount; }


const char* ccmm_option_name(int i) { return (i >= 0 && i < kOptCount) ? kOptDesc[i].name : nullptr; }

static int set_opt(Options& o, const char* name, int value) {
  const int i = option_id(name);
  if (i < 0) {
    g_err = std::string("unknown option '") + (name ? name : "(null)") + "'";
    return CCMM_ERR_ARG;
  }
  if (value < kOptDesc[i].lo || value > kOptDesc[i].hi) {
    g_err = std::string("option '") + name + "' out of range [" + std::to_string(kOptDesc[i].lo) + ", " +
            std::to_string(kOptDesc[i].hi) + "]";
    return CCMM_ERR_ARG;
  }
  o.v[i] = value;
  return CCMM_OK;
}

static int get_opt(const Options& o, const char* name, int* value) {
  const int i = option_id(name);
  if (i < 0 || !value) {
    g_err = std::string("unknown option '") + (name ? name : "(null)") + "'";
    return CCMM_ERR_ARG;
  }
  *value = o.v[i];
  return CCMM_OK;
}

int ccmm_option_default(const char* name, int* value) {
  const Options o;  // what a new context starts from (a default build: the built-in values)
  return get_opt(o, name, value);
}

int ccmm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

ccmm_ctx* ccmm_create(int device) {
  ccmm_ctx* ctx = nullptr;
  int rc = guarded([&] {
    int n = 0;
    HIPCHECK(hipGetDeviceCount(&n));
    require(device >= 0 && device < n, "device index out of range");
    HIPCHECK(hipSetDevice(device));
    ctx = new ccmm_ctx;
    ctx->device = device;
    // a BLOCKING stream: host uploads use hipMemcpy on the null stream, and a pageable
    // host-to-device copy may return before its DMA has landed; only a stream that
    // synchronises with the null stream orders the kernels after it
    HIPCHECK(hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault));
    return 0;
  });
  if (rc != 0) {
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void ccmm_destroy(ccmm_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int ccmm_set_option(ccmm_ctx* ctx, const char* name, int value) {
  if (!ctx) {
    g_err = "null context";
    return CCMM_ERR_ARG;
  }
  return set_opt(ctx->opt, name, value);
}

int ccmm_get_option(ccmm_ctx* ctx, const char* name, int* value) {
  if (!ctx) {
    g_err = "null context";
    return CCMM_ERR_ARG;
  }
  return get_opt(ctx->opt, name, value);
}

int ccmm_synchronize(ccmm_ctx* ctx) {
  return guarded([&] {
    require(ctx != nullptr, "null context");
    HIPCHECK(hipSetDevice(ctx->device));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    return 0;
  });
}

// ------------------------------------------------------------ block-level drop-ins
static ccmm_chain_config block_cfg(int B, int T, int N, int K) {
  ccmm_chain_config cf{};
  cf.model = CCMM_MODEL_LINEAR;
  cf.N = N;
  cf.p = (K - 1) / (N > 0 ? N : 1);
  cf.K = K;
  cf.T = T;
  cf.B = B;
  cf.ndata = 1;
  cf.dPHI = N + 3;
  cf.rng_crn = 1;
  cf.logy2offset = 1e-3;
  cf.seed = 0;
  return cf;
}

static int cta_impl(ccmm_ctx* ctx, int B, int T, int N, int K, const double* Y, int y_per_chain,
                    const double* X, int nx, int x_per_chain, const double* A, const double* Aelb,
                    const uint8_t* atELB, const double* sqrtht, const double* iVdiag, const double* iVb,
                    double* PAI, const double* z, int* status) {
  return guarded([&] {
    require(ctx && Y && X && A && sqrtht && iVdiag && iVb && PAI, "null argument");
    require(nx == 1 || nx == N, "nx must be 1 (CTA) or N (CTAsys)");
    require((Aelb == nullptr) == (atELB == nullptr), "Aelb and atELB go together");
    HIPCHECK(hipSetDevice(ctx->device));
    ccmm_chains ch;
    ccmm_chain_config cf = block_cfg(B, T, N, K);
    cf.p = 0;  // K free-form for the block call
    const int nX = nx * (x_per_chain ? B : 1), nY = y_per_chain ? B : 1;
    ch.init(ctx, cf, nX, nY);
    if (Aelb) {
      require(!ch.big, "CTAsysAswitching: supported for K <= 256 and N <= 32");
      ch.aswitch = true;
      ch.AelbD.alloc((size_t)B * N * N);
      HIPCHECK(hipMemcpy(ch.AelbD.p, Aelb, (size_t)B * N * N * sizeof(double), hipMemcpyHostToDevice));
      std::vector<uint8_t> at((size_t)B * ch.d.TP, 0);
      for (int c = 0; c < B; ++c)
        for (int t = 0; t < T; ++t) at[(size_t)c * ch.d.TP + t] = atELB[t] ? 1 : 0;
      ch.atELBD.alloc(at.size());
      HIPCHECK(hipMemcpy(ch.atELBD.p, at.data(), at.size(), hipMemcpyHostToDevice));
    }
    for (int q = 0; q < nX; ++q) ch.upload_X(q, T, X + (size_t)q * T * K);
    ch.upload_TN(ch.Ypool.p, nY, T, Y, 0.0);
    std::vector<int> xi((size_t)B * N), yi(B);
    for (int c = 0; c < B; ++c) {
      yi[c] = y_per_chain ? c : 0;
      for (int j = 0; j < N; ++j) xi[(size_t)c * N + j] = (x_per_chain ? c * nx : 0) + (nx == 1 ? 0 : j);
    }
    HIPCHECK(hipMemcpy(ch.xidx.p, xi.data(), xi.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(ch.yidx.p, yi.data(), yi.size() * sizeof(int), hipMemcpyHostToDevice));
    ch.build_groups(xi);
    ch.upload_KN(ch.iVdiag.p, 1, iVdiag, 1.0);
    ch.upload_KN(ch.iVb.p, 1, iVb, 0.0);
    HIPCHECK(hipMemcpy(ch.A.p, A, (size_t)B * N * N * sizeof(double), hipMemcpyHostToDevice));
    ch.upload_TN(ch.sqrtht.p, B, T, sqrtht, 1.0);
    ch.upload_KN(ch.PAI.p, B, PAI, 0.0);
    DBuf<double> dz;
    if (z) {
      dz.alloc((size_t)B * K * N);
      HIPCHECK(hipMemcpy(dz.p, z, dz.n * sizeof(double), hipMemcpyHostToDevice));
    }
    RngArgs ra = ch.rng_args(dz.p, (int64_t)K * N);
    ra.off[CCMM_RNG_PAI] = 0;
    ch.snapshot_pai();
    ch.run_cta(ra);
    ch.cta_fallback(ra);  // CTA.m:80-92 for the chains whose Cholesky failed
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    ch.download_KN(ch.PAI.p, B, PAI);
    std::vector<int> st(B);
    HIPCHECK(hipMemcpy(st.data(), ch.status.p, B * sizeof(int), hipMemcpyDeviceToHost));
    int any = 0;
    for (int c = 0; c < B; ++c) {
      if (status) status[c] = st[c] & 1;
      any |= st[c];
    }
    if (any & ~1) {
      g_err = "posterior precision singular: QR fallback failed";
      return CCMM_ERR_NOTSPD;
    }
    if (any & 1) {
      g_err = "switching to QR routine";  // CTA.m:82
      return CCMM_WARN_QR_FALLBACK;
    }
    return 0;
  });
}

int ccmm_cta(ccmm_ctx* ctx, int B, int T, int N, int K, const double* Y, int y_per_chain,
             const double* X, int nx, int x_per_chain, const double* A, const double* sqrtht,
             const double* iVdiag, const double* iVb, double* PAI, const double* z, int* status) {
  return cta_impl(ctx, B, T, N, K, Y, y_per_chain, X, nx, x_per_chain, A, nullptr, nullptr, sqrtht, iVdiag,
                  iVb, PAI, z, status);
}

int ccmm_cta_aswitching(ccmm_ctx* ctx, int B, int T, int N, int K, const double* Y, int y_per_chain,
                        const double* X, int nx, int x_per_chain, const double* A, const double* Aelb,
                        const uint8_t* atELB, const double* sqrtht, const double* iVdiag, const double* iVb,
                        double* PAI, const double* z, int* status) {
  if (!Aelb || !atELB) {
    g_err = "null argument";
    return CCMM_ERR_ARG;
  }
  return cta_impl(ctx, B, T, N, K, Y, y_per_chain, X, nx, x_per_chain, A, Aelb, atELB, sqrtht, iVdiag, iVb,
                  PAI, z, status);
}

int ccmm_astep(ccmm_ctx* ctx, int B, int T, int N, const double* RESID, const double* sqrtht,
               const double* z, double* A, double* invA) {
  return guarded([&] {
    require(ctx && RESID && sqrtht && A && invA, "null argument");
    HIPCHECK(hipSetDevice(ctx->device));
    ccmm_chains ch;
    ccmm_chain_config cf = block_cfg(B, T, N, 1);
    cf.p = 0;
    ch.init(ctx, cf, 1, 1);
    ch.upload_TN(ch.E.p, B, T, RESID, 0.0);
    ch.upload_TN(ch.sqrtht.p, B, T, sqrtht, 1.0);
    DBuf<double> dz;
    const int64_t nz = (int64_t)N * (N - 1) / 2;
    if (z && nz > 0) {
      dz.alloc((size_t)B * nz);
      HIPCHECK(hipMemcpy(dz.p, z, dz.n * sizeof(double), hipMemcpyHostToDevice));
    }
    RngArgs ra = ch.rng_args(dz.p, nz);
    ra.off[CCMM_RNG_A] = 0;
    ch.run_astep(ra);
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(A, ch.A.p, (size_t)B * N * N * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(invA, ch.invA.p, (size_t)B * N * N * sizeof(double), hipMemcpyDeviceToHost));
    return ch.check_status();
  });
}

int ccmm_sv_ksc(ccmm_ctx* ctx, int B, int T, int N, const double* logy2T, const double* hprevT,
                const double* sqrtPHI, const double* h0mean, const double* h0vcvsqrt,
                const double* u, const double* z, double* hT, double* h0, double* shocksT,
                int8_t* kai2) {
  return guarded([&] {
    require(ctx && logy2T && hprevT && sqrtPHI && h0mean && h0vcvsqrt, "null argument");
    HIPCHECK(hipSetDevice(ctx->device));
    ccmm_chains ch;
    ccmm_chain_config cf = block_cfg(B, T, N, 1);
    cf.p = 0;
    ch.init(ctx, cf, 1, 1);
    // N x T (x B) -> internal [c][i][t]
    std::vector<double> tmp((size_t)B * N * T);
    auto transpose_in = [&](const double* src) {
      for (int c = 0; c < B; ++c)
        for (int t = 0; t < T; ++t)
          for (int i = 0; i < N; ++i)
            tmp[((size_t)c * N + i) * T + t] = src[((size_t)c * T + t) * N + i];
    };
    transpose_in(logy2T);
    ch.upload_TN(ch.logy2.p, B, T, tmp.data(), 0.0);
    transpose_in(hprevT);
    ch.upload_TN(ch.h.p, B, T, tmp.data(), 0.0);
    HIPCHECK(hipMemcpy(ch.sqrtPHI.p, sqrtPHI, (size_t)B * N * N * sizeof(double), hipMemcpyHostToDevice));
    ch.set_slot_h0(0, h0mean, h0vcvsqrt);
    // CRN: u (N x T) and z (N x (T+1)) per chain, packed into one buffer
    DBuf<double> dc;
    const int64_t nu = (int64_t)N * T, nzz = (int64_t)N * (T + 1);
    RngArgs ra = ch.rng_args(nullptr, 0);
    if (u || z) {
      require(u && z, "u and z must both be given or both NULL");
      std::vector<double> buf((size_t)B * (nu + nzz));
      for (int c = 0; c < B; ++c) {
        std::memcpy(&buf[(size_t)c * (nu + nzz)], u + (size_t)c * nu, nu * sizeof(double));
        std::memcpy(&buf[(size_t)c * (nu + nzz) + nu], z + (size_t)c * nzz, nzz * sizeof(double));
      }
      dc.alloc(buf.size());
      HIPCHECK(hipMemcpy(dc.p, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice));
      ra = ch.rng_args(dc.p, nu + nzz);
      ra.off[CCMM_RNG_SVU] = 0;
      ra.off[CCMM_RNG_SVZ] = nu;
    }
    ch.run_sv(ra);
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    auto transpose_out = [&](const double* dsrc, double* dst) {
      ch.download_TN(dsrc, B, T, tmp.data());
      for (int c = 0; c < B; ++c)
        for (int t = 0; t < T; ++t)
          for (int i = 0; i < N; ++i)
            dst[((size_t)c * T + t) * N + i] = tmp[((size_t)c * N + i) * T + t];
    };
    if (hT) transpose_out(ch.h.p, hT);
    if (shocksT) transpose_out(ch.eta.p, shocksT);
    if (h0) {
      // x_0 = h_1 - shock_1
      std::vector<double> hh((size_t)B * N * T), ee((size_t)B * N * T);
      ch.download_TN(ch.h.p, B, T, hh.data());
      ch.download_TN(ch.eta.p, B, T, ee.data());
      for (int c = 0; c < B; ++c)
        for (int i = 0; i < N; ++i)
          h0[(size_t)c * N + i] = hh[((size_t)c * N + i) * T] - ee[((size_t)c * N + i) * T];
    }
    if (kai2) {
      std::vector<int8_t> kk((size_t)B * N * ch.d.TP);
      HIPCHECK(hipMemcpy(kk.data(), ch.kai.p, kk.size(), hipMemcpyDeviceToHost));
      for (int c = 0; c < B; ++c)
        for (int t = 0; t < T; ++t)
          for (int i = 0; i < N; ++i)
            kai2[((size_t)c * T + t) * N + i] = kk[((size_t)c * N + i) * ch.d.TP + t];
    }
    return ch.check_status();
  });
}

int ccmm_phi_iw(ccmm_ctx* ctx, int B, int T, int N, const double* eta, const double* sPHI,
                int dPHI, const double* Zdraw, double* sqrtPHI, double* PHI) {
  return guarded([&] {
    require(ctx && eta && sPHI && sqrtPHI && PHI, "null argument");
    HIPCHECK(hipSetDevice(ctx->device));
    ccmm_chains ch;
    ccmm_chain_config cf = block_cfg(B, T, N, 1);
    cf.p = 0;
    cf.dPHI = dPHI;
    ch.init(ctx, cf, 1, 1);
    ch.upload_TN(ch.eta.p, B, T, eta, 0.0);
    HIPCHECK(hipMemcpy(ch.sPHI.p, sPHI, (size_t)N * N * sizeof(double), hipMemcpyHostToDevice));
    DBuf<double> dz;
    const int64_t nz = (int64_t)N * (T + dPHI);
    if (Zdraw) {
      dz.alloc((size_t)B * nz);
      HIPCHECK(hipMemcpy(dz.p, Zdraw, dz.n * sizeof(double), hipMemcpyHostToDevice));
    }
    RngArgs ra = ch.rng_args(dz.p, nz);
    ra.off[CCMM_RNG_PHI] = 0;
    ch.run_phi(ra);
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(sqrtPHI, ch.sqrtPHI.p, (size_t)B * N * N * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(PHI, ch.PHI.p, (size_t)B * N * N * sizeof(double), hipMemcpyDeviceToHost));
    return ch.check_status();
  });
}

// erfcinv on the host (Giles 2010 single-precision seed + Halley refinement)
static double host_erfcinv(double y) {
  if (y <= 0.0) return INFINITY;
  if (y >= 2.0) return -INFINITY;
  // work with x = erfinv(1 - y) using the symmetric form for accuracy near 0
  const bool upper = y > 1.0;
  const double yy = upper ? 2.0 - y : y;  // yy in (0, 1]
  if (yy < 1e-30) {
    // deep tail: asymptotic seed erfc(x) ~ exp(-x^2)/(x sqrt(pi)), then Newton on log erfc
    const double ly = std::log(yy);
    double x = std::sqrt(-ly);
    for (int it = 0; it < 4; ++it) x = std::sqrt(-ly - std::log(1.7724538509055159 * x));
    for (int it = 0; it < 3; ++it) {
      const double e = std::erfc(x);
      const double f = std::log(e) - ly;
      const double df = -1.1283791670955126 * std::exp(-x * x) / e;
      x -= f / df;
    }
    return upper ? -x : x;
  }
  // seed: Giles' approximation of erfinv(1 - yy)
  double w = -std::log(yy * (2.0 - yy));
  double p;
  if (w < 6.25) {
    w -= 3.125;
    p = -3.6444120640178196996e-21;
    p = -1.685059138182016589e-19 + p * w;
    p = 1.2858480715256400167e-18 + p * w;
    p = 1.115787767802518096e-17 + p * w;
    p = -1.333171662854620906e-16 + p * w;
    p = 2.0972767875968561637e-17 + p * w;
    p = 6.6376381343583238325e-15 + p * w;
    p = -4.0545662729752068639e-14 + p * w;
    p = -8.1519341976054721522e-14 + p * w;
    p = 2.6335093153082322977e-12 + p * w;
    p = -1.2975133253453532498e-11 + p * w;
    p = -5.4154120542946279317e-11 + p * w;
    p = 1.051212273321532285e-09 + p * w;
    p = -4.1126339803469836976e-09 + p * w;
    p = -2.9070369957882005086e-08 + p * w;
    p = 4.2347877827932403518e-07 + p * w;
    p = -1.3654692000834678645e-06 + p * w;
    p = -1.3882523362786468719e-05 + p * w;
    p = 0.0001867342080340571352 + p * w;
    p = -0.00074070253416626697512 + p * w;
    p = -0.0060336708714301490533 + p * w;
    p = 0.24015818242558961693 + p * w;
    p = 1.6536545626831027356 + p * w;
  } else if (w < 16.0) {
    w = std::sqrt(w) - 3.25;
    p = 2.2137376921775787049e-09;
    p = 9.0756561938885390979e-08 + p * w;
    p = -2.7517406297064545428e-07 + p * w;
    p = 1.8239629214389227755e-08 + p * w;
    p = 1.5027403968909827627e-06 + p * w;
    p = -4.013867526981545969e-06 + p * w;
    p = 2.9234449089955446044e-06 + p * w;
    p = 1.2475304481671778723e-05 + p * w;
    p = -4.7318229009055733981e-05 + p * w;
    p = 6.8284851459573175448e-05 + p * w;
    p = 2.4031110387097893999e-05 + p * w;
    p = -0.0003550375203628474796 + p * w;
    p = 0.00095328937973738049703 + p * w;
    p = -0.0016882755560235047313 + p * w;
    p = 0.0024914420961078508066 + p * w;
    p = -0.0037512085075692412107 + p * w;
    p = 0.005370914553590063617 + p * w;
    p = 1.0052589676941592334 + p * w;
    p = 3.0838856104922207635 + p * w;
  } else {
    w = std::sqrt(w) - 5.0;
    p = -2.7109920616438573243e-11;
    p = -2.5556418169965252055e-10 + p * w;
    p = 1.5076572693500548083e-09 + p * w;
    p = -3.7894654401267369937e-09 + p * w;
    p = 7.6157012080783393804e-09 + p * w;
    p = -1.4960026627149240478e-08 + p * w;
    p = 2.9147953450901080826e-08 + p * w;
    p = -6.7711997758452339498e-08 + p * w;
    p = 2.2900482228026654717e-07 + p * w;
    p = -9.9298272942317002539e-07 + p * w;
    p = 4.5260625972231537039e-06 + p * w;
    p = -1.9681778105531670567e-05 + p * w;
    p = 7.5995277030017761139e-05 + p * w;
    p = -0.00021503011930044477347 + p * w;
    p = -0.00013871931833623122026 + p * w;
    p = 1.0103004648645343977 + p * w;
    p = 4.8499064014085844221 + p * w;
  }
  double x = p * (1.0 - yy);  // erfinv(1 - yy) >= 0
  // Halley refinement on erfc(x) = yy
  for (int it = 0; it < 3; ++it) {
    const double f = std::erfc(x) - yy;
    const double dfx = -1.1283791670955126 * std::exp(-x * x);  // d/dx erfc
    const double d2 = -2.0 * x * dfx;
    x -= f / (dfx - 0.5 * f * d2 / dfx);
  }
  return upper ? -x : x;
}

double ccmm_draw_trunc_normal(double mu, double sig, double elb, double u, uint8_t* flags) {
  const double tol = 1e-10;
  const double eps = 2.220446049250313080847e-16;
  sig = std::fabs(sig);
  if (sig > tol) {
    const double ub = (elb - mu) / sig;
    const double PHIbar = 0.5 * std::erfc(-std::sqrt(0.5) * ub);
    double zz;
    if (PHIbar > eps) {
      zz = -std::sqrt(2.0) * host_erfcinv(2.0 * u * PHIbar);
      if (flags) *flags = 3;
    } else {
      zz = ub;
      if (flags) *flags = 1;
    }
    return mu + sig * zz;
  }
  if (flags) *flags = 0;
  return mu;
}

int ccmm_draw_trunc_normal_batch(ccmm_ctx* ctx, int n, const double* mu, const double* sig,
                                 double elb, const double* u, double* out, uint8_t* flags) {
  return guarded([&] {
    require(ctx && mu && sig && u && out && n >= 0, "null argument");
    if (n == 0) return 0;
    HIPCHECK(hipSetDevice(ctx->device));
    DBuf<double> dmu, dsig, du, dout;
    DBuf<uint8_t> dfl;
    dmu.alloc(n);
    dsig.alloc(n);
    du.alloc(n);
    dout.alloc(n);
    dfl.alloc(n);
    HIPCHECK(hipMemcpy(dmu.p, mu, n * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dsig.p, sig, n * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(du.p, u, n * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_truncnorm, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, n, dmu.p,
                       dsig.p, elb, du.p, dout.p, dfl.p);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(out, dout.p, n * sizeof(double), hipMemcpyDeviceToHost));
    if (flags) HIPCHECK(hipMemcpy(flags, dfl.p, n, hipMemcpyDeviceToHost));
    return 0;
  });
}

// ------------------------------------------------------------ sweep-level API
// gibbsdrawShadowrates (b3 = 0) and gibbsdrawShadowratesB3 (b3 = 1; Psi K x Ny x elbT per chain when
// psi3d, else K x Ny) on one chain set holding each call as a data slot
static int gibbs_shadowrates_impl(ccmm_ctx* ctx, int B, int Ny, int elbT, int Ns, int p, const uint8_t* ndxS,
                                  const uint8_t* sNaN, const double* Y, const double* STATE0,
                                  const double* YHAT0, const double* C, const double* Psi, const double* SVol,
                                  double elbBound, int Ndraws, int burnin, const double* u, double* out,
                                  uint8_t* flags, int b3, int psi3d) {
  return guarded([&] {
    require(ctx && ndxS && sNaN && Y && STATE0 && C && Psi && SVol && out, "null argument");
    require(B >= 1 && Ny >= 1 && Ny <= 128 && p >= 1 && elbT >= 1 && burnin >= 0, "bad size");
    require(Ndraws == 1, "Ndraws must be 1 (the value used at mcmcVARshadowrateBlockHybrid.m:436)");
    std::vector<int> nd;
    for (int i = 0; i < Ny; ++i)
      if (ndxS[i]) nd.push_back(i);
    if ((int)nd.size() != Ns) {  // gibbsdrawShadowrates.m:50-52
      g_err = "dimension mismatch";
      return CCMM_ERR_DIM;
    }
    require(Ns >= 1 && Ns <= kElbNsMax, "Ns must be in [1, 5]");
    HIPCHECK(hipSetDevice(ctx->device));
    const int K = Ny * p + 1, T = elbT, passes = burnin + Ndraws;
    ccmm_chain_config cf{};
    cf.model = CCMM_MODEL_BLOCKHYBRID;
    cf.B = B;
    cf.N = Ny;
    cf.p = p;
    cf.T = T;
    cf.K = K;
    cf.ndata = B;  // one data slot per chain: its own Y window and STATE0
    cf.dPHI = Ny + 1;
    cf.logy2offset = 1e-3;
    cf.Ns = Ns;
    cf.elbTmax = T;
    cf.elb_gibbsburn = burnin;
    cf.elb = elbBound;
    cf.rng_crn = u ? 1 : 0;
    cf.seed = 0;
    ccmm_chains ch;
    ch.init(ctx, cf, 2 * B, 2 * B);
    const size_t KK = (size_t)K * K;
    std::vector<double> Xc((size_t)T * K, 0.0), Yc((size_t)T * Ny), ivd((size_t)K * Ny, 1.0),
        ivb((size_t)K * Ny, 0.0), sP((size_t)Ny * Ny, 0.0), h0m(Ny, 0.0), h0v((size_t)Ny * Ny, 0.0);
    for (int i = 0; i < Ny; ++i) sP[i + (size_t)i * Ny] = h0v[i + (size_t)i * Ny] = 1.0;
    std::vector<int> sl(B);
    for (int c = 0; c < B; ++c) {
      // X row 1 = STATE0 (elb.X0 = X(elbT0+1,:)', mcmcVARshadowrateBlockHybrid.m:417), Y = the window
      for (int k = 0; k < K; ++k) Xc[(size_t)k * T] = STATE0[(size_t)c * K + k];
      for (int t = 0; t < T; ++t)
        for (int i = 0; i < Ny; ++i) Yc[t + (size_t)i * T] = Y[((size_t)c * T + t) * Ny + i];
      ch.set_T(c, T);
      ch.upload_X(c, T, Xc.data());
      ch.upload_TN(ch.Ypool.p + (size_t)c * ch.d.N * ch.d.TP, 1, T, Yc.data(), 0.0);
      ch.set_slot_prior(c, ivd.data(), ivb.data(), sP.data(), h0m.data(), h0v.data());
      ch.have_slot[c] = true;
      sl[c] = c;
    }
    ch.set_slots(sl.data());
    std::vector<uint8_t> none(Ny, 0);
    ch.set_elb_model(nd.data(), none.data());
    for (int c = 0; c < B; ++c) ch.set_elb_slot(c, 0, sNaN);
    // state: PAI = C(2:Ny+1, :)' (elb.A rows, :404-407), A = Psi(2:Ny+1, :) \ I, sqrtht = SVol'
    std::vector<double> PAI((size_t)K * Ny * B), A((size_t)Ny * Ny * B, 0.0), sh((size_t)T * Ny * B),
        hh((size_t)T * Ny * B), sq((size_t)Ny * Ny * B, 0.0);
    // A = Psi(2:Ny+1, :) \ I: forward substitution when the impact matrix is lower triangular (every
    // reference caller passes invA, mcmcVARshadowrateBlockHybrid.m:418); otherwise Gauss-Jordan with
    // partial pivoting, and the ELB kernels take the full structural matrix (gibbsdrawShadowrates.m:49-58,
    // 74-95 QR-factor M = Cpowerp Psi diag(SVol) for any Psi: the same conditionals)
    const int nPsi = psi3d ? T : 1;
    bool lower = true;
    for (int c = 0; c < B && lower; ++c)
      for (int m = 0; m < nPsi && lower; ++m) {
        const double* Pc = Psi + ((size_t)c * nPsi + m) * K * Ny;
        for (int col = 1; col < Ny && lower; ++col)
          for (int r = 0; r < col; ++r)
            if (Pc[(1 + r) + (size_t)col * K] != 0.0) {
              lower = false;
              break;
            }
      }
    bool singular = false;
    auto inv_struct = [&](const double* Pc, double* Ac) {
      if (lower) {
        for (int col = 0; col < Ny; ++col)
          for (int r = col; r < Ny; ++r) {
            double v = (r == col) ? 1.0 : 0.0;
            for (int q = col; q < r; ++q) v -= Pc[(1 + r) + (size_t)q * K] * Ac[q + (size_t)col * Ny];
            Ac[r + (size_t)col * Ny] = v / Pc[(1 + r) + (size_t)r * K];
          }
        return;
      }
      std::vector<double> M((size_t)Ny * Ny), I((size_t)Ny * Ny, 0.0);
      for (int col = 0; col < Ny; ++col) {
        I[col + (size_t)col * Ny] = 1.0;
        for (int r = 0; r < Ny; ++r) M[r + (size_t)col * Ny] = Pc[(1 + r) + (size_t)col * K];
      }
      for (int col = 0; col < Ny; ++col) {
        int piv = col;
        for (int r = col + 1; r < Ny; ++r)
          if (std::fabs(M[r + (size_t)col * Ny]) > std::fabs(M[piv + (size_t)col * Ny])) piv = r;
        if (!(std::fabs(M[piv + (size_t)col * Ny]) > 0.0)) {
          singular = true;
          return;
        }
        if (piv != col)
          for (int q = 0; q < Ny; ++q) {
            std::swap(M[col + (size_t)q * Ny], M[piv + (size_t)q * Ny]);
            std::swap(I[col + (size_t)q * Ny], I[piv + (size_t)q * Ny]);
          }
        const double ip = 1.0 / M[col + (size_t)col * Ny];
        for (int q = 0; q < Ny; ++q) {
          M[col + (size_t)q * Ny] *= ip;
          I[col + (size_t)q * Ny] *= ip;
        }
        for (int r = 0; r < Ny; ++r) {
          if (r == col) continue;
          const double f = M[r + (size_t)col * Ny];
          if (f == 0.0) continue;
          for (int q = 0; q < Ny; ++q) {
            M[r + (size_t)q * Ny] -= f * M[col + (size_t)q * Ny];
            I[r + (size_t)q * Ny] -= f * I[col + (size_t)q * Ny];
          }
        }
      }
      std::copy(I.begin(), I.end(), Ac);
    };
    std::vector<double> Am(psi3d ? (size_t)B * T * Ny * Ny : 0, 0.0);
    for (int c = 0; c < B; ++c) {
      const double* Cc = C + (size_t)c * KK;
      const double* Pc = Psi + (size_t)c * nPsi * K * Ny;
      for (int i = 0; i < Ny; ++i)
        for (int k = 0; k < K; ++k) PAI[((size_t)c * Ny + i) * K + k] = Cc[(1 + i) + (size_t)k * K];
      double* Ac = A.data() + (size_t)c * Ny * Ny;
      inv_struct(Pc, Ac);
      for (int m = 0; m < (psi3d ? T : 0); ++m)
        inv_struct(Pc + (size_t)m * K * Ny, Am.data() + ((size_t)c * T + m) * Ny * Ny);
      for (int i = 0; i < Ny; ++i) {
        sq[(size_t)c * Ny * Ny + i + (size_t)i * Ny] = 1.0;
        for (int t = 0; t < T; ++t) {
          const double v = SVol[((size_t)c * T + t) * Ny + i];
          sh[((size_t)c * Ny + i) * T + t] = v;
          hh[((size_t)c * Ny + i) * T + t] = 2.0 * std::log(v);
        }
      }
    }
    if (singular) {
      g_err = std::string(b3 ? "ccmm_gibbs_shadowrates_b3: B" : "ccmm_gibbs_shadowrates: Psi") +
              "(2:Ny+1, :) is singular";
      return CCMM_ERR_ARG;
    }
    ch.elb_Afull = lower ? 0 : 1;
    ch.upload_KN(ch.PAI.p, B, PAI.data(), 0.0);
    HIPCHECK(hipMemcpy(ch.A.p, A.data(), A.size() * sizeof(double), hipMemcpyHostToDevice));
    ch.upload_TN(ch.sqrtht.p, B, T, sh.data(), 1.0);
    ch.upload_TN(ch.h.p, B, T, hh.data(), 0.0);
    HIPCHECK(hipMemcpy(ch.sqrtPHI.p, sq.data(), sq.size() * sizeof(double), hipMemcpyHostToDevice));
    ch.have_elb_model = true;
    ch.reset_chain_slabs();
    // YHAT0 (Ny x elbT per chain, or zeros) -> [B][elbT][Ny]
    DBuf<double> dyh;
    dyh.alloc((size_t)B * T * Ny);
    {
      std::vector<double> yh((size_t)B * T * Ny, 0.0);
      if (YHAT0) std::memcpy(yh.data(), YHAT0, yh.size() * sizeof(double));
      HIPCHECK(hipMemcpy(dyh.p, yh.data(), yh.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    ch.elb_yhat = dyh.p;
    ch.elb_b3 = b3;
    DBuf<double> dAm;
    if (psi3d) {
      dAm.alloc(Am.size());
      HIPCHECK(hipMemcpy(dAm.p, Am.data(), Am.size() * sizeof(double), hipMemcpyHostToDevice));
      ch.elb_Amon = dAm.p;
    }
    DBuf<uint8_t> dfl;
    if (flags) {
      dfl.alloc((size_t)B * passes * T * Ns);
      HIPCHECK(hipMemset(dfl.p, 0, dfl.n));
      ch.elb_flags = dfl.p;
    }
    DBuf<double> du;
    RngArgs ra = ch.rng_args(nullptr, 0);
    if (u) {  // rand(Ns, elbT, burnin + Ndraws) per chain (gibbsdrawShadowrates.m:173)
      du.alloc((size_t)B * Ns * T * passes);
      HIPCHECK(hipMemcpy(du.p, u, du.n * sizeof(double), hipMemcpyHostToDevice));
      ra = ch.rng_args(du.p, (int64_t)Ns * T * passes);
      ra.off[CCMM_RNG_ELB] = 0;
    }
    ch.run_elb(ra, false);
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(out, ch.eScur.p, (size_t)B * Ns * T * sizeof(double), hipMemcpyDeviceToHost));
    if (flags) HIPCHECK(hipMemcpy(flags, dfl.p, dfl.n, hipMemcpyDeviceToHost));
    return 0;
  });
}

int ccmm_gibbs_shadowrates(ccmm_ctx* ctx, int B, int Ny, int elbT, int Ns, int p, const uint8_t* ndxS,
                           const uint8_t* sNaN, const double* Y, const double* STATE0,
                           const double* YHAT0, const double* C, const double* Psi, const double* SVol,
                           double elbBound, int Ndraws, int burnin, const double* u, double* out,
                           uint8_t* flags) {
  return gibbs_shadowrates_impl(ctx, B, Ny, elbT, Ns, p, ndxS, sNaN, Y, STATE0, YHAT0, C, Psi, SVol, elbBound,
                                Ndraws, burnin, u, out, flags, 0, 0);
}

int ccmm_gibbs_shadowrates_b3(ccmm_ctx* ctx, int B, int Ny, int elbT, int Ns, int p, const uint8_t* ndxS,
                              const uint8_t* sNaN, const double* Y, const double* STATE0, const double* A,
                              const double* Bmat, int B3d, const double* SVol, double elbBound, int Ndraws,
                              int burnin, const double* u, double* out, uint8_t* flags) {
  return gibbs_shadowrates_impl(ctx, B, Ny, elbT, Ns, p, ndxS, sNaN, Y, STATE0, nullptr, A, Bmat, SVol,
                                elbBound, Ndraws, burnin, u, out, flags, 1, B3d ? 1 : 0);
}

ccmm_chains* ccmm_chains_create(ccmm_ctx* ctx, const ccmm_chain_config* cfg) {
  ccmm_chains* ch = nullptr;
  int rc = guarded([&] {
    require(ctx && cfg, "null argument");
    require(cfg->model == CCMM_MODEL_LINEAR || cfg->model == CCMM_MODEL_BLOCKHYBRID ||
                cfg->model == CCMM_MODEL_HYBRID || cfg->model == CCMM_MODEL_SHADOWRATE, "unknown model");
    HIPCHECK(hipSetDevice(ctx->device));
    ch = new ccmm_chains;
    const int extra = cfg->model != CCMM_MODEL_LINEAR ? cfg->B : 0;
    ch->init(ctx, *cfg, cfg->ndata + extra, cfg->ndata + extra);
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    const std::string ign = ignored_list();
    if (!ign.empty())  // a warning, not an error: the draws are valid, the switches had no effect
      g_err = "default build: timing-only ablation switches ignored (" + ign + "); build libccmm_ablation.so to use them";
    return 0;
  });
  if (rc != 0) {
    delete ch;
    return nullptr;
  }
  return ch;
}

int ccmm_chains_set_option(ccmm_chains* ch, const char* name, int value) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    const int i = option_id(name);
    const int old = i >= 0 ? ch->opt[i] : 0;
    const int rc = set_opt(ch->opt, name, value);
    if (rc != CCMM_OK) return rc;
    if (i == OPT_LARGE_PATH && value != old) {  // the path's grouping of systems follows the choice
      require(!ch->have_state, "option large_path: set it before ccmm_chains_set_data / set_state");
      HIPCHECK(hipSetDevice(ch->ctx->device));
      ch->big = ch->d.KP > 256 || ch->cfg.N > kMaxNSmall || value != 0;
      ch->init_colx();
      std::vector<int> sl(ch->cfg.B);
      HIPCHECK(hipMemcpy(sl.data(), ch->slot.p, ch->cfg.B * sizeof(int), hipMemcpyDeviceToHost));
      ch->set_slots(sl.data());
    }
    if (i == OPT_SOLVE_SPLIT || i == OPT_SOLVE_ASYNC) ch->split_resident = -1;
    return CCMM_OK;
  });
}

int ccmm_chains_get_option(ccmm_chains* ch, const char* name, int* value) {
  if (!ch) {
    g_err = "null argument";
    return CCMM_ERR_ARG;
  }
  return get_opt(ch->opt, name, value);
}

void ccmm_chains_destroy(ccmm_chains* ch) {
  if (!ch) return;
  (void)hipSetDevice(ch->ctx->device);
  (void)hipStreamSynchronize(ch->ctx->stream);
  delete ch;
}

int ccmm_chains_set_data(ccmm_chains* ch, int slot, int T, const double* Y, const double* X,
                         const double* iVdiag, const double* iVb, const double* sPHI,
                         const double* h0mean, const double* h0vcvsqrt) {
  return guarded([&] {
    require(ch && Y && X && iVdiag && iVb && sPHI && h0mean && h0vcvsqrt, "null argument");
    require(slot >= 0 && slot < ch->cfg.ndata, "slot out of range");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    ch->set_T(slot, T);
    ch->upload_X(slot, T, X);
    ch->try_upload_D(slot, T, Y, X);
    ch->try_upload_Dc(slot, T, X);
    ch->upload_TN(ch->Ypool.p + (size_t)slot * ch->d.N * ch->d.TP, 1, T, Y, 0.0);
    ch->set_slot_prior(slot, iVdiag, iVb, sPHI, h0mean, h0vcvsqrt);
    ch->have_slot[slot] = true;
    ch->resid_valid = false;
    return 0;
  });
}

int ccmm_chains_set_slots(ccmm_chains* ch, const int* slot_of_chain) {
  return guarded([&] {
    require(ch && slot_of_chain, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    ch->set_slots(slot_of_chain);
    return 0;
  });
}

int ccmm_chains_get_kai(ccmm_chains* ch, int8_t* kai) {
  return guarded([&] {
    require(ch && kai, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const int B = ch->d.B, N = ch->d.N, TP = ch->d.TP, T = ch->cfg.T;
    std::vector<int8_t> kk((size_t)B * N * TP);
    HIPCHECK(hipMemcpy(kk.data(), ch->kai.p, kk.size(), hipMemcpyDeviceToHost));
    for (int c = 0; c < B; ++c)
      for (int i = 0; i < N; ++i)
        for (int t = 0; t < T; ++t) kai[t + (size_t)T * (i + (size_t)N * c)] = kk[((size_t)c * N + i) * TP + t];
    return 0;
  });
}

int ccmm_chains_record_elb_flags(ccmm_chains* ch, int enable) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    require(ch->bh, "chain set was not created with CCMM_MODEL_BLOCKHYBRID / CCMM_MODEL_HYBRID");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    if (enable) {
      ch->dElbFlags.alloc((size_t)ch->d.B * (ch->cfg.elb_gibbsburn + 1) * std::max(ch->cfg.elbTmax, 1) *
                          ch->cfg.Ns);
      HIPCHECK(hipMemset(ch->dElbFlags.p, 0, ch->dElbFlags.n));
      ch->elb_flags = ch->dElbFlags.p;
    } else {
      ch->elb_flags = nullptr;
    }
    return 0;
  });
}

int ccmm_chains_get_elb_flags(ccmm_chains* ch, uint8_t* flags) {
  return guarded([&] {
    require(ch && flags, "null argument");
    require(ch->elb_flags != nullptr, "ccmm_chains_record_elb_flags(ch, 1) was not called");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    HIPCHECK(hipMemcpy(flags, ch->dElbFlags.p, ch->dElbFlags.n, hipMemcpyDeviceToHost));
    return 0;
  });
}

int ccmm_chains_set_mfma_lock(ccmm_chains* ch, int id) {
  return guarded([&] {
    require(ch != nullptr && id >= 0, "bad argument");
    require(ch->mfma_ev == nullptr || id == ch->mfma_lock, "MFMA lock id already set");
    ch->mfma_lock = id;
    return 0;
  });
}

int ccmm_chains_set_rng_ids(ccmm_chains* ch, const uint32_t* ids) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    if (!ids) {
      ch->have_ids = false;
      return 0;
    }
    ch->rngIds.alloc(ch->cfg.B);
    HIPCHECK(hipMemcpy(ch->rngIds.p, ids, ch->cfg.B * sizeof(uint32_t), hipMemcpyHostToDevice));
    ch->have_ids = true;
    return 0;
  });
}

int ccmm_chains_get_status(ccmm_chains* ch, int* status) {
  return guarded([&] {
    require(ch && status, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    HIPCHECK(hipMemcpy(status, ch->status.p, ch->cfg.B * sizeof(int), hipMemcpyDeviceToHost));
    int any = 0;
    for (int c = 0; c < ch->cfg.B; ++c) any |= status[c] & ~CCMM_STATUS_INFO;  // bits 1, 64: informational
    return any ? 1 : 0;
  });
}

int ccmm_chains_set_state(ccmm_chains* ch, const double* PAI, const double* A,
                          const double* sqrtht, const double* h, const double* sqrtPHI) {
  return guarded([&] {
    require(ch && PAI && A && sqrtht && h && sqrtPHI, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const int B = ch->d.B, N = ch->d.N, T = ch->cfg.T;
    ch->upload_KN(ch->PAI.p, B, PAI, 0.0);
    HIPCHECK(hipMemcpy(ch->A.p, A, (size_t)B * N * N * sizeof(double), hipMemcpyHostToDevice));
    ch->upload_TN(ch->sqrtht.p, B, T, sqrtht, 1.0);
    ch->upload_TN(ch->h.p, B, T, h, 0.0);
    HIPCHECK(hipMemcpy(ch->sqrtPHI.p, sqrtPHI, (size_t)B * N * N * sizeof(double), hipMemcpyHostToDevice));
    if (ch->bh) {
      if (!ch->have_elb_model) {
        g_err = "ccmm_chains_set_elb_model must be called before set_state";
        return CCMM_ERR_STATE;
      }
      for (int s = 0; s < ch->cfg.ndata; ++s)
        if (!ch->have_slot[s]) {
          g_err = "ccmm_chains_set_data missing for a data slot";
          return CCMM_ERR_STATE;
        }
      ch->reset_chain_slabs();
    }
    ch->sweep = 0;
    ch->stored = 0;
    ch->mom_done = 0;  // the store restarts: the running PAI sums are re-based on reset (pai_moments)
    HIPCHECK(hipMemset(ch->status.p, 0, ch->cfg.B * sizeof(int)));
    if (ch->psCount.p) HIPCHECK(hipMemset(ch->psCount.p, 0, 2 * (size_t)ch->cfg.B * sizeof(int)));
    if (ch->have_fcst) ch->reset_fcst();
    ch->resid_valid = false;
    ch->have_state = true;
    return 0;
  });
}

int ccmm_chains_get_state(ccmm_chains* ch, double* PAI, double* A, double* invA, double* sqrtht,
                          double* h, double* sqrtPHI, double* PHI, double* RESID) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const int B = ch->d.B, N = ch->d.N, T = ch->cfg.T;
    const size_t nn = (size_t)B * N * N * sizeof(double);
    if (PAI) ch->download_KN(ch->PAI.p, B, PAI);
    if (A) HIPCHECK(hipMemcpy(A, ch->A.p, nn, hipMemcpyDeviceToHost));
    if (invA) HIPCHECK(hipMemcpy(invA, ch->invA.p, nn, hipMemcpyDeviceToHost));
    if (sqrtht) ch->download_TN(ch->sqrtht.p, B, T, sqrtht);
    if (h) ch->download_TN(ch->h.p, B, T, h);
    if (sqrtPHI) HIPCHECK(hipMemcpy(sqrtPHI, ch->sqrtPHI.p, nn, hipMemcpyDeviceToHost));
    if (PHI) HIPCHECK(hipMemcpy(PHI, ch->PHI.p, nn, hipMemcpyDeviceToHost));
    if (RESID) ch->download_TN(ch->E.p, B, T, RESID);
    return 0;
  });
}

int64_t ccmm_chains_crn_len(const ccmm_chains* ch) { return ch ? ch->crn_len : -1; }

int ccmm_chains_sweep(ccmm_chains* ch, int nsweeps, const double* crn, int store) {
  return guarded([&] {
    require(ch != nullptr && nsweeps >= 0, "bad argument");
    if (!ch->have_state) {
      g_err = "ccmm_chains_set_state must be called before sweeping";
      return CCMM_ERR_STATE;
    }
    for (int s = 0; s < ch->cfg.ndata; ++s)
      if (!ch->have_slot[s] || (ch->bh && !ch->have_elb_slot[s])) {
        g_err = "ccmm_chains_set_data / set_elb_slot missing for a data slot";
        return CCMM_ERR_STATE;
      }
    if (ch->cfg.rng_crn) require(crn != nullptr, "chain set was created in CRN mode: crn required");
    if (ch->have_fcst && store)
      for (int s = 0; s < ch->cfg.ndata; ++s)
        if (!ch->have_fcst_slot[s]) {
          g_err = "ccmm_chains_set_fcst_slot missing for a data slot";
          return CCMM_ERR_STATE;
        }
    HIPCHECK(hipSetDevice(ch->ctx->device));
    if (crn) {
      ch->crn.alloc((size_t)ch->d.B * nsweeps * ch->crn_len);
      HIPCHECK(hipMemcpyAsync(ch->crn.p, crn, (size_t)ch->d.B * nsweeps * ch->crn_len * sizeof(double),
                              hipMemcpyHostToDevice, ch->ctx->stream));
    }
    for (int m = 0; m < nsweeps; ++m) {
      const double* base = crn ? ch->crn.p + (size_t)m * ch->crn_len : nullptr;
      ch->sweep_once(base, (int64_t)nsweeps * ch->crn_len, store != 0);
    }
    ch->join_fcst();
    if (ch->profiling) ch->collect_profile();
    if (crn) {
      HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
      return ch->check_status();
    }
    return 0;
  });
}

int ccmm_chains_stored(const ccmm_chains* ch) { return ch ? ch->stored : -1; }

int ccmm_chains_get_draws(ccmm_chains* ch, double* PAI_all, double* PHI_all, double* invA_all,
                          double* sqrtht_all, double* shadowrate_all) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const size_t B = ch->d.B, N = ch->d.N, K = ch->d.K, cap = ch->cfg.store_capacity;
    const size_t M = ch->stored, T = ch->cfg.T;
    auto fetch = [&](const DBuf<double>& src, size_t per, double* dst) {
      if (!dst || M == 0) return;
      std::vector<double> buf(B * cap * per);
      HIPCHECK(hipMemcpy(buf.data(), src.p, buf.size() * sizeof(double), hipMemcpyDeviceToHost));
      // device [c][m][e] -> MATLAB M x (e...) x B, i.e. dst[m + M*(e + per*c)]
      for (size_t c = 0; c < B; ++c)
        for (size_t m = 0; m < M; ++m)
          for (size_t e = 0; e < per; ++e) dst[m + M * (e + per * c)] = buf[(c * cap + m) * per + e];
    };
    fetch(ch->sPAI, K * N, PAI_all);
    fetch(ch->sPHI_, N * (N + 1) / 2, PHI_all);
    fetch(ch->sInvA, N * N, invA_all);
    fetch(ch->sSqrtht, T * N, sqrtht_all);
    if (ch->bh && ch->cfg.elbTmax > 0) fetch(ch->sShadow, (size_t)ch->cfg.Ns * ch->cfg.elbTmax, shadowrate_all);
    ch->stored = 0;
    ch->mom_done = 0;
    return 0;
  });
}

int ccmm_chains_pai_moments(ccmm_chains* ch, int reset, double* sum, double* sumsq) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    const size_t B = ch->d.B, per = (size_t)ch->d.K * ch->d.N;
    if (!ch->paiMom.p || reset) {
      ch->paiMom.alloc(2 * B * per);
      HIPCHECK(hipMemsetAsync(ch->paiMom.p, 0, 2 * B * per * sizeof(double), ch->ctx->stream));
      ch->mom_done = 0;
    }
    require(ch->stored >= ch->mom_done, "ccmm_chains_pai_moments: the store was reset; call with reset != 0");
    if (ch->stored > ch->mom_done && ch->sPAI.p) {
      hipLaunchKernelGGL(k_pai_moments, dim3((unsigned)((B * per + 255) / 256)), dim3(256), 0, ch->ctx->stream,
                         ch->sPAI.p, ch->cfg.store_capacity, ch->mom_done, ch->stored, (int)per, (int)B,
                         ch->paiMom.p, ch->paiMom.p + B * per);
      HIPCHECK(hipGetLastError());
      ch->mom_done = ch->stored;
    }
    if (sum || sumsq) {
      std::vector<double> buf(2 * B * per);
      HIPCHECK(hipMemcpyAsync(buf.data(), ch->paiMom.p, buf.size() * sizeof(double), hipMemcpyDeviceToHost,
                              ch->ctx->stream));
      HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
      // device [c][e] (e = a + K j) -> K x N x B
      if (sum) std::copy(buf.begin(), buf.begin() + B * per, sum);
      if (sumsq) std::copy(buf.begin() + B * per, buf.end(), sumsq);
    }
    return 0;
  });
}

int ccmm_chains_set_fcst(ccmm_chains* ch, int H, int Nd, const uint8_t* ndxYields, int keep_paths) {
  return guarded([&] {
    require(ch && ndxYields, "null argument");
    require(!ch->bh || ch->have_elb_model, "ccmm_chains_set_elb_model must be called before set_fcst");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    ch->set_fcst(H, Nd, ndxYields, keep_paths);
    return 0;
  });
}

int ccmm_chains_set_fcst_slot(ccmm_chains* ch, int slot, const double* yrealized) {
  return guarded([&] {
    require(ch && yrealized, "null argument");
    require(ch->have_fcst, "ccmm_chains_set_fcst must be called first");
    require(slot >= 0 && slot < ch->cfg.ndata, "slot out of range");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    HIPCHECK(hipMemcpy(ch->fYreal.p + (size_t)slot * ch->cfg.N, yrealized, ch->cfg.N * sizeof(double),
                       hipMemcpyHostToDevice));
    ch->have_fcst_slot[slot] = true;
    return 0;
  });
}

int ccmm_chains_set_fcst_censor(ccmm_chains* ch, const uint8_t* floor_in_recursion) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    require(ch->have_fcst, "ccmm_chains_set_fcst must be called first");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    if (!floor_in_recursion) {
      ch->have_rec_floor = false;
      return 0;
    }
    ch->fRecFloor.alloc(ch->cfg.N);
    HIPCHECK(hipMemcpy(ch->fRecFloor.p, floor_in_recursion, ch->cfg.N, hipMemcpyHostToDevice));
    ch->have_rec_floor = true;
    return 0;
  });
}

int ccmm_chains_fcst_stored(const ccmm_chains* ch) { return ch && ch->have_fcst ? ch->fstored : -1; }

int ccmm_chains_get_fcst(ccmm_chains* ch, double* scores, double* fYsum, double* fYcsum,
                         double* yhatsum, double* paths, double* paths_censored) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    require(ch->have_fcst, "ccmm_chains_set_fcst was not called");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const size_t B = ch->cfg.B, N = ch->cfg.N, H = ch->fH, Nd = ch->fNd;
    const size_t cap = ch->cfg.store_capacity, M = ch->fstored, HN = H * N;
    if (scores && M) {
      std::vector<double> buf(B * cap * Nd * 4);
      HIPCHECK(hipMemcpy(buf.data(), ch->fScStore.p, buf.size() * sizeof(double), hipMemcpyDeviceToHost));
      // device [c][m][job][k] -> Nd x M x 4 x B
      for (size_t c = 0; c < B; ++c)
        for (size_t m = 0; m < M; ++m)
          for (size_t job = 0; job < Nd; ++job)
            for (size_t k = 0; k < 4; ++k)
              scores[job + Nd * (m + M * (k + 4 * c))] = buf[((c * cap + m) * Nd + job) * 4 + k];
    }
    auto sums = [&](const DBuf<double>& src, double* dst) {
      if (dst) HIPCHECK(hipMemcpy(dst, src.p, B * HN * sizeof(double), hipMemcpyDeviceToHost));
    };
    sums(ch->fYsum, fYsum);
    sums(ch->fYcsum, fYcsum);
    sums(ch->fYhatsum, yhatsum);
    auto fetch_paths = [&](const DBuf<double>& src, double* dst) {
      if (!dst || !M) return;
      require(ch->fKeep != 0, "paths were not kept (keep_paths = 0)");
      const size_t per = M * Nd * HN;  // N x H x Nd x M per chain: the device order
      for (size_t c = 0; c < B; ++c)
        HIPCHECK(hipMemcpy(dst + c * per, src.p + c * cap * Nd * HN, per * sizeof(double),
                           hipMemcpyDeviceToHost));
    };
    fetch_paths(ch->fPaths, paths);
    fetch_paths(ch->fPathsC, paths_censored);
    std::vector<int> st(B);
    HIPCHECK(hipMemcpy(st.data(), ch->fStatus.p, B * sizeof(int), hipMemcpyDeviceToHost));
    int rc = 0;
    for (int v : st)
      if (v & 2) rc = CCMM_WARN_MVNCDF;
    if (rc) g_err = "censored log score with >= 4 series at the ELB (mvncdf) is NaN";
    ch->reset_fcst();
    return rc;
  });
}

int ccmm_chains_set_elb_model(ccmm_chains* ch, const int* ndxS, const uint8_t* actual_block) {
  return guarded([&] {
    require(ch && ndxS, "null argument");
    require(ch->bh, "chain set was not created with CCMM_MODEL_BLOCKHYBRID / CCMM_MODEL_HYBRID");
    const bool no_block = ch->hybrid || ch->cfg.model == CCMM_MODEL_SHADOWRATE;
    require(actual_block || no_block, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    std::vector<uint8_t> none(ch->cfg.N, 0);
    if (no_block) {
      for (int i = 0; actual_block && i < ch->cfg.N; ++i)
        require(!actual_block[i], "hybrid / shadow-rate model has no actual-rate block (pass NULL or zeros)");
      actual_block = none.data();
    }
    ch->set_elb_model(ndxS, actual_block);
    return 0;
  });
}

int ccmm_chains_set_elb_slot(ccmm_chains* ch, int slot, int elbT0, const uint8_t* sNaN) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    require(ch->bh, "chain set was not created with CCMM_MODEL_BLOCKHYBRID");
    require(slot >= 0 && slot < ch->cfg.ndata, "slot out of range");
    require(ch->have_slot[slot], "ccmm_chains_set_data must be called before set_elb_slot");
    require(sNaN != nullptr || ch->hT[slot] <= elbT0, "null sNaN");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    ch->set_elb_slot(slot, elbT0, sNaN);
    return 0;
  });
}

int ccmm_chains_set_elb_ps(ccmm_chains* ch, int nproposals, int ps_from_m) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    require(ch->bh, "chain set was not created with CCMM_MODEL_BLOCKHYBRID / CCMM_MODEL_HYBRID");
    require(nproposals == 0 || ps_from_m >= 1, "ps_from_m must be >= 1");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    ch->set_elb_ps(nproposals, ps_from_m);
    return 0;
  });
}

int ccmm_chains_get_ps(ccmm_chains* ch, int* countAccept, int* countAcceptBurnin, int* stackAccept) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    require(ch->ps_np > 0, "ccmm_chains_set_elb_ps was not called");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const size_t B = ch->cfg.B, cap = ch->cfg.store_capacity, M = ch->stored;
    std::vector<int> cnt(2 * B, 0);
    if (ch->psCount.p) HIPCHECK(hipMemcpy(cnt.data(), ch->psCount.p, cnt.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (size_t c = 0; c < B; ++c) {
      if (countAcceptBurnin) countAcceptBurnin[c] = cnt[2 * c];
      if (countAccept) countAccept[c] = cnt[2 * c + 1];
    }
    if (stackAccept && M) {
      std::vector<int> buf(B * cap, 0);
      if (ch->sAccept.p) HIPCHECK(hipMemcpy(buf.data(), ch->sAccept.p, buf.size() * sizeof(int), hipMemcpyDeviceToHost));
      for (size_t c = 0; c < B; ++c)
        for (size_t m = 0; m < M; ++m) stackAccept[m + M * c] = buf[c * cap + m];
    }
    return 0;
  });
}

int ccmm_chains_keep_missingrate(ccmm_chains* ch, int enable) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    require(ch->bh, "chain set has no ELB step (shadow-rate models only)");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    require(ch->stored == 0, "ccmm_chains_keep_missingrate: call before storing draws");
    ch->keep_first = enable != 0;
    return 0;
  });
}

int ccmm_chains_get_missingrate(ccmm_chains* ch, double* missingrate_all) {
  return guarded([&] {
    require(ch && missingrate_all, "null argument");
    require(ch->keep_first, "ccmm_chains_keep_missingrate was not enabled");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const size_t B = ch->cfg.B, cap = ch->cfg.store_capacity, M = ch->stored;
    const size_t per = (size_t)ch->cfg.Ns * ch->cfg.elbTmax;
    if (M == 0 || per == 0) return 0;
    std::vector<double> buf(B * cap * per);
    HIPCHECK(hipMemcpy(buf.data(), ch->sMissing.p, buf.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (size_t c = 0; c < B; ++c)
      for (size_t m = 0; m < M; ++m)
        for (size_t e = 0; e < per; ++e) missingrate_all[m + M * (e + per * c)] = buf[(c * cap + m) * per + e];
    return 0;
  });
}

int ccmm_chains_get_ps_mean(ccmm_chains* ch, double* mean) {
  return guarded([&] {
    require(ch && mean, "null argument");
    require(ch->ps_np > 0 && ch->psL.p, "ccmm_chains_set_elb_ps was not called or no PS sweep ran");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const size_t B = ch->cfg.B, nmax = ch->ps_nmax, W = ch->psW, per = (size_t)ch->cfg.Ns * ch->cfg.elbTmax;
    std::vector<double> L(B * nmax * W), yb(B * nmax);
    std::vector<int> cell(B * nmax), n(B);
    HIPCHECK(hipMemcpy(L.data(), ch->psL.p, L.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(yb.data(), ch->psY.p, yb.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(cell.data(), ch->psCell.p, cell.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(n.data(), ch->psN.p, n.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (size_t c = 0; c < B; ++c) {
      double* o = mean + c * per;
      for (size_t q = 0; q < per; ++q) o[q] = std::nan("");
      const double* Lc = L.data() + c * nmax * W;
      std::vector<double> x(n[c], 0.0);
      for (int i = n[c] - 1; i >= 0; --i) {  // x = L'^-1 ybar, band storage L(i + j, i) at [i][j]
        double v = yb[c * nmax + i];
        for (size_t j = 1; j < W && i + (int)j < n[c]; ++j) v -= Lc[(size_t)i * W + j] * x[i + j];
        x[i] = v / Lc[(size_t)i * W];
        o[cell[c * nmax + i]] = x[i];
      }
    }
    return 0;
  });
}

int ccmm_draw_summaries(ccmm_ctx* ctx, int S, int n, const double* draws, const double* realized, int nq,
                        const double* pct, double* mean, double* median, double* quantiles, double* stdev,
                        double* crps) {
  return guarded([&] {
    require(ctx && draws, "null argument");
    require(S >= 1 && n >= 1, "S and n must be positive");  // sorted in batches of < 2^31 items
    require(nq >= 0 && (nq == 0 || pct), "bad quantile list");
    HIPCHECK(hipSetDevice(ctx->device));
    DBuf<double> A, Bs, out;
    DBuf<char> ws;
    A.alloc((size_t)S * n);
    Bs.alloc((size_t)S * n);
    HIPCHECK(hipMemcpy(A.p, draws, (size_t)S * n * sizeof(double), hipMemcpyHostToDevice));
    const size_t wb = post_workspace_bytes(S, n);
    ws.alloc(wb);
    out.alloc((size_t)nq + (size_t)S * (5 + nq));
    double* dp = out.p;
    double* dr = dp + nq;
    double* dm = dr + S;
    double* dmed = dm + S;
    double* dsd = dmed + S;
    double* dcr = dsd + S;
    double* dq = dcr + S;
    if (nq) HIPCHECK(hipMemcpy(dp, pct, nq * sizeof(double), hipMemcpyHostToDevice));
    if (realized) HIPCHECK(hipMemcpy(dr, realized, S * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(post_summaries(ctx->stream, S, n, A.p, Bs.p, ws.p, wb, realized ? dr : nullptr, nq, dp, dm, dmed,
                            nq ? dq : nullptr, dsd, crps ? dcr : nullptr));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    auto get = [&](double* dst, const double* src, size_t cnt) {
      if (dst) HIPCHECK(hipMemcpy(dst, src, cnt * sizeof(double), hipMemcpyDeviceToHost));
    };
    get(mean, dm, S);
    get(median, dmed, S);
    get(stdev, dsd, S);
    get(crps, dcr, S);
    get(quantiles, dq, (size_t)S * nq);
    return 0;
  });
}

int ccmm_chains_summaries(ccmm_chains* ch, int source, int slot, const uint8_t* rows, const uint8_t* cumcode,
                          const double* realized, int nq, const double* pct, double* mean, double* median,
                          double* quantiles, double* stdev, double* crps) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    ch->summaries(source, slot, rows, cumcode, nullptr, 0.0, realized, nq, pct, mean, median, quantiles, stdev,
                  crps);
    return 0;
  });
}

int ccmm_chains_summaries_floor(ccmm_chains* ch, int source, int slot, const uint8_t* rows, const uint8_t* cumcode,
                                const uint8_t* floor_rows, double floor, const double* realized, int nq,
                                const double* pct, double* mean, double* median, double* quantiles, double* stdev,
                                double* crps) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    ch->summaries(source, slot, rows, cumcode, floor_rows, floor, realized, nq, pct, mean, median, quantiles, stdev,
                  crps);
    return 0;
  });
}

// bh: 0 linear, 1 block hybrid (ring = ndxYields, actual = actualrateBlock), 2 hybrid (ring =
// ring_vars = ndxSHADOWRATE, PAI (K + Ns p) x N x M); the output floor is ndxYields in both
static int girf_impl(ccmm_ctx* ctx, int M, int N, int p, int H, int nsim, const double* PAI, const double* invA,
                     const double* sqrtPHI, const double* SV0, const double* Xjumpoff, int bh, const uint8_t* actual,
                     const uint8_t* ring_vars, const uint8_t* ndxYields, double elb, const uint8_t* cumcode,
                     double np_, double shock11, const double* z, const double* svz, uint64_t seed, double* yhat) {
  return guarded([&] {
    require(ctx && PAI && invA && sqrtPHI && SV0 && Xjumpoff && yhat, "null argument");
    require(M >= 1 && N >= 1 && N <= 32 && p >= 1 && H >= 1 && nsim >= 1, "bad dimensions (N <= 32)");
    require(bh != 1 || (actual && ndxYields), "block hybrid needs actual and ndxYields");
    require(bh != 2 || (ring_vars && ndxYields), "hybrid needs ndxShadow and ndxYields");
    require((z == nullptr) == (svz == nullptr), "z and svz: both or neither");
    HIPCHECK(hipSetDevice(ctx->device));
    const int K = N * p + 1;
    std::vector<int> yi;
    if (bh)
      for (int i = 0; i < N; ++i)
        if (ring_vars[i]) yi.push_back(i);
    const int Ny = (int)yi.size();
    require(bh == 0 || Ny >= 1, "no ring variables");
    const int ldX = K + Ny * p;
    const int ldP = (bh == 2) ? ldX : K;
    require((K + Ny * p + N + 3) / 4 <= 96, "state too large for the GIRF kernel (K + Ny p + N <= 384)");
    const size_t nch = (size_t)(nsim + 3) / 4;
    DBuf<double> dPAI, dA, dS, dSV, dX, dZ, dSZ, dPart, dOut;
    DBuf<uint8_t> dAct, dCum, dFl;
    DBuf<int> dY;
    auto up = [&](auto& buf, const auto* src, size_t n) {
      buf.alloc(n);
      HIPCHECK(hipMemcpy(buf.p, src, n * sizeof(src[0]), hipMemcpyHostToDevice));
    };
    // PAI ldP x N x M column-major == [M][N][ldP]
    up(dPAI, PAI, (size_t)ldP * N * M);
    up(dA, invA, (size_t)N * N * M);
    up(dS, sqrtPHI, (size_t)N * N * M);
    up(dSV, SV0, (size_t)N * M);
    up(dX, Xjumpoff, (size_t)ldX * M);
    if (z) {
      up(dZ, z, (size_t)N * H * nsim * M);
      up(dSZ, svz, (size_t)N * H * nsim * M);
    }
    if (bh == 1) up(dAct, actual, (size_t)N);
    if (bh) {
      up(dY, yi.data(), yi.size());
      up(dFl, ndxYields, (size_t)N);
    }
    if (cumcode) up(dCum, cumcode, (size_t)N);
    dPart.alloc((size_t)M * 3 * nch * H * N);
    dOut.alloc((size_t)M * 3 * H * N);
    GirfArgs a{};
    a.M = M; a.N = N; a.p = p; a.H = H; a.nsim = nsim; a.bh = bh; a.Ny = Ny;
    a.PAI = dPAI.p; a.invA = dA.p; a.sqrtPHI = dS.p; a.SV0 = dSV.p; a.Xj = dX.p; a.ldX = ldX;
    a.actual = bh == 1 ? dAct.p : nullptr; a.yidx = bh ? dY.p : nullptr; a.yfloor = bh ? dFl.p : nullptr;
    a.elb = elb; a.shock11 = shock11;
    a.z = z ? dZ.p : nullptr; a.svz = z ? dSZ.p : nullptr; a.seed = seed;
    a.cumcode = cumcode ? dCum.p : nullptr; a.np_ = np_; a.part = dPart.p; a.out = dOut.p;
    a.force_generic = ctx->opt[OPT_GIRF_GENERIC];  // A/B of the specialised kernel
    HIPCHECK(girf_launch(ctx->stream, a));
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(yhat, dOut.p, dOut.n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
  });
}

int ccmm_girf(ccmm_ctx* ctx, int M, int N, int p, int H, int nsim, const double* PAI, const double* invA,
              const double* sqrtPHI, const double* SV0, const double* Xjumpoff, int bh, const uint8_t* actual,
              const uint8_t* ndxYields, double elb, const uint8_t* cumcode, double np_, double shock11,
              const double* z, const double* svz, uint64_t seed, double* yhat) {
  return girf_impl(ctx, M, N, p, H, nsim, PAI, invA, sqrtPHI, SV0, Xjumpoff, bh ? 1 : 0, actual, ndxYields,
                   ndxYields, elb, cumcode, np_, shock11, z, svz, seed, yhat);
}

int ccmm_girf_hybrid(ccmm_ctx* ctx, int M, int N, int p, int H, int nsim, const double* PAI, const double* invA,
                     const double* sqrtPHI, const double* SV0, const double* Xjumpoff, const uint8_t* ndxShadow,
                     const uint8_t* ndxYields, double elb, const uint8_t* cumcode, double np_, double shock11,
                     const double* z, const double* svz, uint64_t seed, double* yhat) {
  return girf_impl(ctx, M, N, p, H, nsim, PAI, invA, sqrtPHI, SV0, Xjumpoff, 2, nullptr, ndxShadow, ndxYields,
                   elb, cumcode, np_, shock11, z, svz, seed, yhat);
}

int ccmm_chains_get_cta_gram(ccmm_chains* ch, double* G) {
  return guarded([&] {
    require(ch && G, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    ch->export_cta_gram(G);
    return 0;
  });
}

int ccmm_chains_get_cta_factor(ccmm_chains* ch, double* F) {
  return guarded([&] {
    require(ch && F, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    ch->export_cta_factor(F);
    return 0;
  });
}

int ccmm_chains_get_shadowrate(ccmm_chains* ch, double* shadowrate) {
  return guarded([&] {
    require(ch && shadowrate, "null argument");
    require(ch->bh, "chain set was not created with CCMM_MODEL_BLOCKHYBRID");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    if (ch->cfg.elbTmax > 0)
      HIPCHECK(hipMemcpy(shadowrate, ch->eScur.p,
                         (size_t)ch->d.B * ch->cfg.Ns * ch->cfg.elbTmax * sizeof(double),
                         hipMemcpyDeviceToHost));
    return 0;
  });
}

int ccmm_chains_get_xy(ccmm_chains* ch, double* X, double* Y) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    HIPCHECK(hipStreamSynchronize(ch->ctx->stream));
    const int B = ch->d.B, N = ch->d.N, K = ch->d.K, KP = ch->d.KP, TP = ch->d.TP, T = ch->cfg.T;
    std::vector<int> sl(B);
    HIPCHECK(hipMemcpy(sl.data(), ch->slot.p, B * sizeof(int), hipMemcpyDeviceToHost));
    std::vector<double> xb((size_t)KP * TP), yb((size_t)N * TP);
    for (int c = 0; c < B; ++c) {
      const int xs = ch->bh ? ch->cfg.ndata + c : sl[c];
      if (X) {
        HIPCHECK(hipMemcpy(xb.data(), ch->Xpool.p + (size_t)xs * KP * TP, xb.size() * sizeof(double),
                           hipMemcpyDeviceToHost));
        for (int a = 0; a < K; ++a)
          for (int t = 0; t < T; ++t) X[((size_t)c * K + a) * T + t] = xb[(size_t)a * TP + t];
      }
      if (Y) {
        HIPCHECK(hipMemcpy(yb.data(), ch->Ypool.p + (size_t)xs * N * TP, yb.size() * sizeof(double),
                           hipMemcpyDeviceToHost));
        for (int i = 0; i < N; ++i)
          for (int t = 0; t < T; ++t) Y[((size_t)c * N + i) * T + t] = yb[(size_t)i * TP + t];
      }
    }
    return 0;
  });
}

int ccmm_chains_profile(ccmm_chains* ch, int enable) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    ch->collect_profile();
    ch->profiling = enable != 0;
    for (int k = 0; k < KID_COUNT; ++k) {
      ch->kms[k] = 0.0;
      ch->kcount[k] = 0;
    }
    return 0;
  });
}

int ccmm_chains_kernel_times(ccmm_chains* ch, int max, double* ms, int64_t* launches, char* names,
                             int names_len) {
  return guarded([&] {
    require(ch != nullptr, "null argument");
    HIPCHECK(hipSetDevice(ch->ctx->device));
    ch->collect_profile();
    const int n = std::min<int>(max, KID_COUNT);
    for (int k = 0; k < n; ++k) {
      if (ms) ms[k] = ch->kms[k];
      if (launches) launches[k] = ch->kcount[k];
    }
    if (names && names_len > 0) {
      std::string s;
      for (int k = 0; k < KID_COUNT; ++k) {
        if (k) s += ";";
        s += kKernelNames[k];
      }
      std::strncpy(names, s.c_str(), names_len - 1);
      names[names_len - 1] = 0;
    }
    return KID_COUNT;
  });
}

int ccmm_fcst(ccmm_ctx* ctx, int B, int N, int p, int H, int Nd, const double* PAI,
              const double* invA, const double* logSV0, const double* sqrtPHI,
              const double* Xjumpoff, const double* yrealized, const uint8_t* ndxYields,
              double elb, const double* svz, const double* z, uint64_t seed, int sweep,
              double* fcstY, double* fcstYcensor, double* yhat, double* scores, int* status) {
  return guarded([&] {
    require(ctx && PAI && invA && logSV0 && sqrtPHI && Xjumpoff && yrealized && ndxYields &&
                fcstY && fcstYcensor && yhat && scores,
            "null argument");
    require(B > 0 && N > 0 && N <= kFcstMaxN && p > 0 && H > 0 && Nd > 0, "unsupported size");
    require((svz == nullptr) == (z == nullptr), "svz and z must both be given or both NULL");
    const int K = N * p + 1;
    int nwx = 0;
    for (int i = 0; i < N; ++i) nwx += ndxYields[i] ? 0 : 1;
    require(nwx > 0 && nwx < N, "need at least one macro series and one yield");
    HIPCHECK(hipSetDevice(ctx->device));
    require(fcst_paths_lds_doubles(N, K, p, fcst_chunk(N, K, p, H)) * sizeof(double) <= 160 * 1024,
            "forecast state does not fit LDS");
    static const GLNodes gl = make_gl_nodes();
    auto up = [&](DBuf<double>& d, const double* h, size_t n) {
      d.alloc(n);
      HIPCHECK(hipMemcpyAsync(d.p, h, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    };
    DBuf<double> dPAI, dinvA, dlog, dsq, dXj, dy, dsvz, dz, dfY, dfYc, dyhat, dsc, dsv1;
    DBuf<uint8_t> dmask;
    DBuf<int> dst;
    up(dPAI, PAI, (size_t)B * K * N);
    up(dinvA, invA, (size_t)B * N * N);
    up(dlog, logSV0, (size_t)B * N);
    up(dsq, sqrtPHI, (size_t)B * N * N);
    up(dXj, Xjumpoff, (size_t)B * K);
    up(dy, yrealized, (size_t)N);
    if (svz) {
      up(dsvz, svz, (size_t)B * N * H * Nd);
      up(dz, z, (size_t)B * N * H * Nd);
    }
    dmask.alloc(N);
    HIPCHECK(hipMemcpyAsync(dmask.p, ndxYields, N, hipMemcpyHostToDevice, ctx->stream));
    const size_t nout = (size_t)B * N * H * Nd;
    dfY.alloc(nout);
    dfYc.alloc(nout);
    dyhat.alloc((size_t)B * N * H);
    dsc.alloc((size_t)B * 4 * Nd);
    dst.alloc(B);
    HIPCHECK(hipMemsetAsync(dst.p, 0, B * sizeof(int), ctx->stream));
    FcstArgs a{};
    a.B = B; a.N = N; a.p = p; a.K = K; a.Kx = K; a.H = H; a.Nd = Nd; a.bh = 0;
    a.PAI = dPAI.p; a.ldPAI = K; a.invA = dinvA.p; a.logSV = dlog.p; a.ldSV = 1;
    a.svT = nullptr; a.slot = nullptr; a.sqrtPHI = dsq.p; a.Xj = dXj.p; a.ldXj = K;
    a.yreal = dy.p; a.ldY = 0; a.ndxYields = dmask.p; a.actual = nullptr; a.elb = elb;
    a.svz = svz ? dsvz.p : nullptr;
    a.z = svz ? dz.p : nullptr;
    a.crnStride = (int64_t)N * H * Nd;
    a.seed = seed; a.sweep = (uint32_t)sweep;
    a.fY = dfY.p; a.fYc = dfYc.p; a.yhat = dyhat.p; a.scores = dsc.p; a.status = dst.p;
    a.gl = gl;
    dsv1.alloc((size_t)B * Nd * N);
    launch_fcst(ctx->stream, a, dsv1.p, ctx->opt[OPT_FCST_REG] != 0);
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(fcstY, dfY.p, nout * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(fcstYcensor, dfYc.p, nout * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(yhat, dyhat.p, (size_t)B * N * H * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(scores, dsc.p, (size_t)B * 4 * Nd * sizeof(double), hipMemcpyDeviceToHost));
    std::vector<int> st(B);
    HIPCHECK(hipMemcpy(st.data(), dst.p, B * sizeof(int), hipMemcpyDeviceToHost));
    int rc = 0;
    for (int c = 0; c < B; ++c) {
      if (status) status[c] = st[c];
      if (st[c] & 2) rc = CCMM_WARN_MVNCDF;
    }
    if (rc) g_err = "censored log score with >= 3 series at the ELB (mvncdf) is NaN";
    return rc;
  });
}

int ccmm_selftest_mfma_f64(ccmm_ctx* ctx, const double* A16x4, const double* B4x16, double* D16x16) {
  return guarded([&] {
    require(ctx && A16x4 && B4x16 && D16x16, "null argument");
    HIPCHECK(hipSetDevice(ctx->device));
    DBuf<double> a, b, dd;
    a.alloc(64);
    b.alloc(64);
    dd.alloc(256);
    HIPCHECK(hipMemcpy(a.p, A16x4, 64 * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(b.p, B4x16, 64 * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_mfma_selftest, dim3(1), dim3(64), 0, ctx->stream, a.p, b.p, dd.p);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(D16x16, dd.p, 256 * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
  });
}

int ccmm_selftest_mfma_f64_acc(ccmm_ctx* ctx, int nprobe, const double* A16x4, const double* B4x16,
                               const double* C16x16, double* D16x16) {
  return guarded([&] {
    require(ctx && A16x4 && B4x16 && C16x16 && D16x16 && nprobe > 0 && nprobe <= (1 << 20), "bad argument");
    HIPCHECK(hipSetDevice(ctx->device));
    DBuf<double> a, b, cc, dd;
    a.alloc((size_t)64 * nprobe);
    b.alloc((size_t)64 * nprobe);
    cc.alloc((size_t)256 * nprobe);
    dd.alloc((size_t)256 * nprobe);
    HIPCHECK(hipMemcpy(a.p, A16x4, (size_t)64 * nprobe * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(b.p, B4x16, (size_t)64 * nprobe * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(cc.p, C16x16, (size_t)256 * nprobe * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_mfma_selftest_acc, dim3(nprobe), dim3(64), 0, ctx->stream, a.p, b.p, cc.p, dd.p, nprobe);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(ctx->stream));
    HIPCHECK(hipMemcpy(D16x16, dd.p, (size_t)256 * nprobe * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
  });
}

}  // extern "C"
