// Device views, record layouts and kernel declarations of the ELB shadow-rate step and its
// acceptance-sampling branch.  The kernels are defined (and instantiated for every template argument
// ccmm_abi.hip launches) in their own translation units, ccmm_elb.hip and ccmm_ps.hip; this header is
// what the host side (ccmm_abi.hip) and the predictive-density kernels see.
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

constexpr int kElbNsMax = 5;  // Ns = 5: the Krippner / Wu-Xia datasets at ELB > 0.25 (setShadowYields.m:1-5)
constexpr int kElbColMax = 128;  // 2 p Ns neighbour columns, two per lane

struct ElbDev {
  int Ns, p, elbTmax, passes;    // passes = gibbsburn + 1
  double elb;
  const int* ndxS;               // [Ns]
  const uint8_t* actual;         // [N] actualrateBlock
  const int* elbT0;              // [ndata]
  const int* elbT;               // [ndata]
  const uint8_t* sNaN;           // [ndata][elbTmax][Ns]  (t-major)
  const int* ncens;              // [ndata]
  const int* cens;               // [ndata][elbTmax] censored months in increasing order
  const double* Xactual;         // X pool (slot slabs first)
  // per chain scratch
  double* Phi;    // [B][N][N*p]   Phi[i][(l-1)N + q] = PAIshadow(1+(l-1)N+q, i)
  double* Y0;     // [B][elbTmax][N]  scratch: Yb - Yhatactual
  double* Yt;     // [B][elbTmax][N]  Yb: the chain's Y, censored shadow-rate cells at 0
  double* Et;     // [B][elbTmax][N]  ε_τ (stable residual form, see k_elb_prep)
  double* cond;   // [B][elbTmax][condStride]
  double* Scur;   // [B][elbTmax][Ns] shadow rates (in/out)
  int condStride;
  int kshadow, K;  // hybrid model: PAI rows kshadow..K-1 load the actual-rate lags (K > kshadow)
  int mode;        // CCMM_ELB_MODE timing ablation (0 in production)
  const double* yhat;  // [B][elbTmax][N] explicit YHAT0 (ccmm_gibbs_shadowrates) or nullptr
  uint8_t* flags;      // [B][passes][elbTmax][Ns] truncated-normal branch flags or nullptr
  // acceptance-sampling branch (mcmcVARshadowrateBlockHybrid.m:438-466, ccmm_ps.hip)
  int ps;              // 1: k_elb_prep / k_elb_cond also build the PS precision records
  double* EtPS;        // [B][elbTmax][N] residuals of the PS model (Yhatactual as intercept)
  const int* psFlag;   // [B] PS outcome of this sweep: > 0 accepted (k_elb_gibbs skips the chain)
  // gibbsdrawShadowratesB3 (ccmm_gibbs_shadowrates_b3): the VAR on Y itself with the intercept in the
  // state (base residuals in the PS model's form, yhat = 0) and, when Amon is set, a structural matrix
  // per window month, A_tau = B(2:Ny+1, :, tau)^-1 ([B][elbTmax][N][N], lower)
  int b3;
  const double* Amon;
  // 1: the structural matrices A (cs.A / Amon) are full -- the inverse of a general impact matrix
  // Psi(2:Ny+1, :) (ccmm_gibbs_shadowrates); 0: unit lower triangular (every sweep; invA's inverse)
  int Afull;
  // speculative Gibbs step (k_elb_gibbs_wf ASYNC / k_elb_gibbs_mp, small B): the passes start beside the PS
  // branch (ccmm_ps.hip) on another stream; k_ps_apply posts psState[c] = psEpoch << 1 | accepted, the
  // waves stop early once they see an accepted proposal (a poll, never a wait: the streams need not run
  // concurrently), the draw goes to ScurSpec, and k_elb_spec_select keeps it only where the PS branch
  // rejected -- the reference's order (PS first, the Gibbs draw as the fallback, :438-466), same draws
  int spec;
  const unsigned long long* psState;
  unsigned long long psEpoch;
  double* ScurSpec;  // [B][elbTmax][Ns]
};

// condition record per censored month (doubles):
//   a_t [Ns] | beta1 [Ns][Ns-1] | sqrtOmega1 [Ns] | 1 / sqrtOmega1 [Ns] | Ω [Ns][Ns] | G [2p Ns][Ns]
// (1 / sqrtOmega1: the Gibbs kernels form ub = (elb - mu) / sig as a product, off the division's latency)
// G column col = kk*Ns + s': kk < p past lag kk+1, kk >= p future lead kk-p+1.
// With the PS branch (e.ps) the record continues (elb_cond_ps_off):
//   P [Ns][Ns] (the month's precision, Ω^-1) | b_PS [Ns] | gP [p Ns][Ns]
// b_PS = the PS model's linear term with every censored cell at 0; gP = the raw unit
// responses of the past neighbours (-gP = the off-diagonal precision blocks).
__host__ __device__ inline int elb_cond_head(int Ns) { return Ns + Ns * (Ns - 1) + 2 * Ns + Ns * Ns; }
__host__ __device__ inline int elb_cond_ps_off(int Ns, int p) {
  return elb_cond_head(Ns) + 2 * p * Ns * Ns;
}
__host__ __device__ inline int elb_cond_stride(int Ns, int p, int ps = 0) {
  return elb_cond_ps_off(Ns, p) + (ps ? Ns * Ns + Ns + p * Ns * Ns : 0);
}

constexpr int kElbPrepThreads = 512;
constexpr int kElbOctMinB = 384;  // k_elb_gibbs_oct from this many chains (option elb_oct = 1)
// k_elb_gibbs_mp (multi-CU wavefront, small B): granule exchange between the parts of a chain
constexpr int kElbMpMaxB = 64;  // auto: the multi-CU wavefront for B <= 64 chains
struct ElbXch {
  double* gran;                // [B][PARTS][elbTmax][NS] granules of 2 doubles {value, tag bits}
  unsigned long long epoch;    // launch counter (host): tags of older launches never match
};

constexpr int kPsWMax = 80;  // band width limit: Ns (p + 1) <= 80 (Ns = 5 with p = 12: 65)

struct PsDev {
  int nmax, W, NP;  // max censored cells over slots, band width, proposals per sweep
  double elb;
  double* L;        // [B][nmax][W]  L(i + j, i) at [i][j], zero beyond n
  double* ybar;     // [B][nmax]     L^-1 b
  int* cell;        // [B][nmax]     shadow-rate offset t Ns + a of censored cell i
  int* n;           // [B]           censored cells (0: PS skipped this sweep)
  int* acc;         // [B]           smallest accepted proposal (0-based), INT_MAX none
  int* flag;        // [B]           ndxAccept of this sweep (1-based), 0 none
  int* count;       // [B][2]        accepted sweeps: [0] burn-in, [1] kept (countELBaccept*)
  double* first;    // [B][Ns elbTmax] proposal 1 over the window (shadowrateProposals(:,:,1), kept as
                    //               missingrate, mcmcVARshadowrate.m:435); nullptr: not kept
  int per;          // Ns elbTmax
  unsigned long long* state;  // [B] speculative Gibbs step: epoch << 1 | accepted, posted by k_ps_apply
  unsigned long long epoch;   //     (nullptr / 0: no Gibbs step waits on the decision)
};

constexpr int kPsChunk = 64;  // assembled band rows per LDS chunk

__host__ __device__ inline size_t ps_chol_w_lds_bytes(int W, int elbTmax, int nmax) {
  return (size_t)(kPsChunk * W + kPsChunk + W) * sizeof(double) + (size_t)(elbTmax + nmax) * sizeof(int);
}

// ---------------------------------------------------------------- kernels (ccmm_elb.hip)
__global__ void k_elb_prep(Dims d, ElbDev e, XSel xs, ChainState cs, int phi_lds, int rows);
template <int NS> __global__ void k_elb_cond(Dims d, ElbDev e, ChainState cs, int a_lds, int kb);
template <int NS> __global__ void k_elb_gibbs(Dims d, ElbDev e, ChainState cs, RngArgs ra);
template <int NS, int W, bool ASYNC> __global__ void k_elb_gibbs_wf(Dims d, ElbDev e, ChainState cs, RngArgs ra);
template <int NS, int WPC, int PARTS>
__global__ void k_elb_gibbs_mp(Dims d, ElbDev e, ChainState cs, RngArgs ra, ElbXch xc);
template <int NS> __global__ void k_elb_gibbs_oct(Dims d, ElbDev e, ChainState cs, RngArgs ra);
__global__ void k_elb_spec_select(ElbDev e, const int* slot, int B);
__global__ void k_elb_rebuild(Dims d, ElbDev e, XSel xs, ChainState cs, int xslab0, double* dpool, int ldd, int drows,
                              double* dcpool, int dcld, long long dcslab);
__global__ void k_elb_store(ElbDev e, ChainState cs, double* out, int cap, int m);
// ---------------------------------------------------------------- kernels (ccmm_ps.hip)
__global__ void k_ps_chol(Dims d, ElbDev e, PsDev ps, ChainState cs);
template <int W> __global__ void k_ps_chol_w(Dims d, ElbDev e, PsDev ps, ChainState cs);
template <int W> __global__ void k_ps_prop(ElbDev e, PsDev ps, RngArgs ra);
template <int W> __global__ void k_ps_apply(ElbDev e, PsDev ps, RngArgs ra, int kept);
__global__ void k_ps_first_store(const double* first, const int* elbT, const int* slot, double* out, int per,
                                 int Ns, int cap, int m);
__global__ void k_ps_store(const int* flag, int* out, int B, int cap, int m);

}  // namespace ccmm
