// Arguments, LDS budgets and kernel declarations of the predictive-density kernels (defined and
// instantiated in their own translation unit, ccmm_fcst.hip; launched by ccmm_abi.hip).
#pragma once
#include <algorithm>

#include "ccmm_internal.h"
#include "ccmm_elb.h"  // kElbNsMax

namespace ccmm {

constexpr int kFcstMaxN = 32;

struct GLNodes {  // Gauss-Legendre half rules (negative nodes) for n = 6, 12, 20 (Genz BVN)
  double x[3][10];
  double w[3][10];
};

struct FcstArgs {
  int B, N, p, K, H, Nd;
  int bh;                 // 1: block-hybrid companion (mcmcVARshadowrateBlockHybrid.m:147-159,566-625);
                          // 2: hybrid (mcmcVARhybridGibbs.m:160-172,566-635): PAI has Kx = K + Ns p
                          //    rows, the last Ns p multiply the Ns actual-rate lags max(shadow, ELB)
  int Kx;                 // rows of PAI used (K, or K + Ns p for the hybrid model)
  int Ns;                 // hybrid: shadow-rate variables
  const int* ndxS;        // hybrid: [Ns] their indices
  const double* PAI;      // [B][N][ldPAI]  (Kx x N column-major per chain, ld Kx or KP)
  int ldPAI;
  const double* invA;     // [B][N][N]
  const double* logSV;    // logSV0(c, i) = logSV[(c N + i) ldSV + (svT ? svT[slot c] - 1 : 0)]
  int ldSV;
  const int* svT;         // per-slot T (chain set: Vol_states(end,:) of the vintage) or nullptr
  const int* slot;        // [B] data slot of chain c, or nullptr (slot 0)
  const double* sqrtPHI;  // [B][N][N]
  const double* Xj;       // [B][ldXj] Xjumpoff: K states [1, y(T), .., y(T-p+1)]; block hybrid:
  int ldXj;               //   then p blocks of N actual-data lags Xj[K + l N + i] (:88-96,511-520);
                          //   hybrid: p blocks of Ns floored actual rates Xj[K + l Ns + s] (:111-121)
  const double* yreal;    // yrealized(:,1) of chain c at yreal + slot(c) * ldY
  int ldY;
  const uint8_t* ndxYields;  // [N]
  const uint8_t* recFloor;   // [N] linear model: variables floored inside the censored recursion
                             //   (nullptr: ndxYields, mcmcVAR.m:360-366; mcmcVARshadowrate.m:539-546
                             //   floors ndxOTHERYIELDS only)
  const uint8_t* actual;     // [N] actualrateBlock (bh) or nullptr
  double elb;
  const double* svz;      // randn(N, H*Nd) of chain c at svz + c * crnStride, or nullptr (Philox)
  const double* z;        // randn(N, H, Nd) of chain c at z + c * crnStride, or nullptr
  int64_t crnStride;
  uint64_t seed;
  uint32_t sweep;
  const uint32_t* ids;    // Philox stream id of chain c, or nullptr (c)
  double* fY;             // [B][Nd][H][N]  simulated paths (bh: uncensored)
  double* fYc;            // [B][Nd][H][N]  censored simulation (bh: yields floored at the ELB)
  double* yhat;           // [B][H][N]      zero-shock mean path (linear only)
  double* scores;         // [B][Nd][4]
  int* status;            // [B]  bit 1: NaN score (more than kMvnMaxD censored series)
  GLNodes gl;
  int mode;               // timing-only ablation (CCMM_FCST_MODE; results invalid): 1 no scores, 2 no horizons
  int hc;                 // horizons per shock chunk of k_fcst (fcst_paths_lds_doubles)
  double* sv1;            // [B][Nd][N] SV at horizon 1 of each draw (k_fcst -> k_fcst_scores)
};

// k_fcst<kFcstRegN> (N <= 21, p <= 3 kFcstRegLags, not hybrid) holds each lane's PAI column
// entries for its lags in registers instead of staging PAI in LDS: the lag sums then read only
// the ring from LDS, and the workgroup's LDS drops from ~52 KB to ~18 KB (hc <= 16) so that
// eight waves share a CU instead of three.  Same fma order, same sums.
constexpr int kFcstRegN = 21, kFcstRegLags = 4;  // k_fcst<20>: the same for even N <= 20

__host__ __device__ inline bool fcst_reg_path(int N, int p, int bh) {
  return N <= kFcstRegN && p <= 3 * kFcstRegLags && bh != 2;
}

__host__ __device__ inline size_t fcst_paths_lds_doubles(int N, int Kx, int p, int hc, bool reg = false) {
  return (reg ? 0 : (size_t)Kx * N) + 2 * (size_t)N * N + 2 * (size_t)p * N + 3 * (size_t)hc * N;
}

__host__ __device__ inline size_t fcst_scores_lds_doubles(int N) {
  return 2 * (size_t)N * N + 6 * (size_t)N + kFcstMaxN * kFcstMaxN;
}

// horizons per shock chunk so that k_fcst's LDS fits one CU (at most H; at least 1)
// (the register path: at most 16 horizons, so that eight workgroups share a CU)
inline int fcst_chunk(int N, int Kx, int p, int H, bool reg = false) {
  int hc = reg ? std::min(H, 16) : H;
  while (hc > 1 && fcst_paths_lds_doubles(N, Kx, p, hc, reg) * sizeof(double) > 160 * 1024) hc = (hc + 1) / 2;
  return hc;
}

template <int RN> __global__ void k_fcst(FcstArgs a);
__global__ void k_fcst_scores(FcstArgs a);
__global__ void k_fcst_jumpoff(int N, int p, int K, int TP, const int* __restrict__ Tslot,
                               const int* __restrict__ slot, const double* __restrict__ ypool,
                               const int* __restrict__ yidx, int ldXj, double* __restrict__ Xj, int Ns,
                               const int* __restrict__ ndxS, double elb);
__global__ void k_fcst_accum(int N, int H, int Nd, int cap, int m, const double* __restrict__ fY,
                             const double* __restrict__ fYc, const double* __restrict__ yhat,
                             const double* __restrict__ sc, double* __restrict__ sum,
                             double* __restrict__ sumc, double* __restrict__ sumhat,
                             double* __restrict__ scStore, double* __restrict__ paths,
                             double* __restrict__ pathsc);

}  // namespace ccmm
