// Generalized impulse responses by antithetic simulation on the device (ccmm_girf.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ccmm {

struct GirfArgs {
  int M, N, p, H, nsim, bh, Ny;  // MCMC draws, variables, lags, horizons, shock paths, model
                                 // (bh: 0 linear, 1 block hybrid, 2 hybrid: the ring holds the Ny
                                 // shadow-rate variables and PAI has K + Ny p rows per equation)
  const double* PAI;             // device [M][N][K]
  const double* invA;            // device [M][N][N]
  const double* sqrtPHI;         // device [M][N][N] lower Cholesky of PHI
  const double* SV0;             // device [M][N] jump-off sqrtht
  const double* Xj;              // device [M][ldX] Xjumpoff
  int ldX;
  const uint8_t* actual;         // device [N] actualrateBlock (block hybrid) or null
  const int* yidx;               // device [Ny] ring variables (block hybrid: yields; hybrid: shadow rates)
  const uint8_t* yfloor;         // device [N] variables floored at the ELB in the output (ndxYIELDS) or null
  double elb, shock11;
  const double* z;               // device [M][nsim][H][N] or null (Philox)
  const double* svz;             // device [M][nsim][H][N] or null
  uint64_t seed;
  const uint8_t* cumcode;        // device [N] or null
  double np_;
  double* part;                  // device workspace [M][3][ceil(nsim/4)][H][N]
  double* out;                   // device [M][3][H][N]: baseline, +shock, -shock mean paths
  int force_generic;             // 1: the table-driven kernel even where a specialised one exists
};

size_t girf_lds_bytes(int N, int p, int KT);
hipError_t girf_launch(hipStream_t st, const GirfArgs& a);

}  // namespace ccmm
