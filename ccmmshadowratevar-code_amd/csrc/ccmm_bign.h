// Large-N Gibbs blocks (ccmm_bign.hip, its own translation unit): A-step, PHI and SV for
// 32 < N <= 128, used by ccmm_abi.hip in place of the per-chain small-matrix kernels.
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

// doubles of SV scratch per chain: Q, L_0..L_T, M_0..M_T (N x N each), w_0..w_T
size_t bign_sv_scratch(const Dims& d);

// padded Gram dimension of the A-step (64 for N <= 64, else 128)
int bign_astep_npad(const Dims& d);
// gbuf: B x (N - 1) x NPAD x NPAD (the weighted Grams of the N - 1 row regressions, k_astep_gram)
hipError_t bign_launch_astep(hipStream_t st, const Dims& d, const int* Tslot, ChainState cs, RngArgs ra,
                             double logy2offset, double* gbuf);
// scr: B x 3 x N x N
hipError_t bign_launch_phi(hipStream_t st, const Dims& d, const int* Tslot, int dPHI, const double* sPHI,
                           ChainState cs, double* scr);
// scr: B x bign_sv_scratch(d); cs.svobs / cs.svir from k_sv_mix
hipError_t bign_launch_sv(hipStream_t st, const Dims& d, const int* Tslot, const double* V0inv,
                          const double* V0invm, ChainState cs, RngArgs ra, double* scr);

}  // namespace ccmm
