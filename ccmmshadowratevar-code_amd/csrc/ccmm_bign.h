// Large-N Gibbs blocks (ccmm_bign.hip, its own translation unit): A-step, PHI and SV for
// 32 < N <= 128, used by ccmm_abi.hip in place of the per-chain small-matrix kernels.
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

// doubles of SV scratch per chain: Q, L_0..L_T, M_0..M_T (N x N each), w_0..w_T
size_t bign_sv_scratch(const Dims& d);

// wbuf: B x N x TP (weights 1 / sqrtht^2 of each row's regression)
hipError_t bign_launch_astep(hipStream_t st, const Dims& d, const int* Tslot, ChainState cs, RngArgs ra,
                             double logy2offset, double* wbuf);
// scr: B x 3 x N x N
hipError_t bign_launch_phi(hipStream_t st, const Dims& d, const int* Tslot, int dPHI, const double* sPHI,
                           ChainState cs, double* scr);
// scr: B x bign_sv_scratch(d); cs.svobs / cs.svir from k_sv_mix
hipError_t bign_launch_sv(hipStream_t st, const Dims& d, const int* Tslot, const double* V0inv,
                          const double* V0invm, ChainState cs, RngArgs ra, double* scr);

}  // namespace ccmm
