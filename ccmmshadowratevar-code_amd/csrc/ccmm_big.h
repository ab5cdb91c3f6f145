// Large-system CTA (ccmm_big.hip, its own translation unit): host launchers used by
// ccmm_abi.hip when K > 512 or N > 32 (the S120 configuration N = 120, K = 1441).
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

constexpr int kBigMaxN = 128;
constexpr int kBigMaxKP = 1536;

// dynamic LDS of k_cta_solve_big
size_t big_solve_lds_bytes(const Dims& d);

// groups: ngroups x int4 systems (c*N + j) sharing one design X slab (-1 padded);
// phase_mask: 1 Gram, 2 Cholesky, 4 solve.  Ubuf: B x N x TP scratch (U = E A');
// Dinv: nmat x (KP/64) x 64 x 64 inverses of the Cholesky factor's diagonal blocks.
hipError_t big_launch_cta(hipStream_t st, const Dims& d, const int* Tslot, const int* slotIV,
                          const double* iVdiag, const double* iVb, XSel xs, ChainState cs,
                          const int4* groups, int ngroups, double* rdiag, RngArgs ra, double* Ubuf,
                          double* Dinv, int phase_mask);

}  // namespace ccmm
