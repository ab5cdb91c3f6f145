// Large-system CTA (ccmm_big.hip, its own translation unit): host launchers used by
// ccmm_abi.hip when K > 512 or N > 32 (the S120 configuration N = 120, K = 1441).
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

constexpr int kBigMaxN = 128;
constexpr int kBigMaxKP = 1536;

// dynamic LDS of k_cta_solve_big
size_t big_solve_lds_bytes(const Dims& d);

// Column-major lag twin of the X slabs (X = [1, lags 1..p of the slab's data columns], the
// linear and hybrid designs of mcmcVAR.m:62-72 / mcmcVARhybridGibbs.m:69-84): column a of slab x
// is pool + x * slab + off[a] (rows t = 0..TP-1; off[0] -> a column of ones, off[a >= K] -> a zero
// column).  The slab is (T + p) x (N [+ Ns] + 2) doubles instead of KP x TP, so the Gram and the
// solve read a working set that stays in L2.  pool == nullptr: read X itself.
struct ColX {
  const double* pool;
  const int* off;
  long long slab;
  int ld;    // leading dimension of a twin column (off[a] = column * ld + row offset)
  int ncol;  // columns per twin (data, actual rates, ones, zeros)
};

// groups: ngroups x int4 systems (c*N + j) sharing one design X slab (-1 padded);
// phase_mask: 1 Gram, 2 Cholesky, 4 solve.  Ubuf: B x N x TP scratch (U = E A');
// Dinv: nmat x (KP/64) x 64 x 64 inverses of the Cholesky factor's diagonal blocks.
hipError_t big_launch_cta(hipStream_t st, const Dims& d, const int* Tslot, const int* slotIV,
                          const double* iVdiag, const double* iVb, XSel xs, ChainState cs,
                          const int4* groups, int ngroups, double* rdiag, RngArgs ra, double* Ubuf,
                          double* Dinv, int phase_mask, ColX cx);

}  // namespace ccmm
