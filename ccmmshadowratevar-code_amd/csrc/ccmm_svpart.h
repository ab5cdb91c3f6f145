// Partitioned SV sampler (kernels in ccmm_svpart.hip, its own translation unit):
// buffer sizes and the host launcher used by ccmm_abi.hip.
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

constexpr int kSvMaxSeg = 16;  // segments of the partitioned order (oracle.sv_separators)

// matrices are padded to a bucket size NN >= N with identity blocks
inline int sv_bucket(int N) { return N <= 4 ? 4 : N <= 8 ? 8 : N <= 12 ? 12 : N <= 16 ? 16 : N <= 20 ? 20 : N <= 24 ? 24 : N <= 28 ? 28 : 32; }
// doubles per chain of the separator records
inline size_t sv_sep_len(int N) {
  const size_t NN = sv_bucket(N);
  return (kSvMaxSeg - 1) * (3 * NN * NN + 2 * NN);
}
// per-chain block factors C_t: (TP + 1) x NN x NN; w_t and the fill vectors g_t: (TP + 1) x NN
hipError_t sv_launch_part(int N, hipStream_t st, Dims d, const int* Tslot, const double* V0inv,
                          const double* V0invm, ChainState cs, RngArgs ra, double* sep, double* gbuf,
                          int mode, int nwg_opt, bool mfma);  // mode: timing-only phase skips (CCMM_SV_MODE)

}  // namespace ccmm
