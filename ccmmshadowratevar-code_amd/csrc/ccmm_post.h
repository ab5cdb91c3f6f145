// Device post-processing of kept draws (ccmm_post.hip): gathers, segmented sort, summaries.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ccmm {

// workspace for post_summaries over S segments of n draws (sort temp storage + offsets)
size_t post_workspace_bytes(int S, int n);
// draws: device [S][n] (segment s contiguous); sorted: device [S][n] output of the sort;
// realized (device, S) may be null; pct (device, nq); outputs (device) may be null:
// mean/median/sd/crps [S], quant [nq][S]
hipError_t post_summaries(hipStream_t st, int S, int n, const double* draws, double* sorted, void* ws,
                          size_t ws_bytes, const double* realized, int nq, const double* pct, double* mean,
                          double* median, double* quant, double* sd, double* crps);
// forecast paths of chains chain0..chain0+C-1 (M kept records of Nd draws, H x N each, chain
// stride cap records) -> segments of rows[0..nr-1] x H (series r + nr h), cumulated over h
// for the variables with cum[i] != 0 (cum may be null), after flooring the variables with
// flo[i] != 0 at fl (flo may be null)
hipError_t post_gather_fcst(hipStream_t st, const double* src, int chain0, int C, int M, int Nd, int H, int N,
                            int cap, const int* rows, int nr, const uint8_t* cum, const uint8_t* flo, double fl,
                            double* dst);
// stored coefficient draws (KN values per record) -> segments of the KN entries
hipError_t post_gather_pai(hipStream_t st, const double* src, int chain0, int C, int M, int cap, int KN,
                           double* dst);

}  // namespace ccmm
