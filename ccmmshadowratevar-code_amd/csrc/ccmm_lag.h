// Lag-structured CTA path (kernels in ccmm_lag.hip, its own translation unit):
// device views, LDS budgets and host launchers used by ccmm_abi.hip.
#pragma once
#include <algorithm>

#include "ccmm_internal.h"

namespace ccmm {

struct LagSel {
  const double* dpool;  // slabs of rows x ldd doubles, row-major; column ldd-1.. zero
  const int* idx;       // [B*N] D slab of CTA system (c, j)
  const int* colmap;    // [16*NT] offset of lag column a relative to row t (doubles)
  int ldd, rows, p;     // row stride (odd), rows per slab (TP + p), lag order
  int mode;             // timing-only ablation (CCMM_LAG_MODE, results invalid): gram 1 no SYRK,
                        // 2 no Cholesky; solve 16 no v, 32 no X'v, 64 no triangular
                        // substitutions, 128 no X x.  gram 8: write the raw SYRK stage (Gram tiles,
                        // b, c) and stop (ccmm_chains_get_cta_gram, parity tests)
};

// k_cta_solve_lag split over two workgroups per chain (small B): X'v half partials, [B][2 halves]
// [2 equation parities][256], and one progress flag per workgroup; part == nullptr: one workgroup
struct SolveXch {
  double* part;
  unsigned long long* flag;
  unsigned long long epoch;  // launch counter: equation j of this launch posts epoch * 64 + j + 1 (64 bits: no wrap)
};
constexpr int kSolveSplitMaxB = 64;

constexpr int kGlWaves = 8;
constexpr int kGlLd = 17;     // LDS row stride of a 16 x 16 tile
constexpr int kGlTile = 16 * kGlLd;

__host__ __device__ constexpr int gl_ntile(int NT) { return NT * (NT + 1) / 2; }
__host__ __device__ constexpr int gl_tpw(int NT) { return (gl_ntile(NT) + kGlWaves - 1) / kGlWaves; }
// tile (i, j), i >= j, in the column-major enumeration of the lower tiles
__host__ __device__ constexpr int gl_tile(int NT, int i, int j) { return j * NT - j * (j - 1) / 2 + (i - j); }
__host__ __device__ constexpr int gl_tj(int NT, int g) {
  int tj = 0;
  while (tj < NT && g >= NT - tj) {
    g -= NT - tj;
    ++tj;
  }
  return tj;
}
__host__ __device__ constexpr int gl_ti(int NT, int g) {
  int tj = 0;
  while (tj < NT && g >= NT - tj) {
    g -= NT - tj;
    ++tj;
  }
  return tj + g;
}
// output doubles per system
__host__ __device__ constexpr int gl_out_len(int NT) { return gl_ntile(NT) * 256 + 256; }
// LDS of k_gram_chol_lag: max(SYRK stage, factor stage)
inline size_t gl_lds_bytes(int NT, int rows, int ldd, int TP) {
  const size_t syrk = (size_t)rows * ldd + TP + 4;
  const size_t fac = 16 * NT + 8 + 64 + 2 * kGlTile + 2 * (size_t)NT * kGlTile + kGlWaves * kGlTile;
  return std::max(syrk, fac) * sizeof(double);
}

constexpr int kSlThreads = 512;

// LDS of k_cta_solve_lag: D | v + X'v partials | rl | xl | A | red | colmap
__host__ __device__ inline int sl_union(int NT, int TP) { return TP + 512; }
inline size_t sl_lds_bytes(int NT, int rows, int ldd, int TP, int nmax) {
  const size_t n = (size_t)rows * ldd + sl_union(NT, TP) + 256 + 256 + (size_t)nmax * nmax + 16;
  return n * sizeof(double) + (16 * NT + 32) * sizeof(int);  // colmap, then the RO hand-off flags
}

bool lag_supported_nt(int nt);
hipError_t lag_launch_gram(int NT, hipStream_t st, size_t lds, Dims d, const int* Tslot, LagSel ls,
                           ChainState cs, const double* iVdiag);
// workgroups of the solve kernel that can be resident at once on the device (occupancy x CUs)
int lag_solve_resident(int NT, int nmax, size_t lds, int async);
hipError_t lag_launch_solve(int NT, int nmax, int async, hipStream_t st, size_t lds, Dims d, const int* Tslot,
                            const double* iVb, XSel xs, LagSel ls, ChainState cs, RngArgs ra, SolveXch xc);

}  // namespace ccmm
