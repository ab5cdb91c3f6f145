// Kernel declarations and host-visible layouts of the per-sweep kernels of the generic (small-N) path:
// residuals, CTA weights, the A-step, the KSC indicators, PHI, the draw store and the drop-in helpers
// (ccmm_kernels.hip), the fused Gram + Cholesky (ccmm_gram_chol.hip) and the per-chain solve
// (ccmm_cta_solve.hip).  Each file is its own translation unit; ccmm_abi.hip launches the kernels.
#pragma once
#include "ccmm_internal.h"

namespace ccmm {

// ---------------------------------------------------------------- ccmm_gram_chol.hip
constexpr int kGcWaves = 8;
constexpr int kGcTC = 16;     // t rows per SYRK chunk
constexpr int kGcLdp = 17;    // LDS row stride of a 16 x 16 panel tile
// LDS row stride (doubles) of a Z chunk: 16 NT + 16, rows 32 banks apart (272 at NT = 16)
__host__ __device__ constexpr int gc_ldz(int NT) { return 16 * NT + 16; }
constexpr int kGcLdz = gc_ldz(16);

// column-major enumeration of the lower tiles of an NT x NT tile grid
__host__ __device__ constexpr int gc_tj(int NT, int g) {
  int tj = 0;
  while (tj < NT && g >= NT - tj) {
    g -= NT - tj;
    ++tj;
  }
  return tj;
}
__host__ __device__ constexpr int gc_ti(int NT, int g) {
  int tj = 0;
  while (tj < NT && g >= NT - tj) {
    g -= NT - tj;
    ++tj;
  }
  return tj + g;
}
__host__ __device__ constexpr int gc_tpw(int NT) { return (NT * (NT + 1) / 2 + kGcWaves - 1) / kGcWaves; }

struct GcArgs {
  const double* X;   // system's design, KP x TP column-major (ld TP)
  const double* w;   // sqrt weights, TP
  const double* iv;  // prior precision diagonal, KP
  double* L;         // KP x KP output
  double* rd;        // KP output
  int T, TP, KP;
  int mode;  // timing-only ablation (CCMM_GC_MODE): 1 no SYRK, 2 no Cholesky, 4 no trailing
             // update, 8 no panel solve, 16 no diagonal factor
};

template <int NT>
__global__ void k_gram_chol(Dims d, const int* __restrict__ Tslot, XSel xs, ChainState cs,
                            const double* __restrict__ iVdiag, double* __restrict__ rdiag, int mode);

// ---------------------------------------------------------------- ccmm_cta_solve.hip
constexpr int kSolveLd = 65;  // LDS row stride of the staged 64x64 diagonal block
template <int NMAX>
__global__ void k_cta_solve2(Dims d, const int* __restrict__ Tslot, const double* __restrict__ iVb, XSel xs,
                             ChainState cs, const double* __restrict__ rdiag, RngArgs ra);

// ---------------------------------------------------------------- ccmm_kernels.hip
// draw storage
struct Store {
  double* PAI;     // [B][cap][N][K]
  double* PHI;     // [B][cap][N(N+1)/2]
  double* invA;    // [B][cap][N][N]
  double* sqrtht;  // [B][cap][N][T]
  int cap, m, Tmax;
};

__global__ void k_resid(Dims d, const int* __restrict__ Tslot, XSel xs, ChainState cs);
template <int NB> __global__ void k_resid_multi(Dims d, const int* __restrict__ Tslot, XSel xs, ChainState cs);
__global__ void k_cta_weights(Dims d, const int* __restrict__ Tslot, ChainState cs, int sqrt_form);
__global__ void k_astep(Dims d, const int* __restrict__ Tslot, ChainState cs, RngArgs ra, double logy2offset,
                        int es_off, const int* __restrict__ gtab);
template <int NN>
__global__ void k_astep_w(Dims d, const int* __restrict__ Tslot, ChainState cs, RngArgs ra, double logy2offset,
                          int es_off, const int* __restrict__ gtab);
__global__ void k_sv_mix(Dims d, const int* __restrict__ Tslot, ChainState cs, RngArgs ra);
__global__ void k_phi_gen(Dims d, const int* __restrict__ Tslot, int dPHI, ChainState cs, RngArgs ra);
__global__ void k_phi(Dims d, const int* __restrict__ Tslot, int dPHI, const double* __restrict__ sPHIall,
                      ChainState cs, int stage_eta);
__global__ void k_store(Dims d, ChainState cs, Store st);
__global__ void k_pai_moments(const double* __restrict__ sPAI, int cap, int m0, int m1, int per, int B,
                              double* __restrict__ sum, double* __restrict__ sumsq);
__global__ void k_truncnorm(int n, const double* mu, const double* sig, double elb, const double* u, double* out,
                            uint8_t* flags);
__global__ void k_rng_normals(RngArgs ra, int c, int block, int n, double* __restrict__ out);
__global__ void k_mfma_selftest(const double* A, const double* B, double* D);
__global__ void k_mfma_selftest_acc(const double* A, const double* B, const double* C, double* D, int nprobe);

}  // namespace ccmm
