// Internal definitions shared by the HIP kernels and the C-ABI host code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccmm.h"

namespace ccmm {

// ---------------------------------------------------------------- tiling
constexpr int kTChunk = 32;   // t-rows per SYRK K-step chunk; T is padded to a multiple
constexpr int kTile = 64;     // SYRK output tile (64 x 64, 4 waves of 32 x 32)
constexpr int kCholNB = 32;   // Cholesky panel width
constexpr int kMaxNSmall = 32;  // per-chain small-matrix kernels (A, SV, PHI) support N <= 32

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------- RNG
// Philox4x32-10 (Salmon et al. 2011), counter = (pair index, chain, sweep, block),
// key = 64-bit seed.  Two doubles per call; normals by Box-Muller.
constexpr int kRngBlocks = 9;  // CCMM_RNG_* ids 1..8

struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ inline uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// uniform in (0,1) from two 32-bit words (53 bits)
__host__ __device__ inline double u01(uint32_t lo, uint32_t hi) {
  uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
  return ((double)v + 0.5) * 1.1102230246251565404e-16;  // 2^-53
}

struct Rng {
  const double* crn;  // this chain's CRN base for this sweep (nullptr: Philox)
  uint64_t seed;
  uint32_t chain, sweep;
  int64_t off[kRngBlocks];  // CRN block offsets (indexed by CCMM_RNG_* id)

  __host__ __device__ inline u32x4 raw(int block, uint32_t pair) const {
    return philox4x32_10(u32x4{pair, chain, sweep, (uint32_t)block}, (uint32_t)seed,
                         (uint32_t)(seed >> 32));
  }
  __device__ inline double uniform(int block, uint32_t idx) const {
    if (crn) return crn[off[block] + idx];
    u32x4 r = raw(block, idx >> 1);
    return (idx & 1) ? u01(r.z, r.w) : u01(r.x, r.y);
  }
  __device__ inline double normal(int block, uint32_t idx) const {
    if (crn) return crn[off[block] + idx];
    u32x4 r = raw(block, idx >> 1);
    double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
    double rad = sqrt(-2.0 * log(u1));
    double s, c;
    sincospi(2.0 * u2, &s, &c);
    return (idx & 1) ? rad * s : rad * c;
  }
};

// ---------------------------------------------------------------- device views
// All matrices are column-major.  Per-slot data (vintages) and per-chain state
// use padded leading dimensions: TP (rows of T-dimension arrays), KP (rows of
// K-dimension arrays).  The chain index is the slowest dimension.
struct Dims {
  int N, p, K, KP, TP, B, nmat;  // nmat = B*N CTA systems
};

struct SlotData {
  const int* T;           // [ndata]
  const double* Y;        // [ndata][N][TP]
  const double* X;        // [ndata][KP][TP]   zero padded beyond (T, K)
  const double* iVdiag;   // [ndata][N][KP]    padded with 1
  const double* iVb;      // [ndata][N][KP]    padded with 0
  const double* sPHI;     // [ndata][N][N]
  const double* V0inv;    // [ndata][N][N]     (h0vcvsqrt h0vcvsqrt')^-1
  const double* V0invm;   // [ndata][N]        V0inv * h0mean
};

struct ChainState {
  const int* slot;   // [B]
  double* PAI;       // [B][N][KP]
  double* A;         // [B][N][N]
  double* invA;      // [B][N][N]
  double* sqrtht;    // [B][N][TP]
  double* h;         // [B][N][TP]
  double* sqrtPHI;   // [B][N][N]
  double* PHI;       // [B][N][N]
  double* E;         // [B][N][TP]  residual Y - X*PAI (RESID)
  double* logy2;     // [B][N][TP]
  double* eta;       // [B][N][TP]  SV shocks
  double* svobs;     // [B][N][TP]  logy2 - mean_{s}
  double* svir;      // [B][N][TP]  1/var_{s}
  int8_t* kai;       // [B][N][TP]
  double* W;         // [B][N][TP]  CTA weights
  double* ih2;       // [B][N][TP]  1 / sqrtht^2 (CTA weights kernel)
  double* G;         // [B*N][KP][KP]  Gram -> Cholesky factor (L lower, L' upper)
  double* svLd;      // [B][TP+1][N*N] block Cholesky diagonal factors
  double* svw;       // [B][TP+1][N]
  double* Zphi;      // [B][N][TZ]  IW normals scratch
  int* status;       // [B]
  // CTAsysAswitching (CTAsysAswitching.m:61-92): months with atELB[c][t] != 0 use the
  // second A matrix Aelb in the CTA weights and residual map; nullptr = CTA / CTAsys
  const double* Aelb;      // [B][N][N]
  const uint8_t* atELB;    // [B][TP]
};

// ---------------------------------------------------------------- shared device helpers
typedef double dbl4 __attribute__((ext_vector_type(4)));
// pointer into LDS (address space 3): loads/stores through it are ds_* instructions
typedef __attribute__((address_space(3))) double lds_f64;

struct XSel {
  const double* pool;  // slabs of KP x TP (X stored column-major, ld = TP)
  const int* idx;      // [B*N] slab of system (c, j)
  const double* ypool; // slabs of N x TP
  const int* yidx;     // [B] Y slab of chain c
};

struct RngArgs {
  const double* crn;       // CRN base for this sweep (chain 0) or nullptr
  int64_t crn_chain_stride;
  uint64_t seed;
  uint32_t sweep;
  int64_t off[kRngBlocks];
  const uint32_t* ids;     // Philox stream id of chain c (counter word 1), nullptr: c

  __device__ inline Rng make(int c) const {
    Rng r;
    r.crn = crn ? crn + (int64_t)c * crn_chain_stride : nullptr;
    r.seed = seed;
    r.chain = ids ? ids[c] : (uint32_t)c;
    r.sweep = sweep;
#pragma unroll
    for (int i = 0; i < kRngBlocks; ++i) r.off[i] = off[i];
    return r;
  }
};

// Hand-off of LDS data between the lanes of one wave: wavefront-scope release/acquire
// fences around the wave barrier, so that the compiler may not move or forward the LDS
// stores and loads across it (the barrier alone only orders instruction scheduling).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  union {
    double d;
    int i[2];
  } u;
  u.d = v;
  u.i[0] = __builtin_amdgcn_readlane(u.i[0], lane);
  u.i[1] = __builtin_amdgcn_readlane(u.i[1], lane);
  return u.d;
}

// Wave-wide sum returned uniformly, on the DPP path: xor-1 / xor-2 quad permutes, half-row
// and row mirrors leave every lane holding its 16-lane row sum, then four readlanes add
// the rows.  No LDS traffic (the __shfl_xor butterfly above is ds_bpermute per step), so
// it suits latency-bound serial loops.  Summation order differs from wave_sum.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  union {
    double d;
    int i[2];
  } u, r;
  u.d = v;
  r.i[0] = __builtin_amdgcn_update_dpp(0, u.i[0], CTRL, 0xF, 0xF, false);
  r.i[1] = __builtin_amdgcn_update_dpp(0, u.i[1], CTRL, 0xF, 0xF, false);
  return r.d;
}

// v + v[lane ^ 16] and v + v[lane ^ 32] by the gfx950 row swaps (VALU, no LDS round trip):
// a swap of a register with itself leaves the two partners in the two results
__device__ __forceinline__ double xsum16(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}
__device__ __forceinline__ double xsum32(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}

// 1 / sqrt(d) as a deterministic function of d's bits (restated bit for bit by oracle/cta_lag_mirror.c and
// oracle/cta_big_mirror.c): the integer seed 0x5fe6eb50c7b537a9 - (bits >> 1) (relative error <= 3.5 %)
// and two fourth-order steps r <- r + r e (1/2 + e (3/8 + 5/16 e)), e = 1 - d r^2 (error <= 1.4e-16
// over the double range).  The hardware v_rsq_f64 estimate cannot be reproduced off the device.
__device__ __forceinline__ double rsqrt_det(double d) {
  const long long bits = __double_as_longlong(d);
  double r = __longlong_as_double(0x5fe6eb50c7b537a9LL - (bits >> 1));
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double e = __builtin_fma(-(d * r), r, 1.0);
    const double q = __builtin_fma(__builtin_fma(0.3125, e, 0.375), e, 0.5);
    r = __builtin_fma(r * e, q, r);
  }
  return r;
}

__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// row-masked DPP move of a double: lanes of the rows outside ROWS read 0
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_rows_d(double v) {
  union {
    double d;
    int i[2];
  } u, r;
  u.d = v;
  r.i[0] = __builtin_amdgcn_update_dpp(0, u.i[0], CTRL, ROWS, 0xF, false);
  r.i[1] = __builtin_amdgcn_update_dpp(0, u.i[1], CTRL, ROWS, 0xF, false);
  return r.d;
}

// wave_sum_dpp of K independent values at once, stage by stage (the DPP hazards and add latencies of
// one value fill with the others' work), bit-identical to K calls: the same pairwise tree inside each
// row, and the cross-row combine (r0 + r1) + (r2 + r3) formed by row_bcast:15 into rows 1, 3 (r1 + r0,
// r3 + r2) and row_bcast:31 into rows 2, 3 (lane 63: (r3 + r2) + (r1 + r0)) -- the same roundings, as
// IEEE addition commutes -- and read from lane 63 (one readlane pair instead of four).
template <int K>
__device__ __forceinline__ void wave_sum_dpp_n(double (&v)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<0xB1>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<0x4E>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<0x141>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<0x140>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_rows_d<0x142, 0xA>(v[k]);  // row_bcast:15
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_rows_d<0x143, 0xC>(v[k]);  // row_bcast:31
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = readlane_d(v[k], 63);
}

// ---------------------------------------------------------------- kernel options (host)
// Choices between kernel forms and schedules are explicit options of a context or a chain set
// (ccmm_set_option / ccmm_chains_set_option, include/ccmm.h), never environment variables: a stray
// variable cannot change a run's draws or speed.  Schedules (kOptSchedule) give bit-identical draws;
// forms (kOptForm) the same algorithm in another summation order (or the QR branch of CTA.m:80-92).
// The ablation build (-DCCMM_ABLATION, libccmm_ablation.so) also takes each option's default from
// its CCMM_* variable for the timing tools; a default build reads none of them and names the ones set
// through ccmm_env_ignored().
enum OptId {
  OPT_SOLVE_SPLIT,  // k_cta_solve_lag on two workgroups per chain: -1 auto (B <= kSolveSplitMaxB and resident), 0, 1
  OPT_SOLVE_ASYNC,  // k_cta_solve_lag row-owned substitutions with LDS flags (1) or barrier-stepped (0)
  OPT_SV_NWG,       // k_sv_part workgroups per chain: 0 auto, 1, 2, 4
  OPT_ELB_WAVES,    // passes in flight per chain in k_elb_gibbs_wf: 1 (sequential k_elb_gibbs), 4, 8
  OPT_ELB_OCT,      // k_elb_gibbs_oct: 0 never, 1 from B >= kElbOctMinB, 2 always
  OPT_ELB_ASYNC,    // k_elb_gibbs_wf with per-wave progress flags (1) or lock-step barriers (0)
  OPT_ELB_PARTS,    // workgroups (CUs) per chain of the ELB wavefront: 0 auto, 1, 2, 4
  OPT_ELB_SPEC,     // speculative Gibbs step beside the PS branch at small B (1; measured neutral, off) or PS first (0)
  OPT_FCST_REG,     // k_fcst with the lag coefficients in registers (1) or PAI in LDS (0)
  OPT_FCST_OVERLAP, // kept sweeps' predictive density on the auxiliary stream beside the next sweep's CTA (1)
  OPT_PHI_OVERLAP,  // PHI block on the auxiliary stream beside the ELB step (1) or in stream order (0)
  OPT_QR_FALLBACK,  // host QR branch for a failed CTA Cholesky (CTA.m:80-92): 1 on, 0 off
  OPT_BIG_LAGX,     // large path: Gram and solve read the lag twin of a lag-structured X (1) or X itself (0)
  kOptSchedule,     // ---- forms below: same algorithm, other summation order / branch
  OPT_LAG = kOptSchedule,  // lag-structured CTA kernels when the design allows (1) or the generic path (0)
  OPT_LARGE_PATH,   // 1: the large-system CTA path for every shape (set before ccmm_chains_set_data)
  OPT_ASTEP_SERIAL, // 1: k_astep (one thread per regression) instead of k_astep_w
  OPT_PS_CHOL_LDS,  // 1: k_ps_chol (LDS window) instead of k_ps_chol_w
  OPT_SV_MFMA,      // k_sv_part phase-A products on MFMA (N <= 20 buckets): 1, or the FMA pass 0
  OPT_FORCE_QR,     // 1: every chain through the host QR branch of CTA.m:80-92
  OPT_GIRF_GENERIC, // 1: the table-driven GIRF kernel for the reference shape too
  kOptCount
};
struct OptDesc {
  const char* name;  // ccmm_set_option name
  const char* env;   // variable the ablation build reads as the default
  int dflt, lo, hi;
};
extern const OptDesc kOptDesc[kOptCount];
struct Options {
  int v[kOptCount];
  Options();  // defaults (ablation build: from the environment)
  int operator[](int i) const { return v[i]; }
};
int option_id(const char* name);  // -1 when unknown
// timing-only ablation variables (results invalid): read by the ablation build only; a default build
// returns `off` (the bits of keep_mask excepted) and reports the variable through ccmm_env_ignored()
int env_ablation(const char* name, int off, int keep_mask = 0);

// host CTA draw of one chain with the QR branch of CTA.m:80-92 (ccmm_host_cta.cpp)
int host_cta_chain(int N, int K, int T, const double* Y, int ldy, const double* const* Xs, int ldx,
                   const double* A, const double* sqrtht, int ldh, const double* iVdiag,
                   const double* iVb, int ldk, double* PAI, const double* z, bool force_qr,
                   const double* Aelb = nullptr, const uint8_t* atELB = nullptr);

}  // namespace ccmm
