// Partitioned block-tridiagonal sampler of the SV log-variances, the device form of
// oracle/ccmm_oracle.sv_draw_partitioned (declared convention for the absent
// em-matlabbox StochVolKSCcorrsqrt, called at mcmcVAR.m:261,
// mcmcVARshadowrateBlockHybrid.m:379, mcmcVARhybridGibbs.m:405):
//
//   x = P^{-1} b + Pi' L^{-T} z,   x = [h_0; ...; h_T],   L = block Cholesky factor of
//   the posterior precision P in the partitioned order Pi (segment interiors in time
//   order, then the separators).
//
// The time-ordered factor is a Riccati recursion over all T + 1 blocks; here the
// dependency chain is one segment (~T/16 blocks) plus the separators (<= 15).
//
// One workgroup of NW waves per chain:
//   phase A  wave w eliminates segments w, w + NW, ... (time order inside a segment).
//            Per block: C_t = chol(D~_t) in row layout (lane i = row i, readlane
//            broadcasts, rsqrt + 2 Newton steps), w_t = C_t^{-1} b~_t, then
//            [X1 X2] = C_t^{-1} [-Q  M_{t,left}] with one right-hand column per lane,
//            and one uniform product pass over X in LDS gives, per lane group,
//              lanes 0..NN-1      rows of X1'X1 -> successor's Schur complement
//              lanes NN..2NN-1    columns of X1'X2 -> the next fill coupling
//              lanes 2NN..3NN-1   rows of X2'X2 -> the left separator's update
//   phase B  wave 0 eliminates the separators in time order.
//   phase C  wave 0 back-substitutes the separators; every wave then runs its
//            segments' fill recursion g (forward) and back substitution (backward),
//            writing h, sqrtht = exp(h/2) and the shocks h_t - h_{t-1}.
// Matrices are padded to NN (sv_bucket) with identity blocks; the padded
// coordinates decouple exactly and draw 0.  The diagonal of each stored C_t holds
// 1 / C_ii (only reciprocals are used in the substitutions).
#include "ccmm_svpart.h"

#include <algorithm>
#include <cstdlib>

namespace ccmm {

__host__ __device__ inline int sv_nseg(int T) {
  const int P = (T + 1) / 8;
  return P < 1 ? 1 : (P > kSvMaxSeg ? kSvMaxSeg : P);
}
// block index of separator i (0-based, i < P - 1)
__host__ __device__ inline int sv_sep(int i, int T, int P) { return ((i + 1) * (T + 1)) / P - 1; }

// per-wave LDS doubles: C (NN x NN+2), X (NN x 2NN+2), w (NN), fill columns, separator rows.  The
// row strides are even (NN is a multiple of 4), so every row starts 16-byte aligned and the
// substitutions and product passes read two entries per ds_read_b128
__host__ __device__ constexpr int sv_wave_lds(int NN) { return NN * (NN + 2) + NN * (2 * NN + 2) + NN + 2 * NN * NN; }
typedef double sv_d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) sv_d2 lds_d2;
__device__ __forceinline__ sv_d2 sv_ld2(const lds_f64* p) { return *(const lds_d2*)p; }

// v -= sum_{m<k} C(k, m) x_m in order m = 0..k-1 (row k of C at ro, 16-byte aligned), then
// x_k = v * C(k, k) (the stored reciprocal); entries read in pairs
template <int NN>
__device__ __forceinline__ double sv_row_solve(const lds_f64* myC, int ro, int k, const double (&x)[NN], double v) {
#pragma unroll
  for (int m = 0; m + 1 < k; m += 2) {
    const sv_d2 c2 = sv_ld2(myC + ro + m);
    v = fma(-c2.x, x[m], v);
    v = fma(-c2.y, x[m + 1], v);
  }
  double dk;
  if (k & 1) {
    const sv_d2 c2 = sv_ld2(myC + ro + k - 1);
    v = fma(-c2.x, x[k - 1], v);
    dk = c2.y;
  } else {
    dk = myC[ro + k];
  }
  return v * dk;
}

template <int NN>
struct SvRec {
  static constexpr int DR = 0;              // D(s) - X1'X1 of the left segment's last block
  static constexpr int DL = NN * NN;        // -sum X2'X2 of the right segment
  static constexpr int M = 2 * NN * NN;     // M[m*NN + r] = M_{s, s_next}[r][m]
  static constexpr int BR = 3 * NN * NN;    // b(s) - X1'w of the left segment's last block
  static constexpr int BL = 3 * NN * NN + NN;  // -sum X2'w of the right segment
  static constexpr int LEN = 3 * NN * NN + 2 * NN;
};

// 1/sqrt(d) to full precision: hardware estimate + two Newton steps
__device__ __forceinline__ double sv_rsqrt(double d) {
  double r = __builtin_amdgcn_rsq(d);
  const double hd = 0.5 * d;
  r = r * fma(-hd * r, r, 1.5);
  r = r * fma(-hd * r, r, 1.5);
  return r;
}

// LDS hand-off between the lanes of one wave: its LDS operations complete in order,
// so only the compiler has to be kept from moving accesses across this point
__device__ __forceinline__ void sv_wave_sync() {
  wave_lds_sync();
  asm volatile("" ::: "memory");
}

// An opaque copy of the lane id: lane masks derived from it are recomputed where they
// are used instead of being hoisted out of the block loops (dozens of loop-invariant
// 64-bit masks would otherwise spill the scalar file)
__device__ __forceinline__ int sv_lane(int lane) {
  int v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(lane));
  return v;
}

// An offset that the compiler must treat as computed after `dep` is known: the loads of
// a substitution row are then issued row by row instead of all ~NN^2/2 of them being
// hoisted to the top of the block (which spills hundreds of registers)
__device__ __forceinline__ int sv_after(int off, double dep, bool on) {
  if (on) asm volatile("" : "+v"(off) : "v"(dep));
  return off;
}

// Cholesky in row layout: lane i < NN holds row i of the SPD matrix in s[0..i];
// on return row i of the factor with 1 / C_ii on the diagonal (entries k > i are
// garbage) and rps = 1/diag (uniform)
template <int NN>
__device__ __forceinline__ void sv_chol_rows(double (&s)[NN], double (&rps)[NN], int lane0, int& bad) {
  const int lane = sv_lane(lane0);
  double dmin = 1.0;  // smallest pivot (a non-positive one flags the block; no per-pivot masks)
#pragma unroll
  for (int q = 0; q < NN; ++q) {
    double dq = readlane_d(s[q], q);
    dmin = fmin(dmin, dq);
    dq = fmax(dq, 1e-300);
    const double rp = sv_rsqrt(dq);
    rps[q] = rp;
    s[q] = (lane == q) ? rp : s[q] * rp;
#pragma unroll
    for (int k = q + 1; k < NN; ++k) s[k] = fma(-s[q], readlane_d(s[q], k), s[k]);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (!(dmin > 0.0)) bad = 1;
}

// L y = b, lane i holds b_i and row i of L (off-diagonal part)
template <int NN>
__device__ __forceinline__ double sv_fwd(double b, const double (&s)[NN], const double (&rps)[NN], int lane0) {
  const int lane = sv_lane(lane0);
#pragma unroll
  for (int k = 0; k < NN; ++k) {
    const double yk = readlane_d(b, k) * rps[k];
    b = (lane == k) ? yk : ((lane > k) ? fma(-s[k], yk, b) : b);
    __builtin_amdgcn_sched_barrier(0);
  }
  return b;
}

// L' x = r, lane i holds r_i and column i of L (lc[k] = L[k][i], k > i)
template <int NN>
__device__ __forceinline__ double sv_bwd(double r, const double (&lc)[NN], const double (&rps)[NN], int lane0) {
  const int lane = sv_lane(lane0);
#pragma unroll
  for (int k = NN - 1; k >= 0; --k) {
    const double xk = readlane_d(r, k) * rps[k];
    r = (lane == k) ? xk : ((lane < k) ? fma(-lc[k], xk, r) : r);
    __builtin_amdgcn_sched_barrier(0);
  }
  return r;
}

// The same two substitutions with the reciprocal diagonal held per lane (rd = 1 / C_ii on lane i):
// lane k's entry is scaled before the broadcast instead of after it (the same product), so the
// phase-C block loads need no uniform copy of the diagonal
template <int NN>
__device__ __forceinline__ double sv_fwd_d(double b, const double (&s)[NN], double rd, int lane0) {
  const int lane = sv_lane(lane0);
#pragma unroll
  for (int k = 0; k < NN; ++k) {
    const double yk = readlane_d(b * rd, k);
    b = (lane == k) ? yk : ((lane > k) ? fma(-s[k], yk, b) : b);
    __builtin_amdgcn_sched_barrier(0);
  }
  return b;
}
template <int NN>
__device__ __forceinline__ double sv_bwd_d(double r, const double (&lc)[NN], double rd, int lane0) {
  const int lane = sv_lane(lane0);
#pragma unroll
  for (int k = NN - 1; k >= 0; --k) {
    const double xk = readlane_d(r * rd, k);
    r = (lane == k) ? xk : ((lane < k) ? fma(-lc[k], xk, r) : r);
    __builtin_amdgcn_sched_barrier(0);
  }
  return r;
}

template <int NN, int NW, bool PACK, bool SVMFMA>
__global__ __launch_bounds__(64 * NW) void k_sv_part(Dims d, const int* __restrict__ Tslot,
                                                      const double* __restrict__ V0inv,
                                                      const double* __restrict__ V0invm, ChainState cs,
                                                      RngArgs ra, double* __restrict__ sepbuf,
                                                      double* __restrict__ gbuf, int mode, int nwg) {
  constexpr int CLD = NN + 2, XLD = 2 * NN + 2, NN2 = NN * NN;
  // phase A's block products on MFMA (NN = 20; option sv_mfma = 0 keeps the VALU pass)
  constexpr bool kSvMfma = NN == 20 && SVMFMA;
  constexpr bool G3 = 3 * NN <= 64;
  using R = SvRec<NN>;
  extern __shared__ double sm[];
  // explicit LDS address space: keeps every access a 32-bit ds_* op (generic pointers
  // captured by the lambdas below would otherwise become 64-bit flat addresses)
  lds_f64* Ql = (lds_f64*)sm;                        // NN x NN, Q = PHI^-1 (identity padding)
  lds_f64* Dz = Ql + NN2;                            // NN x NN, D0_0 = V0^-1 + Q
  lds_f64* xsep = Dz + NN2;                          // kSvMaxSeg x NN separator solutions
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  lds_f64* myC = xsep + kSvMaxSeg * NN + wave * sv_wave_lds(NN);
  lds_f64* myX = myC + NN * CLD;
  lds_f64* myw = myX + NN * XLD;
  lds_f64* myF = myw + NN;
  lds_f64* myD = myF + NN2;
  const int n = d.N, TP = d.TP;
  const int c = blockIdx.x, s = cs.slot[c], T = Tslot[s];
  const int wg = blockIdx.y;  // segment group of the chain (nwg > 1: phases A and C split over WGs)
  const int ln = lane < NN ? lane : 0;
  const bool real = lane < n;
  const double* sq = cs.sqrtPHI + (size_t)c * n * n;  // column-major lower n x n
  const double* obs = cs.svobs + (size_t)c * n * TP;
  const double* irv = cs.svir + (size_t)c * n * TP;
  double* Cg = cs.svLd + (size_t)c * (TP + 1) * NN2;  // [t][i*NN + k]
  double* Wg = cs.svw + (size_t)c * (TP + 1) * NN;
  double* rec = sepbuf + (size_t)c * (kSvMaxSeg - 1) * R::LEN;
  double* Gb = gbuf + (size_t)c * (TP + 1) * NN;
  double* Zg = gbuf + (size_t)(d.B + c) * (TP + 1) * NN;  // the chain's SV normals, block-major
  double* hout = cs.h + (size_t)c * n * TP;
  double* eta = cs.eta + (size_t)c * n * TP;
  double* sqh = cs.sqrtht + (size_t)c * n * TP;
  const double* V0 = V0inv + (size_t)s * n * n;
  const double* V0m = V0invm + (size_t)s * n;
  int bad = 0;

  // ---------------------------------------------------------------- Q = (sqrtPHI sqrtPHI')^-1
  if (wave == 0) {
    double li[NN];  // column `lane` of sqrtPHI^-1
#pragma unroll
    for (int r = 0; r < NN; ++r) {
      double v = (r == lane) ? 1.0 : 0.0;
      if (r < n && lane < n) {
#pragma unroll
        for (int q = 0; q < r; ++q) v = fma(-sq[r + q * n], li[q], v);
        v = (r >= lane) ? v / sq[r + r * n] : 0.0;
      }
      li[r] = v;
    }
    if (lane < NN) {
#pragma unroll
      for (int r = 0; r < NN; ++r) myX[r * XLD + lane] = li[r];
    }
    sv_wave_sync();
    if (lane < NN) {
#pragma unroll
      for (int r = 0; r < NN; ++r) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < NN; ++q) v = fma(myX[q * XLD + r], li[q], v);
        Ql[r * NN + lane] = v;
      }
    }
    sv_wave_sync();
    if (lane < NN) {  // D0_0 row `lane` (identity on the padding)
#pragma unroll
      for (int m = 0; m < NN; ++m)
        Dz[lane * NN + m] = ((lane < n && m < n) ? V0[lane + m * n] : (m == lane ? 1.0 : 0.0)) +
                            Ql[lane * NN + m];
    }
  }
  __syncthreads();

  const int P = sv_nseg(T);
  // original diagonal block D0_t, row ln, entry m (irt = diag(R_t^-1) entry of row ln)
  auto d0 = [&](int t, int m, double irt) __attribute__((always_inline)) -> double {
    const int lv = sv_lane(ln);
    if (t == 0) return Dz[ln * NN + m];
    return ((t == T) ? 1.0 : 2.0) * Ql[ln * NN + m] + ((m == lv) ? irt : 0.0);
  };
  // the same for t >= 1 (no prior block)
  auto d0n = [&](int t, int m, double irt) __attribute__((always_inline)) -> double {
    const int lv = sv_lane(ln);
    return ((t == T) ? 1.0 : 2.0) * Ql[ln * NN + m] + ((m == lv) ? irt : 0.0);
  };
  auto ir_at = [&](int t) __attribute__((always_inline)) -> double { return (t >= 1 && real) ? irv[(size_t)ln * TP + t - 1] : 1.0; };
  auto ob_at = [&](int t) __attribute__((always_inline)) -> double { return (t >= 1 && real) ? obs[(size_t)ln * TP + t - 1] : 0.0; };
  auto b0 = [&](int t, double irt, double obt) __attribute__((always_inline)) -> double {
    if (t == 0) return real ? V0m[ln] : 0.0;
    return real ? obt * irt : 0.0;
  };
  // the normals z_t (block t, row ln) are drawn grid-wide by k_sv_normals before this
  // kernel (independent work off the per-chain serial path) and read back from Zg
  auto zdraw = [&](int t) __attribute__((always_inline)) -> double {
    if (mode & 32) return 0.0;  // timing ablation only
    return real ? Zg[(size_t)t * NN + ln] : 0.0;
  };
  // C_t row (lane < NN) -> LDS, and its lower triangle packed by rows to HBM
  // (Ct[i (i + 1) / 2 + m], m <= i), the diagonal as its reciprocal
  auto store_factor = [&](int t, const double (&sr)[NN], const double (&rps)[NN], double w)
                          __attribute__((always_inline)) {
    if (lane < NN) {
#pragma unroll
      for (int m = 0; m < NN; ++m) myC[lane * CLD + m] = sr[m];
      myw[lane] = w;
      Wg[(size_t)t * NN + lane] = w;
    }
  };
  // packed entry e -> its LDS offset row * CLD + col (rows of the lower triangle, or full rows)
  auto unpack_at = [&](int e) __attribute__((always_inline)) -> int {
    if (!PACK) return (e / NN) * CLD + (e % NN);
    int r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
    r += ((r + 1) * (r + 2)) / 2 <= e ? 1 : 0;
    r -= (r * (r + 1)) / 2 > e ? 1 : 0;
    return r * CLD + (e - (r * (r + 1)) / 2);
  };
  constexpr int NP = PACK ? NN * (NN + 1) / 2 : NN * NN;
  constexpr int kST = (NP + 63) / 64;
  // the factor of block t leaves the wave's LDS copy for HBM as kST coalesced 64-lane
  // stores (after the sv_wave_sync that follows store_factor)
  auto flush_factor = [&](int t) __attribute__((always_inline)) {
    double* Ct = Cg + (size_t)t * NN2;
#pragma unroll
    for (int i = 0; i < kST; ++i) {
      const int e = lane + 64 * i;
      if (e < NP) Ct[e] = myC[unpack_at(e)];
    }
  };

  // ---------------------------------------------------------------- phase A: segments
  // per-wave LDS: myF[k*NN + r] fill column r of M_{t,left} (right-hand side of lane NN+r),
  // myD[r*NN + m] the left separator's accumulated -sum X2'X2 (row r)
  for (int q = wave + NW * wg; q < ((mode & 1) ? 0 : P); q += NW * nwg) {
    const int first = (q == 0) ? 0 : sv_sep(q - 1, T, P) + 1;
    const int last = (q == P - 1) ? T : sv_sep(q, T, P) - 1;
    const bool hasL = q > 0, hasR = q < P - 1;
    const int rB = lane - NN, rD = G3 ? lane - 2 * NN : lane - NN;  // group B column, group C/D row
    const bool inB = rB >= 0 && rB < NN, inD = rD >= 0 && rD < NN;
    double sr[NN];
    double dbl = 0.0, bcur;
    {
      const double irt = ir_at(first), obt = ob_at(first);
#pragma unroll
      for (int m = 0; m < NN; ++m) sr[m] = d0(first, m, irt);
      if (inB) {
#pragma unroll
        for (int k = 0; k < NN; ++k) myF[k * NN + rB] = -Ql[k * NN + rB];  // M_{first,left} = -Q
      }
      if (inD) {
#pragma unroll
        for (int m = 0; m < NN; ++m) myD[rD * NN + m] = 0.0;
      }
      bcur = b0(first, irt, obt);
    }
    sv_wave_sync();
    for (int t = first; t <= last; ++t) {
      const bool hasN = t < T;
      const double irn = hasN ? ir_at(t + 1) : 1.0, obn = hasN ? ob_at(t + 1) : 0.0;
      {
        double rps[NN];
        sv_chol_rows<NN>(sr, rps, lane, bad);
        const double w = sv_fwd<NN>(bcur, sr, rps, lane);
        store_factor(t, sr, rps, w);
      }
      sv_wave_sync();
      flush_factor(t);
      // [X1 X2] = C^-1 [-Q  M_{t,left}], one right-hand column per lane (the diagonal
      // of myC holds 1 / C_kk)
      {
        const int rcol = (lane < NN) ? lane : (inB ? rB : 0);
        const lds_f64* rhs = (lane < NN) ? Ql : myF;
        const double sgn = (lane < NN) ? -1.0 : 1.0;
        double x[NN];
#pragma unroll
        for (int k = 0; k < NN; ++k) {
          // row k's factor entries are read once x[k - 2] is known, i.e. while row k - 1 is being
          // solved (one row in flight ahead: the LDS latency leaves the serial chain)
          const int ro = sv_after(k * CLD, x[k > 1 ? k - 2 : 0], k > 1);
          x[k] = sv_row_solve<NN>(myC, ro, k, x, sgn * rhs[k * NN + rcol]);
        }
        if (lane < 2 * NN) {
#pragma unroll
          for (int k = 0; k < NN; ++k) myX[k * XLD + lane] = x[k];
        }
      }
      sv_wave_sync();
      double pr[NN];
      double wd = 0.0;
      if constexpr (kSvMfma) {
        // NN = 20: the three 20 x 20 blocks X1'X1, X2'X1, X2'X2 are blocks of the Gram X'X of the
        // 20 x 40 block [X1 X2]: six lower 16 x 16 tiles of it on v_mfma_f64_16x16x4_f64 (fragment
        // F(I, s) = X[4s + l/16][16I + l%16], columns >= 40 zero), written as the row blocks the lane
        // groups read -- P1 = G(:, 0:20) (40 x 20) and P2 = G(20:40, 20:40) -- over the wave's C and
        // X area (both dead until the next block).  w'X: each column's own sum (k in order), lanes
        // 2NN.. take column lane - NN's.
        {
          double wo = 0.0;
#pragma unroll
          for (int k = 0; k < NN; k += 2) {
            const sv_d2 w2 = sv_ld2(myw + k);
            wo = fma(myX[k * XLD + (lane < 2 * NN ? lane : 0)], w2.x, wo);
            wo = fma(myX[(k + 1) * XLD + (lane < 2 * NN ? lane : 0)], w2.y, wo);
          }
          const double wsh = __shfl(wo, (lane >= 2 * NN && lane < 3 * NN) ? lane - NN : lane, 64);
          wd = (lane >= 2 * NN && lane < 3 * NN) ? wsh : wo;
        }
        const int lr = lane & 15, lk = lane >> 4;
        double F[3][5];
#pragma unroll
        for (int I = 0; I < 3; ++I)
#pragma unroll
          for (int s5 = 0; s5 < 5; ++s5) {
            const int col = 16 * I + lr;
            F[I][s5] = (col < 2 * NN) ? myX[(4 * s5 + lk) * XLD + col] : 0.0;
          }
        dbl4 g[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) g[q] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s5 = 0; s5 < 5; ++s5) {
          g[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[0][s5], F[0][s5], g[0], 0, 0, 0);
          g[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[1][s5], F[0][s5], g[1], 0, 0, 0);
          g[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[1][s5], F[1][s5], g[2], 0, 0, 0);
          g[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[2][s5], F[0][s5], g[3], 0, 0, 0);
          g[4] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[2][s5], F[1][s5], g[4], 0, 0, 0);
          g[5] = __builtin_amdgcn_mfma_f64_16x16x4f64(F[2][s5], F[2][s5], g[5], 0, 0, 0);
        }
        sv_wave_sync();  // every fragment read before the C / X area is overwritten
        lds_f64* P1 = myC;                   // 40 x 20
        lds_f64* P2 = myC + 2 * NN * NN;     // 20 x 20
        constexpr int TI[6] = {0, 1, 1, 2, 2, 2}, TJ[6] = {0, 0, 1, 0, 1, 2};
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int a = 16 * TI[q] + lk + 4 * r, b = 16 * TJ[q] + lr;  // D(row a, col b)
            const double v = g[q][r];
            if (a < 2 * NN && b < 2 * NN) {
              if (b < NN) P1[a * NN + b] = v;
              else if (a >= NN) P2[(a - NN) * NN + (b - NN)] = v;
              if (TI[q] != TJ[q]) {  // the transposed entry (b, a), a > b
                if (a < NN) P1[b * NN + a] = v;
                else if (b >= NN) P2[(b - NN) * NN + (a - NN)] = v;
              }
            }
          }
        sv_wave_sync();
        const lds_f64* prow = (lane < 2 * NN) ? P1 + lane * NN : P2 + (lane < 3 * NN ? lane - 2 * NN : 0) * NN;
#pragma unroll
        for (int m = 0; m < NN; m += 2) {
          const sv_d2 p2 = sv_ld2(prow + m);
          pr[m] = p2.x;
          pr[m + 1] = p2.y;
        }
      } else {
        // one uniform product pass: pr[m] = sum_k a[k] X[k][m + boff], a = own column
        // (lanes < 2NN) or the X2 column of lane - NN (lanes 2NN..3NN-1)
        const int boff = (lane < 2 * NN) ? 0 : NN;
        const int acol = (lane < 2 * NN) ? lane : ((lane < 3 * NN) ? lane - NN : NN);
#pragma unroll
        for (int m = 0; m < NN; ++m) pr[m] = 0.0;
#pragma unroll 1
        for (int k = 0; k < NN; ++k) {
          const lds_f64* xr = myX + k * XLD;
          const double ak = xr[acol];
#pragma unroll
          for (int m = 0; m < NN; m += 2) {
            const sv_d2 b2 = sv_ld2(xr + boff + m);
            pr[m] = fma(ak, b2.x, pr[m]);
            pr[m + 1] = fma(ak, b2.y, pr[m + 1]);
          }
          wd = fma(ak, myw[k], wd);
        }
      }
      // epilogue, uniform over the lanes (each lane group keeps only its own values):
      //   lanes 0..NN-1:    successor's D~ row / b~ entry (after the last block of a
      //                     segment with a right separator: that separator's record)
      //   lanes NN..2NN-1:  next fill column M_{t+1,left}(:, r) = -(X2'X1)(r, :)'
      //   lanes 2NN..3NN-1: left separator's -sum X2'X2 row
#pragma unroll
      for (int m = 0; m < NN; ++m) sr[m] = d0n(t + 1, m, irn) - pr[m];
      bcur = (real ? obn * irn : 0.0) - wd;
      if (hasL) {
        if (inB) {
#pragma unroll
          for (int m = 0; m < NN; ++m) myF[m * NN + rB] = -pr[m];
          dbl -= wd;
        }
        if (G3 && inD) {
#pragma unroll
          for (int m = 0; m < NN; ++m) myD[rD * NN + m] -= pr[m];
        }
      }
      if constexpr (!G3) {  // 3 NN > 64: X2'X2 rows on lanes NN..2NN-1 in a second pass
        if (hasL) {
#pragma unroll
          for (int m = 0; m < NN; ++m) pr[m] = 0.0;
#pragma unroll 1
          for (int k = 0; k < NN; ++k) {
            const lds_f64* xr = myX + k * XLD;
            const double ak = xr[(lane < 2 * NN) ? lane : NN];  // own column (lanes < 2NN)
#pragma unroll
            for (int m = 0; m < NN; m += 2) {
              const sv_d2 b2 = sv_ld2(xr + NN + m);
              pr[m] = fma(ak, b2.x, pr[m]);
              pr[m + 1] = fma(ak, b2.y, pr[m + 1]);
            }
          }
          if (inD) {
#pragma unroll
            for (int m = 0; m < NN; ++m) myD[rD * NN + m] -= pr[m];
          }
        }
      }
      sv_wave_sync();
    }
    sv_wave_sync();
    if (hasR) {  // the right separator: D(s) - X1'X1, b(s) - X1'w of the last block
      double* r = rec + (size_t)q * R::LEN;
      if (lane < NN) {
#pragma unroll
        for (int m = 0; m < NN; ++m) r[R::DR + lane * NN + m] = sr[m];
        r[R::BR + lane] = bcur;
      }
      if (hasL && inB) {  // coupling M_{left,right}: rec.M[m*NN + r] = M[r][m]
        double* rl = rec + (size_t)(q - 1) * R::LEN;
        for (int m = 0; m < NN; ++m) rl[R::M + m * NN + rB] = myF[m * NN + rB];
      }
    }
    if (hasL) {
      double* r = rec + (size_t)(q - 1) * R::LEN;
      if (inB) r[R::BL + rB] = dbl;
      if (inD) {
#pragma unroll
        for (int m = 0; m < NN; ++m) r[R::DL + rD * NN + m] = myD[rD * NN + m];
      }
    }
    sv_wave_sync();
  }
  __syncthreads();

  // ---------------------------------------------------------------- phase B: separators
  if (wave == 0 && P > 1 && !(mode & 2)) {
    double cg[NN], sr[NN];
#pragma unroll
    for (int m = 0; m < NN; ++m) cg[m] = 0.0;
    double cb = 0.0;
    for (int i = 0; i < P - 1; ++i) {
      const int sb = sv_sep(i, T, P);
      const double* r = rec + (size_t)i * R::LEN;
#pragma unroll
      for (int m = 0; m < NN; ++m)
        sr[m] = (lane < NN) ? r[R::DR + ln * NN + m] + r[R::DL + ln * NN + m] - cg[m] : 0.0;
      const double bcur = (lane < NN) ? r[R::BR + ln] + r[R::BL + ln] - cb : 0.0;
      {
        double rps[NN];
        sv_chol_rows<NN>(sr, rps, lane, bad);
        const double w = sv_fwd<NN>(bcur, sr, rps, lane);
        store_factor(sb, sr, rps, w);
      }
      sv_wave_sync();
      flush_factor(sb);
      if (i + 1 < P - 1) {
        // X1 = C^-1 M_{sep i, sep i+1}: column `lane` of M is r[M + lane*NN + k]
        double x[NN];
#pragma unroll
        for (int k = 0; k < NN; ++k) {
          const int ro = sv_after(k * CLD, x[k > 0 ? k - 1 : 0], k > 0);
          x[k] = sv_row_solve<NN>(myC, ro, k, x, (lane < NN) ? r[R::M + ln * NN + k] : 0.0);
        }
        if (lane < NN) {
#pragma unroll
          for (int k = 0; k < NN; ++k) myX[k * XLD + lane] = x[k];
        }
        sv_wave_sync();
#pragma unroll
        for (int m = 0; m < NN; ++m) cg[m] = 0.0;
        cb = 0.0;
#pragma unroll 1
        for (int k = 0; k < NN; ++k) {
          const lds_f64* xr = myX + k * XLD;
          const double ak = xr[ln];
#pragma unroll
          for (int m = 0; m < NN; m += 2) {
            const sv_d2 b2 = sv_ld2(xr + m);
            cg[m] = fma(ak, b2.x, cg[m]);
            cg[m + 1] = fma(ak, b2.y, cg[m + 1]);
          }
          cb = fma(ak, myw[k], cb);
        }
      }
      sv_wave_sync();
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- phase C: back substitution
  // (the normals z_t were drawn into Zg by k_sv_normals before this kernel)
  double qrow[NN];
#pragma unroll
  for (int m = 0; m < NN; ++m) qrow[m] = Ql[ln * NN + m];
  // C_t -> LDS (whole wave), then row / column / reciprocal diagonal per lane
  // row ln (entry pairs), column ln and the lane's own reciprocal diagonal of the block in LDS
  auto read_factor = [&](double (&lr)[NN], double (&lc)[NN], double& rd) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < NN; m += 2) {
      const sv_d2 r2 = sv_ld2(myC + ln * CLD + m);
      lr[m] = r2.x;
      lr[m + 1] = r2.y;
    }
#pragma unroll
    for (int m = 0; m < NN; ++m) lc[m] = myC[m * CLD + ln];
    rd = myC[ln * CLD + ln];
  };
  auto load_factor = [&](int t, double (&lr)[NN], double (&lc)[NN], double& rd) __attribute__((always_inline)) {
    const double* Ct = Cg + (size_t)t * NN2;
    for (int e = lane; e < NP; e += 64) myC[unpack_at(e)] = Ct[e];
    sv_wave_sync();
    read_factor(lr, lc, rd);
    sv_wave_sync();
  };
  // software-pipelined form (NN <= 20): the next block's factor is fetched into registers
  // (kPF per lane) while the current block's substitutions run, so the serial block loops
  // of phase C no longer wait a full HBM latency per block
  constexpr bool kPipe = NN <= 20;
  constexpr int kPF = kPipe ? (NP + 63) / 64 : 1;
  int upk[kPF];  // unpacked LDS offsets of this lane's packed entries
#pragma unroll
  for (int i = 0; i < kPF; ++i) upk[i] = unpack_at(min(lane + 64 * i, NP - 1));
  auto fetch_factor = [&](int t, double (&pf)[kPF]) __attribute__((always_inline)) {
    const double* Ct = Cg + (size_t)t * NN2;
#pragma unroll
    for (int i = 0; i < kPF; ++i) {
      const int e = lane + 64 * i;
      pf[i] = (e < NP) ? __builtin_nontemporal_load(Ct + e) : 0.0;
    }
  };
  auto commit_factor = [&](const double (&pf)[kPF], double (&lr)[NN], double (&lc)[NN], double& rd)
                           __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kPF; ++i)
      if (lane + 64 * i < NP) myC[upk[i]] = pf[i];
    sv_wave_sync();
    read_factor(lr, lc, rd);
    sv_wave_sync();
  };
  if (wave == 0 && P > 1 && !(mode & 4)) {
    for (int i = P - 2; i >= 0; --i) {
      const int sb = sv_sep(i, T, P);
      double lr[NN], lc[NN], rd;
      load_factor(sb, lr, lc, rd);
      double rv = (lane < NN) ? Wg[(size_t)sb * NN + ln] + zdraw(sb) : 0.0;
      if (i + 1 < P - 1) {
        const double* Mr = rec + (size_t)i * R::LEN + R::M;  // row ln of M: Mr[m*NN + ln]
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < NN; ++m) acc = fma(Mr[m * NN + ln], xsep[(i + 1) * NN + m], acc);
        rv -= sv_fwd_d<NN>(acc, lr, rd, lane);
      }
      const double x = sv_bwd_d<NN>(rv, lc, rd, lane);
      if (lane < NN) xsep[i * NN + lane] = x;
      if (real) {
        hout[(size_t)ln * TP + sb - 1] = x;
        sqh[(size_t)ln * TP + sb - 1] = exp(0.5 * x);
      }
      sv_wave_sync();
    }
  }
  __syncthreads();
  for (int q = wave + NW * wg; q < ((mode & 8) ? 0 : P); q += NW * nwg) {
    const int first = (q == 0) ? 0 : sv_sep(q - 1, T, P) + 1;
    const int last = (q == P - 1) ? T : sv_sep(q, T, P) - 1;
    const bool hasL = q > 0, hasR = q < P - 1;
    if (hasL && !(mode & 16)) {  // g_first = -Q x_left, g_{t+1} = Q C_t^-T C_t^-1 g_t
      double g = 0.0;
#pragma unroll
      for (int m = 0; m < NN; ++m) g = fma(-qrow[m], xsep[(q - 1) * NN + m], g);
      double pf[kPF];
      if (kPipe && first < last) fetch_factor(first, pf);
      for (int t = first; t <= last; ++t) {
        if (lane < NN) Gb[(size_t)t * NN + lane] = g;
        if (t < last) {
          double lr[NN], lc[NN], rd;
          if constexpr (kPipe) {
            commit_factor(pf, lr, lc, rd);
            if (t + 1 < last) fetch_factor(t + 1, pf);
          } else {
            load_factor(t, lr, lc, rd);
          }
          double v = sv_fwd_d<NN>(g, lr, rd, lane);
          v = sv_bwd_d<NN>(v, lc, rd, lane);
          if (lane < NN) myw[lane] = v;
          sv_wave_sync();
          g = 0.0;
#pragma unroll
          for (int m = 0; m < NN; m += 2) {
            const sv_d2 w2 = sv_ld2(myw + m);
            g = fma(qrow[m], w2.x, g);
            g = fma(qrow[m + 1], w2.y, g);
          }
          sv_wave_sync();
        }
      }
    }
    // successor of `last`: the right separator (x known) or nothing (t == T)
    if (hasR && lane < NN) myw[lane] = xsep[q * NN + lane];
    sv_wave_sync();
    double pfb[kPF];
    if (kPipe) fetch_factor(last, pfb);
    for (int t = last; t >= first; --t) {
      double lr[NN], lc[NN], rd;
      if constexpr (kPipe) {
        commit_factor(pfb, lr, lc, rd);
        if (t > first) fetch_factor(t - 1, pfb);
      } else {
        load_factor(t, lr, lc, rd);
      }
      double acc = 0.0, xn = 0.0;
      if (t < T) {
#pragma unroll
        for (int m = 0; m < NN; m += 2) {
          const sv_d2 w2 = sv_ld2(myw + m);
          acc = fma(-qrow[m], w2.x, acc);
          acc = fma(-qrow[m + 1], w2.y, acc);
        }
        xn = myw[ln];
      }
      if (hasL && lane < NN) acc += Gb[(size_t)t * NN + ln];
      double rv = (lane < NN) ? Wg[(size_t)t * NN + ln] + zdraw(t) : 0.0;
      double x;
      if (mode & 64) {  // timing ablation only
        x = rv - acc;
      } else {
        rv -= sv_fwd_d<NN>(acc, lr, rd, lane);
        x = sv_bwd_d<NN>(rv, lc, rd, lane);
      }
      if (real) {
        if (t >= 1) {
          hout[(size_t)ln * TP + t - 1] = x;
          sqh[(size_t)ln * TP + t - 1] = exp(0.5 * x);
        }
        if (t < T) eta[(size_t)ln * TP + t] = xn - x;          // shock of block t + 1
        if (t == first && hasL) eta[(size_t)ln * TP + t - 1] = x - xsep[(q - 1) * NN + ln];
      }
      sv_wave_sync();
      if (lane < NN) myw[lane] = x;
      sv_wave_sync();
    }
  }
  // padding beyond T
  for (int e = wg == 0 ? tid : n * (TP - T); e < n * (TP - T); e += 64 * NW) {
    const int r = e / (TP - T), t = T + e % (TP - T);
    hout[(size_t)r * TP + t] = 0.0;
    eta[(size_t)r * TP + t] = 0.0;
    sqh[(size_t)r * TP + t] = 1.0;
  }
  if (bad && lane == 0) atomicOr(&cs.status[c], 8);
}

// randn(N, T+1) of every chain (CCMM_RNG_SVZ; CRN: the host block) -> Zg, block-major
// [t][NN]: drawn by the whole GPU ahead of k_sv_part instead of inside its serial chain
__global__ void k_sv_normals(Dims d, const int* __restrict__ Tslot, ChainState cs, RngArgs ra, double* gbuf,
                             int NN) {
  const int c = blockIdx.y;
  const int n = d.N, T = Tslot[cs.slot[c]];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (T + 1) * n) return;
  const int t = e / n, i = e - t * n;
  const Rng rng = ra.make(c);
  gbuf[(size_t)(d.B + c) * (d.TP + 1) * NN + (size_t)t * NN + i] = rng.normal(CCMM_RNG_SVZ, (uint32_t)(i + n * t));
}

template <int NN, int NW, bool PACK, bool MF>
static hipError_t sv_launch_k(hipStream_t st, Dims d, const int* Tslot, const double* V0inv,
                              const double* V0invm, ChainState cs, RngArgs ra, double* sep, double* gbuf,
                              int mode, int nwg) {
  const size_t lds = (size_t)(2 * NN * NN + kSvMaxSeg * NN + NW * sv_wave_lds(NN)) * sizeof(double);
  hipError_t e = hipFuncSetAttribute((const void*)k_sv_part<NN, NW, PACK, MF>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_sv_normals, dim3(((d.TP + 1) * d.N + 255) / 256, d.B), dim3(256), 0, st, d, Tslot, cs, ra,
                     gbuf, NN);
  // small batches (B <= 128, e.g. the OOS chains of one vintage): the segments of phases A and C
  // are spread over nwg = 2 (or 4) workgroups per chain (16 segments = one per wave), as two
  // launches: phase A, then phases B + C, in which every workgroup of the chain redoes the serial
  // separator pass (identical values and stores) instead of a third launch; same draws
  if (nwg == 1) {
    hipLaunchKernelGGL((k_sv_part<NN, NW, PACK, MF>), dim3(d.B), dim3(64 * NW), lds, st, d, Tslot, V0inv, V0invm,
                       cs, ra, sep, gbuf, mode, 1);
  } else {
    hipLaunchKernelGGL((k_sv_part<NN, NW, PACK, MF>), dim3(d.B, nwg), dim3(64 * NW), lds, st, d, Tslot, V0inv,
                       V0invm, cs, ra, sep, gbuf, mode | 2 | 4 | 8, nwg);
    hipLaunchKernelGGL((k_sv_part<NN, NW, PACK, MF>), dim3(d.B, nwg), dim3(64 * NW), lds, st, d, Tslot, V0inv,
                       V0invm, cs, ra, sep, gbuf, mode | 1, nwg);
  }
  return hipGetLastError();
}

// NN = 20: phase A's block products on MFMA unless option sv_mfma = 0 (mode bit 256 here): a different
// accumulation order than the FMA pass, so the two forms agree to rounding, not bit for bit
template <int NN, int NW, bool PACK>
static hipError_t sv_launch_one_(hipStream_t st, Dims d, const int* Tslot, const double* V0inv,
                                const double* V0invm, ChainState cs, RngArgs ra, double* sep, double* gbuf,
                                int mode, int nwg) {
  if constexpr (NN == 20) {
    if (mode & 256)
      return sv_launch_k<NN, NW, PACK, false>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode & ~256, nwg);
  }
  return sv_launch_k<NN, NW, PACK, true>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
}

// block factors stored as packed lower triangles (default: 0.55x the factor traffic of full rows,
// and no register spills at NN = 20; measured 2.16 vs 2.19 ms at N = 20, B = 256 since the factor
// leaves LDS by coalesced stores) or as full rows (mode bit 128, for comparison); same draws
template <int NN, int NW>
static hipError_t sv_launch_one(hipStream_t st, Dims d, const int* Tslot, const double* V0inv,
                                const double* V0invm, ChainState cs, RngArgs ra, double* sep, double* gbuf,
                                int mode, int nwg) {
  if (mode & 128) return sv_launch_one_<NN, NW, false>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
  return sv_launch_one_<NN, NW, true>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
}

// Workgroups per chain: 1 from B = 129 (the chip is full), 2 of 8 waves down to B = 33, and at
// B <= 32 (NN <= 20) 4 of 4 waves -- one wave per SIMD on 4 CUs, so that the serial block chains of
// phases A and C no longer share a SIMD's issue (the OOS floor runs one chain).  Option sv_nwg = 1|2|4
// overrides.  The segments, their order of operations and the draws are the same in every layout.
hipError_t sv_launch_part(int N, hipStream_t st, Dims d, const int* Tslot, const double* V0inv,
                          const double* V0invm, ChainState cs, RngArgs ra, double* sep, double* gbuf, int mode,
                          int nwg_opt, bool mfma) {
  const int nb = sv_bucket(N);
  int nwg = d.B <= 32 && nb <= 20 ? 4 : (d.B <= 128 ? 2 : 1);
  if (nwg_opt > 0) nwg = nwg_opt >= 4 && nb <= 20 ? 4 : std::max(1, std::min(2, nwg_opt));
  if (!mfma) mode |= 256;
  if (nwg == 4) {
    switch (nb) {
      case 4: return sv_launch_one<4, 4>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, 4);
      case 8: return sv_launch_one<8, 4>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, 4);
      case 12: return sv_launch_one<12, 4>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, 4);
      case 16: return sv_launch_one<16, 4>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, 4);
      default: return sv_launch_one<20, 4>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, 4);
    }
  }
  switch (nb) {
    case 4: return sv_launch_one<4, 8>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
    case 8: return sv_launch_one<8, 8>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
    case 12: return sv_launch_one<12, 8>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
    case 16: return sv_launch_one<16, 8>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
    case 20: return sv_launch_one<20, 8>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
    case 24: return sv_launch_one<24, 4>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
    case 28: return sv_launch_one<28, 4>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);
    default: return sv_launch_one<32, 2>(st, d, Tslot, V0inv, V0invm, cs, ra, sep, gbuf, mode, nwg);  // LDS
  }
}

}  // namespace ccmm
