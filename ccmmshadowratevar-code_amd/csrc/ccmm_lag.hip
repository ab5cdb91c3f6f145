// CTA coefficient block on the lag structure of the VAR design (CTA.m:57-98,
// CTAsys.m:57-108; design built at mcmcVAR.m:62-72):
//
//   X(t, 0) = 1,   X(t, 1 + a) = D(t + rowoff(a), col(a))
//
// where D is the (T + p) x N data matrix (presample rows first) and a = N(l-1) + k
// is lag l of variable k.  X is never materialised: one D slab (122 KB at N = 20,
// T = 750) sits in LDS and every X access is D[t * ldd + colmap[a]].
//
//   k_gram_chol_lag  per (chain, equation) system, 512 threads, 1 workgroup / CU:
//       M = X~' diag(w) X~          weighted SYRK of the Np lag columns on
//                                   v_mfma_f64_16x16x4_f64, NT x NT tiles of 16 x 16
//                                   held in registers (8 waves, column-major tile
//                                   enumeration, wave W owns tiles W + 8k)
//       intercept peeled:           G = [c b'; b M + diag(iV~)], L00 = sqrt(c + iV0),
//                                   l = b / L00, M <- M + diag(iV~) - l l'
//                                   (the first step of right-looking Cholesky)
//       L~ = chol(M)                right-looking, 16-wide panels, trailing update on MFMA
//     output per system (doubles): NTILE tiles in the slot layout (tile g = column-major
//     enumeration of the lower tiles) of the block factorisation L~ = L_u D, D = diag(L~_pp),
//     L_u unit block lower with blocks M_ip = L~_ip L~_pp^-1: the diagonal slots hold
//     U~_pp^-1 = L~_pp^-T (the inverses the panel steps form anyway), the others M_ip'; then
//     [256]: [0] = 1 / L00, [1 + a] = L(1 + a, 0)
//
//   k_cta_solve_lag  per chain, equations j = 1..N in order (CTA.m:60-97):
//       v_t = sum_{i>=j} A(i,j) [E_t A(i,:)'] / sqrtht(t,i)^2        thread per t
//       rhs = iVb_j + X' v                                          D in LDS
//       PAI(:,j) = L' \ (L \ rhs + z_j)   (CTA.m:95-96: V rhs + Vc z with V = Vc Vc',
//                                          Vc = Vchol = inv(L)'), block substitutions with
//                                          L_u on the register-resident tiles (one barrier
//                                          per block step) and the D blocks in parallel: the
//                                          explicit inverse CTA.m:77 forms is never needed
//       E(:,j) = Y(:,j) - X PAI(:,j)                                D in LDS
//
// Padded lag columns (a >= Np) map to a spare zero column of D, so they carry zero
// data and the identity prior (iVdiag padding 1): exactly decoupled, x = 0 there.
#include "ccmm_lag.h"

#include <cstdlib>

namespace ccmm {

struct GlArgs {
  const double* w;     // sqrt weights [TP]
  const double* iv;    // iVdiag of (slot, j), K-space (0 = intercept), padded with 1
  const int* colmap;
  double* out;
  int T, ldd, mode;
  const double* Dl;    // LDS D
  const double* swl;   // LDS sqrt weights
};

// Opaque copy of a per-lane value: the factorisation loops below are inlined into the
// panel loop, and without this LLVM hoists every lane-dependent constant they derive
// (the δ_ic of the inverse, per-slot LDS addresses) out of that loop and spills them
// to scratch, putting a scratch reload on the serial path of every panel step.
__device__ __forceinline__ int gl_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// 1 / sqrt(d) as a deterministic function of d's bits (rsqrt_det, ccmm_internal.h), so that the
// factor can be reproduced bit for bit by a restatement (oracle/cta_lag_mirror.c): five dependent
// operations per fourth-order step, against three per Newton step of which four would be needed.
// The hardware v_rsq_f64 estimate is not reproducible off the device, and the IEEE sqrt + division
// pair puts ~25 dependent instructions on the serial pivot path.
__device__ __forceinline__ double gl_rsqrt_det(double d) { return rsqrt_det(d); }

// Per-wave factor + inverse of the SPD 16 x 16 tile Dg (row-major, ld kGlLd, lower
// triangle read): Ws := L^-1 (lower, row-major, ld kGlLd).  Lane i < 16 holds row i.
__device__ __forceinline__ int gl_factor_inv(const double* Dg, double* Ws, int lane_in) {
  const int lane = gl_opaque(lane_in);
  double row[16];
  double rdiag = 1.0, dmin = 1.0;  // smallest pivot: a non-positive one flags the system
#pragma unroll
  for (int m = 0; m < 16; ++m) row[m] = (lane < 16 && m <= lane) ? Dg[lane * kGlLd + m] : 0.0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    double dkk = readlane_d(row[kk], kk);
    dmin = fmin(dmin, dkk);
    const double rp = gl_rsqrt_det(fmax(dkk, 1e-300));
    if (lane == kk) rdiag = rp;
    const double lik = (lane > kk) ? row[kk] * rp : 0.0;
    row[kk] = lik;
#pragma unroll
    for (int m = kk + 1; m < 16; ++m) row[m] = fma(-lik, readlane_d(lik, m), row[m]);
  }
  const int bad = (dmin > 0.0) ? 0 : 1;
  // lane c < 16: column c of L^-1,  x_i = (delta_ic - sum_{m<i} L_im x_m) / L_ii, with L_im and
  // 1 / L_ii read from lane i's registers (row[m], rdiag) as scalars: no LDS round trip on the
  // serial path of the 16 rows
  const int c = lane;
  double x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    double s0 = (i == c) ? 1.0 : 0.0, s1 = 0.0;
#pragma unroll
    for (int m = 0; m < i; m += 2) {
      s0 = fma(-readlane_d(row[m], i), x[m], s0);
      if (m + 1 < i) s1 = fma(-readlane_d(row[m + 1], i), x[m + 1], s1);
    }
    x[i] = (i >= c) ? (s0 + s1) * readlane_d(rdiag, i) : 0.0;
  }
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) Ws[i * kGlLd + c] = x[i];
  }
  wave_lds_sync();
  return bad;
}

// Tile slots: slot gi enumerates the lower tile pairs (ti >= tj) column-major; the
// slot holds the UPPER tile (tj, ti) of the symmetric/triangular matrix, i.e. the
// transpose of the lower tile (ti, tj).  In that form every triangular product of the
// factorisation is a left-multiplication  C = A_lds x acc,  the orientation in which
// v_mfma_f64_16x16x4f64 takes the accumulator tile directly as its B operand.
// SYRK of the lag columns for wave W (compile-time tile ownership, so that the operand
// fragments stay in registers).  Only this loop is specialised per wave: the
// factorisation below runs one copy of the code for all waves (instruction cache).
template <int NT, int W>
__device__ __forceinline__ void gl_syrk(const GlArgs& g, dbl4 (&acc)[gl_tpw(NT)], double& bs0, double& bs1,
                                        double& csum, int lane) {
  constexpr int NTILE = gl_ntile(NT);
  constexpr int TPW = gl_tpw(NT);
  const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int k = 0; k < TPW; ++k) acc[k] = dbl4{0.0, 0.0, 0.0, 0.0};

  int off[NT];
#pragma unroll
  for (int b = 0; b < NT; ++b) off[b] = g.colmap[16 * b + lr];
  bs0 = 0.0;
  bs1 = 0.0;
  csum = 0.0;
  const int nks = (g.mode & 1) ? 0 : (g.T + 3) >> 2;
  // software pipeline over k-steps: step ks scales its raw D values into the MFMA operands,
  // then issues the LDS loads of step ks + 1 into the freed registers before its 15 MFMAs,
  // so those loads complete under ~15 x 64 MFMA cycles instead of stalling the next step
  // (scheduling barriers keep LLVM from sinking them next to their use)
  double raw[NT], sw = 0.0;
  auto load = [&](int ks) {
    const int t = 4 * ks + lq;
    sw = g.swl[t];
    const double* row = g.Dl + t * g.ldd;
#pragma unroll
    for (int b = 0; b < NT; ++b) raw[b] = row[off[b]];
  };
  if (nks > 0) load(0);
  for (int ks = 0; ks < nks; ++ks) {
    double frag[NT];
#pragma unroll
    for (int b = 0; b < NT; ++b) frag[b] = raw[b] * sw;
    const double swc = sw;
    load(ks + 1 < nks ? ks + 1 : ks);  // past the end: a harmless reload
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      if (W + kGlWaves * k < NTILE) {
        const int gi = W + kGlWaves * k;
        acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(frag[gl_tj(NT, gi)], frag[gl_ti(NT, gi)], acc[k],
                                                      0, 0, 0);
      }
    }
    // intercept row b = X~' w: wave W accumulates lag tiles W and W + 8
    if (W < NT) bs0 = fma(frag[W < NT ? W : 0], swc, bs0);
    if (W + kGlWaves < NT) bs1 = fma(frag[W + kGlWaves < NT ? W + kGlWaves : 0], swc, bs1);
    csum = fma(swc, swc, csum);
    __builtin_amdgcn_sched_barrier(0);
  }
  bs0 += __shfl_xor(bs0, 16);
  bs0 += __shfl_xor(bs0, 32);
  bs1 += __shfl_xor(bs1, 16);
  bs1 += __shfl_xor(bs1, 32);
  csum += __shfl_xor(csum, 16);
  csum += __shfl_xor(csum, 32);
}

// Factorisation stage for wave W (runtime, wave-uniform): intercept peel, Cholesky,
// inverse, output.  sti/stj: the (ti, tj) of this wave's slots.
template <int NT>
__device__ __forceinline__ int gram_lag_factor(const GlArgs& g, double* sm, int tid, int W,
                                               dbl4 (&acc)[gl_tpw(NT)], double bs0, double bs1, double csum) {
  constexpr int NTILE = gl_ntile(NT);
  constexpr int TPW = gl_tpw(NT);
  constexpr int KL = 16 * NT;
  const int lane = tid & 63, lr0 = lane & 15, lq0 = lane >> 4;
  const int lr = lr0, lq = lq0;
  int bad = 0;
  int sti[TPW], stj[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int gi = W + kGlWaves * k;
    sti[k] = gi < NTILE ? gl_ti(NT, gi) : 0;
    stj[k] = gi < NTILE ? gl_tj(NT, gi) : 0;
  }
  if (g.mode & 8) {  // parity export (ccmm_chains_get_cta_gram): the SYRK stage as it stands
    double* o = g.out;
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[gi * 256 + 64 * r + lane] = acc[k][r];
      }
    }
    if (lq == 0) {
      if (W < NT) o[NTILE * 256 + 1 + 16 * W + lr] = bs0;
      if (W + kGlWaves < NT) o[NTILE * 256 + 1 + 16 * (W + kGlWaves) + lr] = bs1;
    }
    if (W == 0 && lane == 0) o[NTILE * 256] = csum;
    return 0;
  }
  __syncthreads();  // D no longer needed: the LDS is reused below

  double* lvec = sm;              // KL   b, then l = b / L00
  double* misc = lvec + KL;       // 8
  double* Dg = misc + 8;          // diagonal tile of the current panel
  double* Pn0 = Dg + kGlTile;     // 2 x NT tiles: panel rows; (inverse) U column / Z row
  double* Ws = Pn0 + 2 * NT * kGlTile + W * kGlTile;  // this wave's L_pp^-1

  if (lq == 0) {
    if (W < NT) lvec[16 * W + lr] = bs0;
    if (W + kGlWaves < NT) lvec[16 * (W + kGlWaves) + lr] = bs1;
  }
  if (W == 0 && lane == 0) misc[0] = csum;
  __syncthreads();
  const double G00 = misc[0] + g.iv[0];
  if (!(G00 > 0.0)) bad = 1;
  const double L00 = sqrt(G00 > 0.0 ? G00 : 1.0);
  const double rL00 = 1.0 / L00;
  // + diag(iV~) - l l'   (slot element (lq + 4r, lr) = row 16 tj + lq + 4r, column 16 ti + lr)
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int gi = W + kGlWaves * k;
    if (gi < NTILE) {
      const int ti = sti[k], tj = stj[k];
      const double lc = lvec[16 * ti + lr] * rL00;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rowi = 16 * tj + lq + 4 * r;
        double v = fma(-(lvec[rowi] * rL00), lc, acc[k][r]);
        if (ti == tj && lq + 4 * r == lr) v += g.iv[1 + rowi];
        acc[k][r] = v;
      }
    }
  }
  __syncthreads();
  if (tid < KL) lvec[tid] *= rL00;  // l
  __syncthreads();

  // ------------------------------------------------------------ Cholesky M~ = U'U
  // LinvB (shared) holds L_pp^-1 of the current panel.  Panel p:
  //   U_pi = L_pp^-1 G_pi (slots ti = i > p, tj = p) on MFMA;  slot (p,p) := U_pp^-1
  //   trailing  G_ij -= U_pi' U_pj  (slots ti, tj > p) on MFMA from the LDS panel.
  // Look-ahead: the owner of slot (p+1, p+1) updates that tile first and factors it
  // (gl_factor_inv -> LinvB) while the other waves run their trailing updates, so each
  // panel costs two barriers and one serial 16 x 16 factorisation on one wave.
  double* LinvB = Dg;
  const bool do_chol = !(g.mode & 2);
  if (do_chol) {  // prologue: factor the first diagonal tile
    bool own = false;
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE && sti[k] == 0 && stj[k] == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Ws[(lq + 4 * r) * kGlLd + lr] = acc[k][r];
        own = true;
      }
    }
    wave_lds_sync();
    if (own && !(g.mode & 256)) bad |= gl_factor_inv(Ws, LinvB, lane);
  }
  for (int p = 0; p < (do_chol ? NT : 0); ++p) {
    const int lr = gl_opaque(lr0), lq = gl_opaque(lq0);  // no hoisted per-slot addresses
    __syncthreads();  // LinvB = L_pp^-1 visible; the previous trailing reads of Pn are done
    double* Pn = Pn0;
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE && stj[k] == p) {
        const int ti = sti[k];
        if (ti == p) {  // U_pp^-1 = (L_pp^-1)': element (lq + 4r, lr) = Linv[lr][lq + 4r]
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[k][r] = LinvB[lr * kGlLd + lq + 4 * r];
        } else {
          dbl4 cc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            cc = __builtin_amdgcn_mfma_f64_16x16x4f64(LinvB[lr * kGlLd + 4 * kk + lq], acc[k][kk], cc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) Pn[ti * kGlTile + (lq + 4 * r) * kGlLd + lr] = cc[r];
          // stored form: M'_pi = U_pp^-1 U_pi = (L_ip L_pp^-1)', the block of the unit block
          // factor (k_cta_solve_lag: one barrier per block step); off the panel's critical path
          dbl4 mm = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            mm = __builtin_amdgcn_mfma_f64_16x16x4f64(LinvB[(4 * kk + lq) * kGlLd + lr], cc[kk], mm, 0, 0, 0);
          acc[k] = mm;
        }
      }
    }
    __syncthreads();  // panel visible; LinvB free for the next factorisation
    if (p + 1 < NT && !(g.mode & 1024)) {
      const int q = p + 1;
      // look-ahead: next diagonal tile first, then its factorisation
      bool own = false;
#pragma unroll
      for (int k = 0; k < TPW; ++k) {
        const int gi = W + kGlWaves * k;
        if (gi < NTILE && sti[k] == q && stj[k] == q) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const double pq = Pn[q * kGlTile + (4 * kk + lq) * kGlLd + lr];
            acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(-pq, pq, acc[k], 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) Ws[(lq + 4 * r) * kGlLd + lr] = acc[k][r];
          own = true;
        }
      }
      wave_lds_sync();
      if (own && !(g.mode & 256)) bad |= gl_factor_inv(Ws, LinvB, lane);
#pragma unroll
      for (int k = 0; k < TPW; ++k) {
        const int gi = W + kGlWaves * k;
        if (gi < NTILE && stj[k] > p && !(sti[k] == q && stj[k] == q)) {
          const double* Pa = Pn + stj[k] * kGlTile + lq * kGlLd + lr;
          const double* Pb = Pn + sti[k] * kGlTile + lq * kGlLd + lr;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(-Pa[4 * kk * kGlLd], Pb[4 * kk * kGlLd], acc[k], 0, 0,
                                                          0);
        }
      }
    }
  }

  // ------------------------------------------------------------ intercept column of L
  //   L(1+a, 0) = l_a (lvec, already b / L00); [0] = 1 / L00
  double* o = g.out;
  if (tid < KL) o[NTILE * 256 + 1 + tid] = lvec[tid];
  if (tid == 0) o[NTILE * 256] = rL00;
  // ------------------------------------------------------------ factor tiles -> HBM in slot layout
  //   off-diagonal slots U~_{tj,ti} = L~_{ti,tj}', diagonal slots U~_pp^-1 (the solve's
  //   blocked substitutions, k_cta_solve_lag)
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int gi = W + kGlWaves * k;
    if (gi < NTILE) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[gi * 256 + 64 * r + lane] = acc[k][r];
    }
  }
  return bad;
}

template <int NT>
__global__ __launch_bounds__(512, 1) void k_gram_chol_lag(Dims d, const int* __restrict__ Tslot, LagSel ls,
                                                          ChainState cs, const double* __restrict__ iVdiag) {
  extern __shared__ double sm[];
  const int mat = blockIdx.x;
  const int c = mat / d.N, j = mat % d.N;
  const int s = cs.slot[c];
  const int tid = threadIdx.x;
  const int TP = d.TP;
  // D slab and sqrt weights -> LDS: every load of a thread's share (up to 32 + 2) issued before the
  // first LDS store, so the slab arrives in one HBM/L2 round trip instead of one per element
  {
    const double* src = ls.dpool + (size_t)ls.idx[mat] * ls.rows * ls.ldd;
    const int n = ls.rows * ls.ldd;
    const double* w = cs.W + (size_t)mat * TP;
    double* swl = sm + n;
    int q = tid;
    for (; q < n; q += 32 * 512) {
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = (q + 512 * u < n) ? src[q + 512 * u] : 0.0;
      double wv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) wv[u] = (q == tid && tid + 512 * u < TP) ? w[tid + 512 * u] : 0.0;
#pragma unroll
      for (int u = 0; u < 32; ++u)
        if (q + 512 * u < n) sm[q + 512 * u] = v[u];
      if (q == tid) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (tid + 512 * u < TP + 4) swl[tid + 512 * u] = wv[u];
      }
    }
    for (int t = tid + 1024; t < TP + 4; t += 512) swl[t] = (t < TP) ? w[t] : 0.0;
  }
  __syncthreads();
  GlArgs g;
  g.T = Tslot[s];
  g.ldd = ls.ldd;
  g.mode = ls.mode;
  g.colmap = ls.colmap;
  g.iv = iVdiag + ((size_t)s * d.N + j) * d.KP;
  g.out = cs.G + (size_t)mat * d.KP * d.KP;
  g.Dl = sm;
  g.swl = sm + ls.rows * ls.ldd;
  g.w = nullptr;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  dbl4 acc[gl_tpw(NT)];
  double bs0, bs1, csum;
  switch (wave) {
    case 0: gl_syrk<NT, 0>(g, acc, bs0, bs1, csum, tid & 63); break;
    case 1: gl_syrk<NT, 1>(g, acc, bs0, bs1, csum, tid & 63); break;
    case 2: gl_syrk<NT, 2>(g, acc, bs0, bs1, csum, tid & 63); break;
    case 3: gl_syrk<NT, 3>(g, acc, bs0, bs1, csum, tid & 63); break;
    case 4: gl_syrk<NT, 4>(g, acc, bs0, bs1, csum, tid & 63); break;
    case 5: gl_syrk<NT, 5>(g, acc, bs0, bs1, csum, tid & 63); break;
    case 6: gl_syrk<NT, 6>(g, acc, bs0, bs1, csum, tid & 63); break;
    case 7: gl_syrk<NT, 7>(g, acc, bs0, bs1, csum, tid & 63); break;
    default: __builtin_unreachable();
  }
  const int bad = gram_lag_factor<NT>(g, sm, tid, wave, acc, bs0, bs1, csum);
  if (bad && (tid & 63) == 0) atomicOr(&cs.status[c], 2);
}

// ================================================================== sequential solve
// The factor tiles of the current equation live in registers in the slot layout of
// k_gram_chol_lag (wave W holds slots W + 8k; element (lq + 4r, lr) of slot (ti, tj) =
// M'_{tj,ti}(lq + 4r, lr), U~_pp^-1 on the diagonal): one coalesced HBM read per system,
// issued after the v_t loads so that it overlaps the X'v product.
//
#ifdef CCMM_ABLATION
// timing-only phase attribution of k_cta_solve_lag (ablation build): shader-clock cycles of chain
// 0's first workgroup per phase -- v_t | X'v (+ the halves' swap) | forward | backward | residuals
// -- summed over equations and launches (read by ccmm_solve_prof)
__device__ unsigned long long g_solve_prof[8];
extern "C" int ccmm_solve_prof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solve_prof), sizeof(g_solve_prof)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_solve_prof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#define SL_CLK(x) const unsigned long long x = clock64()
#define SL_ACC(k, a, b) \
  if (c == 0 && blockIdx.y == 0 && tid == 0) atomicAdd(&g_solve_prof[k], (b) - (a))
#else
#define SL_CLK(x)
#define SL_ACC(k, a, b)
#endif
//
// Split (gridDim.y == 2, small B): two workgroups per chain, on two CUs.  Workgroup h owns the months
// of X'v half h, t in [0, th) or [th, T) with th = ceil(T / 2): it forms v_t and the residuals of
// those months only (a month's v_t reads that month's residuals alone, so the halves never read each
// other's months) and the X'v partial of its half; the halves swap partials through global memory
// (one agent-scope flag per workgroup and equation, double-buffered by equation parity), and both
// run the substitutions on the same right-hand side part_0 + part_1 + iVb, so x is the same in both.
// Every sum is formed in the order of the one-workgroup kernel: the draws are bit-identical.
template <int NT, int NMAX, int SW, bool RO>
__global__ __launch_bounds__(64 * SW) void k_cta_solve_lag(Dims d, const int* __restrict__ Tslot,
                                                              const double* __restrict__ iVb, XSel xs, LagSel ls,
                                                              ChainState cs, RngArgs ra, SolveXch xc) {
  constexpr int NTILE = gl_ntile(NT);
  constexpr int NTH = 64 * SW;                      // SW waves (8 or 16)
  // factor tiles held per wave: slots wave + SW k (barrier-stepped substitutions), or with RO (row
  // ownership) whole block rows, NT tiles per wave: wave 0 row NT - 1, wave w >= 1 rows w - 1 and
  // NT - 1 - w (NT = 15: sizes w + (15 - w))
  static_assert(!RO || (SW == 8 && (NT == 1 || NT == 15)), "row-owned substitutions: 8 waves, NT 1 or 15");
  constexpr int TPW = RO ? NT : (gl_ntile(NT) + SW - 1) / SW;
  constexpr int KL = 16 * NT;
  extern __shared__ double sm[];
  const int N = d.N, TP = d.TP, K = d.K, KP = d.KP;
  const int ldd = ls.ldd, rows = ls.rows;
  double* Dl = sm;
  double* vl = Dl + rows * ldd;      // TP            phases 1-2
  double* part = vl + TP;            // 2 x 256       phase 2
  double* rl = vl + sl_union(NT, TP);  // 256  rhs, then c = y + z  (K-space)
  double* xl = rl + 256;             // 256  y, then x            (K-space)
  double* Al = xl + 256;             // N x N, column stride NMAX
  double* red = Al + NMAX * NMAX;    // 16
  int* cm = reinterpret_cast<int*>(red + 16);  // KL
  int* zdone = cm + KL;                        // RO: forward, block z_p final
  int* cnt = zdone + 16;                       // RO: backward, rows p > i pushed into block i
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int T = Tslot[s];
  const int tid = threadIdx.x, lane0 = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Rng rng = ra.make(c);
  const bool split = gridDim.y > 1;
  const int hh = split ? (int)blockIdx.y : 0;
  const int th = (T + 1) >> 1;
  const int tlo = (split && hh) ? th : 0, thi = (split && !hh) ? th : TP;  // this workgroup's months
  const double* ih2 = cs.ih2 + (size_t)c * N * TP;
  const double* Y = xs.ypool + (size_t)xs.yidx[c] * N * TP;
  double* E = cs.E + (size_t)c * N * TP;
  for (int q = tid; q < N * N; q += NTH) Al[(q % N) + (q / N) * NMAX] = cs.A[(size_t)c * N * N + q];
  for (int q = tid; q < KL; q += NTH) cm[q] = ls.colmap[q];
  // this wave's slots: (ti, tj) per register tile
  int sti[TPW], stj[TPW];
  // RO rows: rHi (register tiles 0 .. nHi - 1) and rLo (tiles nHi .. nHi + nLo - 1)
  const int rHi = NT - 1 - wave, rLo = wave - 1;
  const bool hasHi = rHi >= 0, hasLo = wave >= 1 && rLo < rHi;
  const int nHi = hasHi ? rHi + 1 : 0, nLo = hasLo ? rLo + 1 : 0;
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    if constexpr (RO) {
      sti[k] = (k < nHi) ? rHi : rLo;
      stj[k] = (k < nHi) ? k : k - nHi;
    } else {
      const int gi = wave + SW * k;
      sti[k] = gi < NTILE ? gl_ti(NT, gi) : 0;
      stj[k] = gi < NTILE ? gl_tj(NT, gi) : 0;
    }
  }
  // slot of register tile k, or -1
  auto slot_of = [&](int k) -> int {
    if constexpr (RO) return (k < nHi + nLo) ? gl_tile(NT, sti[k], stj[k]) : -1;
    const int gi = wave + SW * k;
    return gi < NTILE ? gi : -1;
  };
  int cur = -1;

  for (int j = 0; j < N; ++j) {
    // per-equation opaque lane ids: no lane-derived address is hoisted out of the
    // equation loop next to the 120 factor registers (see gl_opaque)
    const int lane = gl_opaque(lane0), lr = lane & 15, lq = lane >> 4;
    const int mat = c * N + j;
    const int slab = ls.idx[mat];
    const double* Lo = cs.G + (size_t)mat * KP * KP;
    const double* Lv = Lo + NTILE * 256;  // [0] 1/L00, [1+a] L(1+a,0)
    if (slab != cur) {
      __syncthreads();
      const double* src = ls.dpool + (size_t)slab * rows * ldd;
      // every load of a thread's share issued before the first LDS store (one round trip per 16)
      for (int q = tid; q < rows * ldd; q += 16 * NTH) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = (q + NTH * u < rows * ldd) ? src[q + NTH * u] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (q + NTH * u < rows * ldd) Dl[q + NTH * u] = v[u];
      }
      cur = slab;
    }
    SL_CLK(q0);
    // ---- (1) v_t (E(:,j) = Y(:,j) stands for PAI(:,j) = 0, CTA.m:63)
    for (int t = tlo + tid; t < thi; t += NTH) {
      double acc = 0.0;
      if (t < T && !(ls.mode & 16)) {
        double e[NMAX];
        // per-lane element offsets (k TP + t) advanced in a register, so that no per-k base address
        // is hoisted into scalar registers (the kernel's scalar file would spill)
        int o = t;
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
          if (k < N) e[k] = ((k == j) ? Y : E)[o];
          o += TP;
        }
        // A in LDS with the compile-time column stride NMAX (every A(i, k) read is an immediate offset
        // from row i's address); the row loop stays rolled so that only one row of A is in flight
        // (unrolled, the compiler hoisted all N(N+1)/2 entries into registers and spilled)
        // 1 / sqrtht(t, i)^2 of rows i >= j, fetched four rows ahead through a register queue
        const double* wt = ih2 + t;
        double w0 = (j < N) ? wt[j * TP] : 0.0, w1 = (j + 1 < N) ? wt[(j + 1) * TP] : 0.0;
        double w2 = (j + 2 < N) ? wt[(j + 2) * TP] : 0.0, w3 = (j + 3 < N) ? wt[(j + 3) * TP] : 0.0;
#pragma unroll 1
        for (int i = j; i < N; ++i) {
          const double wi = w0;
          w0 = w1;
          w1 = w2;
          w2 = w3;
          w3 = (i + 4 < N) ? wt[(i + 4) * TP] : 0.0;
          const double* Ai = Al + i;
          double ea = 0.0;
#pragma unroll
          for (int k = 0; k < NMAX; ++k)
            if (k <= i) ea = fma(e[k], Ai[k * NMAX], ea);
          acc = fma(Ai[j * NMAX] * ea, wi, acc);
        }
      }
      vl[t] = acc;
    }
    __syncthreads();
    SL_CLK(q1);
    // factor tiles of this system -> registers (consumed in phases 3-4); issued after the
    // barrier so that they cannot be hoisted into the v_t loop (register pressure)
    dbl4 lt[TPW];
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = slot_of(k);
      if (gi >= 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) lt[k][r] = Lo[gi * 256 + 64 * r + lane];
      } else {
        lt[k] = dbl4{0.0, 0.0, 0.0, 0.0};
      }
    }
    // ---- (2) rhs = iVb_j + X' v, two t-halves per column
    const int nxv = split ? 256 : 512;  // threads forming X'v partials (one half when split)
    {
      const int h = split ? hh : tid >> 8, a = tid & 255;
      const int t0 = h ? th : 0, t1 = h ? T : th;
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
      if ((ls.mode & 32) || tid >= nxv) {  // threads 512.. (SW = 16) idle: the t-halves fix the order
      } else if (a < KL) {
        // four strided chains (t mod 4); the loads of eight months are issued before their
        // fused multiply-adds so that one LDS round trip serves eight products
        const double* col = Dl + cm[a];
        int t = t0;
        for (; t + 7 < t1; t += 8) {
          double cv[8], vv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            cv[u] = col[(t + u) * ldd];
            vv[u] = vl[t + u];
          }
          p0 = fma(cv[0], vv[0], p0);
          p1 = fma(cv[1], vv[1], p1);
          p2 = fma(cv[2], vv[2], p2);
          p3 = fma(cv[3], vv[3], p3);
          p0 = fma(cv[4], vv[4], p0);
          p1 = fma(cv[5], vv[5], p1);
          p2 = fma(cv[6], vv[6], p2);
          p3 = fma(cv[7], vv[7], p3);
        }
        if (t + 3 < t1) {
          p0 = fma(col[t * ldd], vl[t], p0);
          p1 = fma(col[(t + 1) * ldd], vl[t + 1], p1);
          p2 = fma(col[(t + 2) * ldd], vl[t + 2], p2);
          p3 = fma(col[(t + 3) * ldd], vl[t + 3], p3);
          t += 4;
        }
        for (; t < t1; ++t) p0 = fma(col[t * ldd], vl[t], p0);
      } else if (a == KL) {
        // the intercept column: one sequential sum of the half's v_t (the order of the plain loop);
        // sixteen values per LDS round trip, so the chain waits on additions, not on LDS latency
        // (one read per addition made this thread the phase's straggler: ~40k cycles of ~50k)
        int t = t0;
        for (; t + 15 < t1; t += 16) {
          double vv[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) vv[u] = vl[t + u];
#pragma unroll
          for (int u = 0; u < 16; ++u) p0 += vv[u];
        }
        for (; t < t1; ++t) p0 += vl[t];
      }
      if (tid < nxv) part[h * 256 + a] = (p0 + p1) + (p2 + p3);
    }
    __syncthreads();
    SL_CLK(q1b);
    SL_ACC(6, q1, q1b);
    if (split) {  // swap the halves' partials with the chain's other workgroup
      const int par = j & 1;
      double* mine = xc.part + (((size_t)c * 2 + hh) * 2 + par) * 256;
      const double* other = xc.part + (((size_t)c * 2 + (1 - hh)) * 2 + par) * 256;
      // write-through (sc1) partials drained before the flag, the flag an sc1 store, the partner's partials
      // read by sc1 loads: no L2 write-back or L1 invalidate on the equation's path (the microarch guide's
      // R1 hand-off; the fence pair it replaces cost ~5 us per equation at B = 1)
      if (tid <= KL)
        __hip_atomic_store((unsigned long long*)(mine + tid), (unsigned long long)__double_as_longlong(part[hh * 256 + tid]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const unsigned long long seq = xc.epoch * 64ull + (unsigned long long)j + 1ull;
      if (tid == 0) {
        __hip_atomic_store(&xc.flag[c * 2 + hh], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int it = 0;; ++it) {
          if (__hip_atomic_load(&xc.flag[c * 2 + 1 - hh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= seq) break;
          if (it > (1 << 22)) {  // never expected: flag the chain and go on (no hang)
            atomicOr(&cs.status[c], 32);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the poll)
      if (tid <= KL)
        part[(1 - hh) * 256 + tid] = __longlong_as_double((long long)__hip_atomic_load(
            (const unsigned long long*)(other + tid), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      __syncthreads();
    }
    SL_CLK(q2);
    const double* ivb = iVb + ((size_t)s * N + j) * KP;
    if (tid <= KL) {
      const int kx = (tid == KL) ? 0 : 1 + tid;
      rl[kx] = part[tid] + part[256 + tid] + ivb[kx];
    }
    __syncthreads();
    // ---- (3) forward substitution L y = rhs (CTA.m:95's Vchol' rhs without the explicit
    //         inverse): y_0 = rhs_0 / L00, r~ = rhs~ - l y_0, then L_u z = r~ by block steps
    //         (after step p - 1, z_p = r~_p is final; the owners of the slots (i, p) below
    //         take M_ip z_p off r~_i, one barrier), and y_p = L~_pp^-1 z_p for all p at once
    if (tid < KL) rl[1 + tid] = fma(-Lv[1 + tid], rl[0] * Lv[0], rl[1 + tid]);
    if (tid == KL) xl[0] = rl[0] * Lv[0];
    if (RO && tid < 16) {
      zdone[tid] = 0;
      cnt[tid] = 0;
    }
    __syncthreads();
    // slot (ti, tj) times block tj of u, summed over the slot's rows: (M u)_ti (or U^-T u)
    auto colsum = [&](const dbl4& t, const double* u) {
      double v = t[0] * u[0];
      v = fma(t[1], u[4], v);
      v = fma(t[2], u[8], v);
      v = fma(t[3], u[12], v);
      return xsum32(xsum16(v));
    };
    const bool subst = !(ls.mode & 64);
    // RO hand-offs between waves: LDS flags with workgroup-scope release / acquire, polled with a
    // bounded spin (a cap that is never expected to be reached ends the wait and flags the chain)
    bool stuck = false;
    auto wait_eq = [&](int* f, int v) {
      for (int it = 0; it < (1 << 22); ++it) {
        if (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == v) return;
        __builtin_amdgcn_s_sleep(1);
      }
      stuck = true;
    };
    auto post = [&](int* f, int v) {
      if (lane == 0) __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    if constexpr (RO) {
      // rows of L_u: the owner of block row i subtracts M_iq z_q from r~_i in q order as each z_q
      // is posted (the same sequence of subtractions as the stepped form), posts z_i, and forms
      // y_i = L~_ii^-1 z_i with its diagonal tile
      if (subst) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // rLo, then rHi
          const bool has = h ? hasHi : hasLo;
          const int row = h ? rHi : rLo, k0 = h ? 0 : nHi;
          if (has) {
            double racc = rl[1 + 16 * row + lr];
#pragma unroll
            for (int k = 0; k < TPW; ++k) {
              if (k >= k0 && k <= k0 + row) {
                const int q = k - k0;
                if (q < row) {
                  wait_eq(zdone + q, 1);
                  racc -= colsum(lt[k], rl + 1 + 16 * q + lq);
                } else {
                  if (lq == 0) rl[1 + 16 * row + lr] = racc;
                  wave_lds_sync();
                  post(zdone + row, 1);
                  const double v = colsum(lt[k], rl + 1 + 16 * row + lq);
                  if (lq == 0) xl[1 + 16 * row + lr] = v;
                }
              }
            }
          }
        }
      }
    }
    for (int p = 0; p < ((subst && !RO) ? NT - 1 : 0); ++p) {
#pragma unroll
      for (int k = 0; k < TPW; ++k) {
        const int gi = wave + SW * k;
        if (gi < NTILE && stj[k] == p && sti[k] > p) {
          const double v = colsum(lt[k], rl + 1 + 16 * p + lq);
          if (lq == 0) rl[1 + 16 * sti[k] + lr] -= v;
        }
      }
      __syncthreads();
    }
    if (subst && !RO) {
#pragma unroll
      for (int k = 0; k < TPW; ++k) {
        const int gi = wave + SW * k;
        if (gi < NTILE && sti[k] == stj[k]) {
          const double v = colsum(lt[k], rl + 1 + 16 * sti[k] + lq);
          if (lq == 0) xl[1 + 16 * sti[k] + lr] = v;
        }
      }
    }
    __syncthreads();
    SL_CLK(q3);
    // ---- (4) c = y + z_j (randn(K,N) of CTA.m:58, column j); back substitution L' x = c:
    //         w_p = L~_pp^-T c~_p for all p at once, then L_u' x~ = w by block steps from the
    //         bottom (x_p = w_p final; the owners of the slots (p, i) take M_pi' x_p off w_i),
    //         and x_0 = (c_0 - l' x~) / L00
    if (tid <= KL) {
      const int kx = (tid == KL) ? 0 : 1 + tid;
      rl[kx] = xl[kx] + ((kx < K) ? rng.normal(CCMM_RNG_PAI, (uint32_t)(kx + K * j)) : 0.0);
    }
    __syncthreads();
    {
      // slot times block ti of u, per slot row (lq + 4r) = sum_lr t[r] u(lr): four sums over
      // the 16 lanes of a row group, folded so that lane (lr & 3) == 0 ends with r = lr >> 2
      const bool b8 = lr & 8, b4 = lr & 4;
      auto fold = [&](const dbl4& t, double cv) {
        const double v0 = t[0] * cv, v1 = t[1] * cv, v2 = t[2] * cv, v3 = t[3] * cv;
        // lane exchanges inside the 16-lane row by DPP (VALU, ~10 clocks) instead of ds_bpermute
        // (an LDS round trip each): xor 8 = row_ror:8; xor 4 = row_shl:4 (lanes with bit 2 clear take
        // lane + 4) / row_shr:4 (the others take lane - 4)
        double a = b8 ? v2 : v0, b = b8 ? v3 : v1;
        a += dpp_d<0x128>(b8 ? v0 : v2);
        b += dpp_d<0x128>(b8 ? v1 : v3);
        double q = b4 ? b : a;
        const double x4 = b4 ? a : b;
        // both moves on every lane first (a DPP read of a lane masked off by a branch returns 0)
        const double s4l = dpp_d<0x104>(x4), s4r = dpp_d<0x114>(x4);
        q += b4 ? s4r : s4l;
        q += dpp_d<0x4E>(q);  // xor 2 (quad_perm, no LDS round trip)
        q += dpp_d<0xB1>(q);  // xor 1
        return q;
      };
      if (subst) {
#pragma unroll
        for (int k = 0; k < TPW; ++k) {
          const bool diag = RO ? (slot_of(k) >= 0 && sti[k] == stj[k])
                               : (wave + SW * k < NTILE && sti[k] == stj[k]);
          if (diag) {
            const double q = fold(lt[k], rl[1 + 16 * sti[k] + lr]);
            if ((lr & 3) == 0) xl[1 + 16 * sti[k] + lq + 4 * (lr >> 2)] = q;
          }
        }
      }
      __syncthreads();
      if constexpr (RO) {
        // columns of L_u' by pushes: the owner of block row p waits until the rows below have pushed
        // into block p (x_p final), then takes M_pi' x_p off w_i for i = p - 1 .. 0, each push in
        // turn after row p + 1's push into block i (the stepped form's order, p descending)
        if (subst) {
#pragma unroll
          for (int h = 1; h >= 0; --h) {  // rHi, then rLo
            const bool has = h ? hasHi : hasLo;
            const int row = h ? rHi : rLo, k0 = h ? 0 : nHi;
            if (has) {
              wait_eq(cnt + row, NT - 1 - row);
              const double xp = xl[1 + 16 * row + lr];
#pragma unroll
              for (int k = TPW - 1; k >= 0; --k) {
                if (k >= k0 && k < k0 + row) {
                  const int i = k - k0;
                  const double q = fold(lt[k], xp);
                  wait_eq(cnt + i, NT - 1 - row);
                  if ((lr & 3) == 0) xl[1 + 16 * i + lq + 4 * (lr >> 2)] -= q;
                  wave_lds_sync();
                  post(cnt + i, NT - row);
                }
              }
            }
          }
        }
        if (stuck && lane == 0) atomicOr(&cs.status[c], 32);
        __syncthreads();  // every x~ block final before l' x~
      }
      for (int p = ((subst && !RO) ? NT - 1 : 0); p >= 1; --p) {
#pragma unroll
        for (int k = 0; k < TPW; ++k) {
          const int gi = wave + SW * k;
          if (gi < NTILE && sti[k] == p && stj[k] < p) {
            const double q = fold(lt[k], xl[1 + 16 * p + lr]);
            if ((lr & 3) == 0) xl[1 + 16 * stj[k] + lq + 4 * (lr >> 2)] -= q;
          }
        }
        __syncthreads();
      }
    }
    {  // l' x~
      double pr = (tid < KL) ? Lv[1 + tid] * xl[1 + tid] : 0.0;
      pr = wave_sum_dpp(pr);
      if (lane == 0) red[wave] = pr;
    }
    __syncthreads();
    if (tid == KL) {
      double sacc = 0.0;
      for (int w = 0; w < NTH / 64; ++w) sacc += red[w];
      xl[0] = (rl[0] - sacc) * Lv[0];
    }
    __syncthreads();
    SL_CLK(q4);
    // ---- (5) PAI(:,j) = x; E(:,j) = Y(:,j) - X x
    double* pai = cs.PAI + ((size_t)c * N + j) * KP;
    if (hh == 0)
      for (int k = tid; k < KP; k += NTH) pai[k] = (k < K) ? xl[k] : 0.0;
    for (int t = tlo + tid; t < thi; t += NTH) {
      double o = 0.0;
      if (t < T && !(ls.mode & 128)) {
        const double* rowp = Dl + t * ldd;
        double s0 = xl[0], s1 = 0.0, s2 = 0.0, s3 = 0.0;
        if ((N & 3) == 0) {
          // lag l, variable k is column a = (l - 1) N + k at D row t + p - l: with N a multiple
          // of four, a mod 4 = k mod 4, so the chains need no column table (no dependent LDS
          // load per product); the padded columns a >= N p are zero data and are skipped
          const int P = ls.p;
          for (int l = 1; l <= P; ++l) {
            const double* row = rowp + (P - l) * ldd;
            const double* xa = xl + 1 + (l - 1) * N;
#pragma unroll
            for (int k = 0; k < NMAX; k += 4) {
              if (k < N) {
                const double d0 = row[k], d1 = row[k + 1], d2 = row[k + 2], d3 = row[k + 3];
                s0 = fma(d0, xa[k], s0);
                s1 = fma(d1, xa[k + 1], s1);
                s2 = fma(d2, xa[k + 2], s2);
                s3 = fma(d3, xa[k + 3], s3);
              }
            }
          }
        } else {
          int a = 0;
          for (; a + 3 < KL; a += 4) {
            s0 = fma(rowp[cm[a]], xl[1 + a], s0);
            s1 = fma(rowp[cm[a + 1]], xl[2 + a], s1);
            s2 = fma(rowp[cm[a + 2]], xl[3 + a], s2);
            s3 = fma(rowp[cm[a + 3]], xl[4 + a], s3);
          }
          for (; a < KL; ++a) s0 = fma(rowp[cm[a]], xl[1 + a], s0);
        }
        o = Y[(size_t)j * TP + t] - ((s0 + s1) + (s2 + s3));
      }
      E[(size_t)j * TP + t] = o;
    }
    __syncthreads();
    SL_CLK(q5);
    SL_ACC(0, q0, q1);
    SL_ACC(1, q1, q2);
    SL_ACC(2, q2, q3);
    SL_ACC(3, q3, q4);
    SL_ACC(4, q4, q5);
    if (j == 0) SL_ACC(5, 0ull, 1ull);
  }
}


// ------------------------------------------------------------------ host launchers
bool lag_supported_nt(int nt) { return nt == 1 || nt == 15; }

hipError_t lag_launch_gram(int NT, hipStream_t st, size_t lds, Dims d, const int* Tslot, LagSel ls,
                           ChainState cs, const double* iVdiag) {
  const void* fn = nullptr;
  switch (NT) {
    case 1: fn = (const void*)k_gram_chol_lag<1>; break;
    case 15: fn = (const void*)k_gram_chol_lag<15>; break;
    default: return hipErrorInvalidValue;
  }
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  switch (NT) {
    case 1: hipLaunchKernelGGL(k_gram_chol_lag<1>, dim3(d.nmat), dim3(512), lds, st, d, Tslot, ls, cs, iVdiag); break;
    case 15: hipLaunchKernelGGL(k_gram_chol_lag<15>, dim3(d.nmat), dim3(512), lds, st, d, Tslot, ls, cs, iVdiag); break;
  }
  return hipGetLastError();
}

// row-owned substitutions with LDS flag hand-offs (RO, option solve_async = 1) or the barrier-stepped
// form (solve_async = 0).  Same arithmetic either way (per-thread v_t and residual rows, per-tile
// substitution products, the X'v t-halves on threads 0..511).
template <int NT, int NM, bool RO>
static hipError_t solve_ro(hipStream_t st, size_t lds, Dims d, const int* Tslot, const double* iVb, XSel xs,
                           LagSel ls, ChainState cs, RngArgs ra, SolveXch xc) {
  hipError_t e = hipFuncSetAttribute((const void*)k_cta_solve_lag<NT, NM, 8, RO>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_cta_solve_lag<NT, NM, 8, RO>), dim3(d.B, xc.part ? 2 : 1), dim3(64 * 8), lds, st, d,
                     Tslot, iVb, xs, ls, cs, ra, xc);
  return hipGetLastError();
}

template <int NT, int NM, bool RO>
static int solve_resident(size_t lds) {
  const void* fn = (const void*)k_cta_solve_lag<NT, NM, 8, RO>;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return 0;
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * 8, lds) != hipSuccess) return 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return per_cu * cus;
}

int lag_solve_resident(int NT, int nmax, size_t lds, int async) {
#define SR_CASE(NT_, NM_)                                                                              \
  if (NT == NT_ && nmax == NM_) return async ? solve_resident<NT_, NM_, true>(lds) : solve_resident<NT_, NM_, false>(lds);
  SR_CASE(1, 8) SR_CASE(1, 20) SR_CASE(1, 32) SR_CASE(15, 8) SR_CASE(15, 20) SR_CASE(15, 32)
#undef SR_CASE
  return 0;
}

hipError_t lag_launch_solve(int NT, int nmax, int async, hipStream_t st, size_t lds, Dims d, const int* Tslot,
                            const double* iVb, XSel xs, LagSel ls, ChainState cs, RngArgs ra, SolveXch xc) {
#define SL_CASE(NT_, NM_)                                                                           \
  if (NT == NT_ && nmax == NM_)                                                                     \
    return async ? solve_ro<NT_, NM_, true>(st, lds, d, Tslot, iVb, xs, ls, cs, ra, xc)            \
                 : solve_ro<NT_, NM_, false>(st, lds, d, Tslot, iVb, xs, ls, cs, ra, xc);
  SL_CASE(1, 8) SL_CASE(1, 20) SL_CASE(1, 32) SL_CASE(15, 8) SL_CASE(15, 20) SL_CASE(15, 32)
#undef SL_CASE
  return hipErrorInvalidValue;
}

}  // namespace ccmm
