// HIP/CDNA4 (gfx950) kernels of the CCMM BVAR-SV Gibbs sweep.
//
// One "system" is one (chain, equation) pair of the triangular CTA algorithm
// (CTA.m:60-98).  The per-sweep pipeline for B chains is
//
//   k_cta_weights   w_t^(j) = sum_{i>=j} A(i,j)^2 / sqrtht(t,i)^2        (elementwise)
//   k_gram_chol     G_cj = X' diag(w^(j)) X + diag(iV_j) and its Cholesky factor on
//                   v_mfma_f64_16x16x4_f64 (ccmm_gram_chol.hip; ccmm_lag.hip for lag designs)
//   k_cta_solve2    per chain, j = 1..N in order: rhs = iVb_j + X' v^(j) (needs the
//                   draws of equations < j), L L' x = rhs, PAI(:,j) = L'^-1 (L^-1 rhs + z_j),
//                   residual update (ccmm_cta_solve.hip)               (latency bound)
//   k_astep         A-matrix rows (mcmcVAR.m:236-254), invA, logy2 (mcmcVAR.m:259)
//   k_sv_mix        KSC mixture indicators (elementwise)
//   k_sv_part       partitioned block-tridiagonal sampler of h_0..h_T (ccmm_svpart.hip)
//   k_phi_gen/k_phi inverse-Wishart PHI draw (mcmcVAR.m:268-274)
//   k_store         kept-draw storage (mcmcVAR.m:289-292)
//
// The algebraic identity X_j'X_j = X' diag(w) X, X_j'Y_j = X' v
// removes the kron materialisation of CTA.m:69 (T(N-j+1) x K per equation).
#include "ccmm_sweep.h"

namespace ccmm {

// dst[q] = src[q] for q < n (a global -> LDS staging copy): sixteen loads per thread are issued
// before their stores, one round trip per sixteen elements instead of one per element
__device__ __forceinline__ void stage_copy16(double* dst, const double* __restrict__ src, int n, int tid, int nth) {
  for (int q0 = tid; q0 < n; q0 += 16 * nth) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = (q0 + u * nth < n) ? src[q0 + u * nth] : 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (q0 + u * nth < n) dst[q0 + u * nth] = v[u];
  }
}

// ============================================================== residual
// E(:,j) = Y(:,j) - X_j * PAI(:,j)   (mcmcVAR.m:233; CTAsys residual mcmcVARshadowrateBlockHybrid.m:348-351)
__global__ void k_resid(Dims d, const int* __restrict__ Tslot, XSel xs, ChainState cs) {
  const int c = blockIdx.z, j = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= d.TP) return;
  const int T = Tslot[cs.slot[c]];
  double* E = cs.E + ((size_t)c * d.N + j) * d.TP;
  if (t >= T) {
    E[t] = 0.0;
    return;
  }
  const double* X = xs.pool + (size_t)xs.idx[c * d.N + j] * d.KP * d.TP;
  const double* Y = xs.ypool + (size_t)xs.yidx[c] * d.N * d.TP;
  const double* pai = cs.PAI + ((size_t)c * d.N + j) * d.KP;
  double acc = 0.0;
  for (int a = 0; a < d.K; ++a) acc = fma(X[(size_t)a * d.TP + t], pai[a], acc);
  E[t] = Y[(size_t)j * d.TP + t] - acc;
}

// E = Y - X PAI for all N equations of chain c in one pass over each distinct design slab
// (the block-hybrid and hybrid models give equations of one chain a shared shadow-rate or
// actual-rate slab): thread per t, the chain's PAI masked to the slab's equations in LDS
// (row a = NB coefficients, read as broadcasts), NB accumulators per thread.  k_resid reads
// the KP x TP slab once per equation, N times the bytes.  Same fma order over a per
// equation as k_resid (other slabs' equations add exact zeros), so E is bit-identical.
template <int NB>
__global__ __launch_bounds__(256) void k_resid_multi(Dims d, const int* __restrict__ Tslot, XSel xs,
                                                     ChainState cs) {
  extern __shared__ double spai[];  // K x NB
  const int c = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int N = d.N, K = d.K;
  const int T = Tslot[cs.slot[c]];
  const int* idx = xs.idx + (size_t)c * N;
  const double* pai = cs.PAI + (size_t)c * N * d.KP;
  double acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = 0.0;
  const unsigned full = (N >= 32) ? 0xffffffffu : ((1u << N) - 1u);
  unsigned done = 0;
  while (done != full) {
    const int s = idx[__builtin_ctz(~done & full)];
    unsigned m = 0;
    for (int j = 0; j < N; ++j) m |= (idx[j] == s) ? (1u << j) : 0u;
    __syncthreads();  // the previous slab's readers are done with spai
    for (int q = threadIdx.x; q < K * NB; q += 256) {
      const int a = q / NB, j = q - a * NB;
      spai[q] = (j < N && ((m >> j) & 1u)) ? pai[(size_t)j * d.KP + a] : 0.0;
    }
    __syncthreads();
    if (t < T) {
      const double* X = xs.pool + (size_t)s * d.KP * d.TP + t;
      for (int a = 0; a < K; ++a) {
        const double x = X[(size_t)a * d.TP];
        const double* row = spai + a * NB;
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j] = fma(x, row[j], acc[j]);
      }
    }
    done |= m;
  }
  if (t < d.TP) {
    const double* Y = xs.ypool + (size_t)xs.yidx[c] * N * d.TP;
    double* E = cs.E + (size_t)c * N * d.TP;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (j < N) E[(size_t)j * d.TP + t] = (t < T) ? Y[(size_t)j * d.TP + t] - acc[j] : 0.0;
  }
}

// ============================================================== CTA weights
// w_t^(j) = sum_{i>=j} A(i,j)^2 / sqrtht(t,i)^2 : the diagonal of kron(A(j:N,j),X)./lambda's
// Gram (CTA.m:66-73).  Padded rows get weight 0.
__global__ void k_cta_weights(Dims d, const int* __restrict__ Tslot, ChainState cs, int sqrt_form) {
  const int c = blockIdx.z, j = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= d.TP) return;
  const int T = Tslot[cs.slot[c]];
  double w = 0.0;
  if (t < T) {
    const bool elbm = cs.atELB && cs.atELB[(size_t)c * d.TP + t];  // CTAsysAswitching.m:68-80
    const double* A = (elbm ? cs.Aelb : cs.A) + (size_t)c * d.N * d.N;
    const double* sh = cs.sqrtht + (size_t)c * d.N * d.TP;
    for (int i = j; i < d.N; ++i) {
      const double a = A[i + j * d.N] / sh[(size_t)i * d.TP + t];
      w = fma(a, a, w);
    }
  }
  cs.W[((size_t)c * d.N + j) * d.TP + t] = sqrt_form ? sqrt(w) : w;
  // 1 / sqrtht(t, j)^2 for the residual weights of the sequential solve
  double ihv = 0.0;
  if (t < T) {
    const double shv = cs.sqrtht[((size_t)c * d.N + j) * d.TP + t];
    ihv = 1.0 / (shv * shv);
  }
  cs.ih2[((size_t)c * d.N + j) * d.TP + t] = ihv;
}

// ============================================================== A-step
// mcmcVAR.m:236-254 (flat prior: OMEGA_A_inv = 0, MU_A = 0, mcmcVAR.m:153-161),
// invA = A \ I (mcmcVAR.m:254), logy2 = log((RESID*A').^2 + offset) (mcmcVAR.m:259).
// LDS: per ii a packed lower ZZ (ii x ii) followed by Zz (ii).

// The Gram entries of every regression ii = 1..N-1,
//   ZZ_ii(a, b) = sum_t E(a,t) E(b,t) w_ii(t)  (b <= a < ii),   Zz_ii(b) = the same with a = ii,
//   w_ii(t) = 1 / sqrtht(ii,t)^2,
// as 4 x 4 register tiles: gtab = [ntiles, ii << 16 | A << 8 | B ...] (host-built, largest ii first),
// rows 4A.., columns 4B..; each 16-lane row of a wave takes one tile, lane j the months t = j mod 16
// (sequential fused multiply-adds fma(E_a E_b, w, acc)), then a DPP tree over the row's 16 lanes.
// The weights are formed once per chain into the chain's logy2 rows (overwritten by logy2 at the end
// of the A-step).  Per entry the arithmetic depends on the tile alone, so every launch shape gives the
// same sums.  (Before: one wave per entry, 2 LDS reads per product and a 64-lane reduction per entry.)
__device__ __forceinline__ void astep_gram_tiles(const double* Ew, const double* sh, double* W, double* sm,
                                                 const int* boff, const int* __restrict__ gtab, int N, int TP,
                                                 int T, int tid, int nthreads) {
  for (int q = tid; q < (N - 1) * TP; q += nthreads) {
    const int ii = 1 + q / TP, t = q - (ii - 1) * TP;
    const double hv = (t < T) ? sh[(size_t)ii * TP + t] : 1.0;
    W[q] = (t < T) ? 1.0 / (hv * hv) : 0.0;
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6, nwv = nthreads >> 6;
  const int r = lane >> 4, j = lane & 15;
  const int ntiles = gtab[0];
  for (int g0 = 4 * wave; g0 < ntiles; g0 += 4 * nwv) {
    const int gi = g0 + r;
    const int v = gi < ntiles ? gtab[1 + gi] : gtab[1];  // idle rows redo tile 0 and store nothing
    const int ii = v >> 16, A4 = 4 * ((v >> 8) & 255), B4 = 4 * (v & 255);
    const double* ea[4];
    const double* eb[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      ea[p] = Ew + (size_t)min(A4 + p, N - 1) * TP;
      eb[p] = Ew + (size_t)min(B4 + p, N - 1) * TP;
    }
    const double* wr = W + (size_t)(ii - 1) * TP;
    double acc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.0;
    // the weights (global, L2) run kAsPf months ahead of the products in a register ring, so no
    // load latency sits between two batches of fused multiply-adds
    constexpr int kAsPf = 8;
    const int M = (T - j + 15) >> 4;  // months t = j + 16 m < T of this lane
    double wq[kAsPf];
#pragma unroll
    for (int u = 0; u < kAsPf; ++u) wq[u] = (u < M) ? wr[j + 16 * u] : 0.0;
    for (int m0 = 0; m0 < M; m0 += kAsPf) {
      double wn[kAsPf];
#pragma unroll
      for (int u = 0; u < kAsPf; ++u) wn[u] = (m0 + kAsPf + u < M) ? wr[j + 16 * (m0 + kAsPf + u)] : 0.0;
#pragma unroll
      for (int u = 0; u < kAsPf; ++u) {
        if (m0 + u < M) {
          const int t = j + 16 * (m0 + u);
          double xa[4], xb[4];
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            xa[p] = ea[p][t];
            xb[p] = eb[p][t];
          }
#pragma unroll
          for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[4 * p + q] = fma(xa[p] * xb[q], wq[u], acc[4 * p + q]);
        }
      }
#pragma unroll
      for (int u = 0; u < kAsPf; ++u) wq[u] = wn[u];
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] += dpp_d<0xB1>(acc[e]);   // xor 1
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] += dpp_d<0x4E>(acc[e]);   // xor 2
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] += dpp_d<0x141>(acc[e]);  // row_half_mirror
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] += dpp_d<0x140>(acc[e]);  // row_mirror: the row sum
    // lane j of the row stores entry (A4 + j / 4, B4 + j % 4)
    double mine = acc[0];
#pragma unroll
    for (int e = 1; e < 16; ++e) mine = (j == e) ? acc[e] : mine;
    const int a = A4 + (j >> 2), b = B4 + (j & 3);
    if (gi < ntiles && a <= ii && b < ii && b <= a) {
      const int o = (a < ii) ? b * ii - b * (b - 1) / 2 + (a - b) : ii * (ii + 1) / 2 + b;
      sm[boff[ii] + o] = mine;
    }
  }
}

// logy2 = log((RESID * A').^2 + offset) (mcmcVAR.m:259): one month per thread, its residuals read
// once into registers (NN >= N), row i's sum over k <= i in ascending order
template <int NN>
__device__ __forceinline__ void astep_logy2(const double* Ew, const double* Anew, double* ly, int N, int TP,
                                            int T, int tid, int nthreads, double logy2offset) {
  for (int t = tid; t < TP; t += nthreads) {
    double e[NN];
#pragma unroll
    for (int k = 0; k < NN; ++k) e[k] = (k < N && t < T) ? Ew[(size_t)k * TP + t] : 0.0;
    for (int i = 0; i < N; ++i) {
      double sacc = 0.0;
      if (t < T) {
#pragma unroll
        for (int k = 0; k < NN; ++k)
          if (k <= i) sacc = fma(e[k], Anew[i + k * N], sacc);
      }
      ly[(size_t)i * TP + t] = (t < T) ? log(sacc * sacc + logy2offset) : 0.0;
    }
  }
}

__global__ __launch_bounds__(256) void k_astep(Dims d, const int* __restrict__ Tslot, ChainState cs,
                                               RngArgs ra, double logy2offset, int es_off,
                                               const int* __restrict__ gtab) {
  extern __shared__ double sm[];
  const int c = blockIdx.x;
  const int N = d.N, TP = d.TP;
  const int T = Tslot[cs.slot[c]];
  const int tid = threadIdx.x;
  const Rng rng = ra.make(c);
  const double* E = cs.E + (size_t)c * N * TP;
  const double* sh = cs.sqrtht + (size_t)c * N * TP;
  double* Ac = cs.A + (size_t)c * N * N;
  double* Ainv = cs.invA + (size_t)c * N * N;
  // offsets: block ii (1..N-1) has ii*(ii+1)/2 + ii entries
  __shared__ int boff[kMaxNSmall + 1];
  if (tid == 0) {
    int o = 0;
    boff[0] = 0;
    boff[1] = 0;
    for (int ii = 1; ii < N; ++ii) {
      boff[ii] = o;
      o += ii * (ii + 1) / 2 + ii;
    }
    boff[N] = o;
  }
  // es_off >= 0: this chain's residuals E (N x TP) are staged in LDS at sm + es_off
  if (es_off >= 0)
    stage_copy16(sm + es_off, E, N * TP, tid, blockDim.x);
  __syncthreads();
  const double* Ew = (es_off >= 0) ? sm + es_off : E;
  const int total = boff[N];
  double* Anew = sm + total;  // N x N
  astep_gram_tiles(Ew, sh, cs.logy2 + (size_t)c * N * TP, sm, boff, gtab, N, TP, T, tid, blockDim.x);
  for (int q = tid; q < N * N; q += blockDim.x) Anew[q] = ((q % N) == (q / N)) ? 1.0 : 0.0;
  __syncthreads();
  // per-ii Cholesky + solves, one thread per ii
  if (tid >= 1 && tid < N) {
    const int ii = tid;
    double* Lp = sm + boff[ii];  // packed lower by columns, ii x ii
    double* zz = Lp + ii * (ii + 1) / 2;
    auto idx = [ii](int r, int col) { return col * ii - col * (col - 1) / 2 + (r - col); };
    int badf = 0;
    for (int col = 0; col < ii; ++col) {
      double dcc = Lp[idx(col, col)];
      for (int q = 0; q < col; ++q) dcc -= Lp[idx(col, q)] * Lp[idx(col, q)];
      if (!(dcc > 0.0)) {
        badf = 1;
        dcc = 1.0;
      }
      const double piv = sqrt(dcc);
      Lp[idx(col, col)] = piv;
      for (int r = col + 1; r < ii; ++r) {
        double s = Lp[idx(r, col)];
        for (int q = 0; q < col; ++q) s -= Lp[idx(r, q)] * Lp[idx(col, q)];
        Lp[idx(r, col)] = s / piv;
      }
    }
    // tilde = L \ Zz  (in place in zz)
    for (int r = 0; r < ii; ++r) {
      double s = zz[r];
      for (int q = 0; q < r; ++q) s -= Lp[idx(r, q)] * zz[q];
      zz[r] = s / Lp[idx(r, r)];
    }
    const int zoff = ii * (ii - 1) / 2;
    for (int r = 0; r < ii; ++r) zz[r] += rng.normal(CCMM_RNG_A, (uint32_t)(zoff + r));
    // alpha = L' \ (tilde + z)
    for (int r = ii - 1; r >= 0; --r) {
      double s = zz[r];
      for (int q = r + 1; q < ii; ++q) s -= Lp[idx(q, r)] * zz[q];
      zz[r] = s / Lp[idx(r, r)];
    }
    for (int q = 0; q < ii; ++q) Anew[ii + q * N] = -zz[q];
    if (badf) atomicOr(&cs.status[c], 4);
  }
  __syncthreads();
  for (int q = tid; q < N * N; q += blockDim.x) Ac[q] = Anew[q];
  // invA: column col of A^{-1} by forward substitution (unit lower); the column is built
  // in LDS (sm[0..N*N) is free after the solves) rather than a dynamically indexed array
  double* Xs = sm;
  if (tid < N) {
    const int col = tid;
    for (int r = 0; r < N; ++r) {
      double s = (r == col) ? 1.0 : 0.0;
      for (int q = col; q < r; ++q) s -= Anew[r + q * N] * Xs[q + col * N];
      Xs[r + col * N] = (r >= col) ? s : 0.0;
    }
    for (int r = 0; r < N; ++r) Ainv[r + col * N] = Xs[r + col * N];
  }
  astep_logy2<kMaxNSmall>(Ew, Anew, cs.logy2 + (size_t)c * N * TP, N, TP, T, tid, blockDim.x, logy2offset);
}

// ============================================================== A-step, wave-parallel form
// The same draws as k_astep (mcmcVAR.m:236-254, 259) with the per-regression work spread over
// waves instead of one thread per regression: 8 waves share the Gram tiles (astep_gram_tiles,
// E staged in LDS), then each wave factors whole regressions ii in
// registers (lane r holds row r of ZZ_ii: readlane broadcasts of the pivot row, the same
// left-to-right update order as k_astep's left-looking loop) and solves L tilde = Zz,
// alpha = L' \ (tilde + z) by lane substitutions; wave 0 forms invA by lane-per-column
// forward substitution.  Regressions are dealt to waves largest first in snake order.
#ifdef CCMM_ABLATION
// timing-only phase attribution of k_astep_w (ablation build): shader-clock cycles of chain 0's
// workgroup between its barriers (stage E | Gram | factor + solves | invA | logy2), read by
// ccmm_astep_prof
__device__ unsigned long long g_astep_prof[8];
extern "C" int ccmm_astep_prof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_astep_prof), sizeof(g_astep_prof)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_astep_prof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#define AS_CLK(x) const unsigned long long x = clock64()
#define AS_ACC(k, a, b) \
  if (c == 0 && tid == 0) atomicAdd(&g_astep_prof[k], (b) - (a))
#else
#define AS_CLK(x)
#define AS_ACC(k, a, b)
#endif
template <int NN>
__global__ __launch_bounds__(512) void k_astep_w(Dims d, const int* __restrict__ Tslot, ChainState cs,
                                                 RngArgs ra, double logy2offset, int es_off,
                                                 const int* __restrict__ gtab) {
  extern __shared__ double sm[];
  constexpr int kWaves = 8;
  const int c = blockIdx.x;
  const int N = d.N, TP = d.TP;
  const int T = Tslot[cs.slot[c]];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Rng rng = ra.make(c);
  const double* E = cs.E + (size_t)c * N * TP;
  const double* sh = cs.sqrtht + (size_t)c * N * TP;
  double* Ac = cs.A + (size_t)c * N * N;
  double* Ainv = cs.invA + (size_t)c * N * N;
  __shared__ int boff[kMaxNSmall + 1];
  AS_CLK(k0);
  if (tid == 0) {
    int o = 0;
    boff[0] = 0;
    boff[1] = 0;
    for (int ii = 1; ii < N; ++ii) {
      boff[ii] = o;
      o += ii * (ii + 1) / 2 + ii;
    }
    boff[N] = o;
  }
  if (es_off >= 0)
    stage_copy16(sm + es_off, E, N * TP, tid, blockDim.x);
  __syncthreads();
  AS_CLK(k1);
  const double* Ew = (es_off >= 0) ? sm + es_off : E;
  const int total = boff[N];
  double* Anew = sm + total;  // N x N
  // ---- Gram entries (the same tiles as k_astep)
  astep_gram_tiles(Ew, sh, cs.logy2 + (size_t)c * N * TP, sm, boff, gtab, N, TP, T, tid, 512);
  for (int q = tid; q < N * N; q += blockDim.x) Anew[q] = ((q % N) == (q / N)) ? 1.0 : 0.0;
  __syncthreads();
  AS_CLK(k2);
  // ---- per-regression factor + solves, one wave per regression ii (rows on lanes)
  int badf = 0;
  for (int r8 = 0;; ++r8) {
    // snake order over ii = N-1 .. 1: round r8 gives wave w the (w or 7-w)-th of that round
    const int pos = r8 * kWaves + ((r8 & 1) ? (kWaves - 1 - wave) : wave);
    const int ii = N - 1 - pos;
    if (ii < 1) break;
    double* Lp = sm + boff[ii];  // packed lower by columns, ii x ii, then Zz
    const double* zz = Lp + ii * (ii + 1) / 2;
    auto idx = [ii](int r, int col) { return col * ii - col * (col - 1) / 2 + (r - col); };
    const int rl = lane < ii ? lane : 0;
    double s[NN];
#pragma unroll
    for (int q = 0; q < NN; ++q) s[q] = (q <= rl && q < ii && lane < ii) ? Lp[idx(rl, q)] : 0.0;
    double piv[NN];
#pragma unroll
    for (int q = 0; q < NN; ++q) {
      if (q < ii) {
        double dq = readlane_d(s[q], q);
        if (!(dq > 0.0)) {
          badf = 1;
          dq = 1.0;
        }
        const double pq = sqrt(dq);
        piv[q] = pq;
        s[q] = (lane == q) ? pq : s[q] / pq;
        // row r > q, entries q < k <= r: s[k] -= L(r, q) L(k, q)
#pragma unroll
        for (int k = q + 1; k < NN; ++k)
          if (k < ii) s[k] = fma(-s[q], readlane_d(s[q], k), s[k]);
      }
    }
    // tilde = L \ Zz (lane r holds entry r), + z, then alpha = L' \ (tilde + z)
    double y = (lane < ii) ? zz[rl] : 0.0;
#pragma unroll
    for (int k = 0; k < NN; ++k) {
      if (k < ii) {
        const double yk = readlane_d(y, k) / piv[k];
        y = (lane == k) ? yk : ((lane > k) ? fma(-s[k], yk, y) : y);
      }
    }
    const int zoff = ii * (ii - 1) / 2;
    if (lane < ii) y += rng.normal(CCMM_RNG_A, (uint32_t)(zoff + lane));
    // back substitution in k_astep's order: x_r = (v_r - sum_{q > r, ascending} L(q, r) x_q) / L(r, r),
    // evaluated uniformly (the factor goes back to the packed slots and is read by broadcast)
    if (lane < ii) {
#pragma unroll
      for (int q = 0; q < NN; ++q)
        if (q <= rl && q < ii) Lp[idx(rl, q)] = s[q];
    }
    wave_lds_sync();
    double xs[NN];
#pragma unroll
    for (int r = NN - 1; r >= 0; --r) {
      xs[r] = 0.0;
      if (r < ii) {
        double v = readlane_d(y, r);
#pragma unroll
        for (int q = r + 1; q < NN; ++q)
          if (q < ii) v = fma(-Lp[idx(q, r)], xs[q], v);
        xs[r] = v / piv[r];
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < NN; ++q)
        if (q < ii) Anew[ii + q * N] = -xs[q];
    }
    wave_lds_sync();
  }
  if (badf && lane == 0) atomicOr(&cs.status[c], 4);
  __syncthreads();
  AS_CLK(k3);
  for (int q = tid; q < N * N; q += blockDim.x) Ac[q] = Anew[q];
  // invA: lane col forms column col of A^-1 (unit lower forward substitution, A read by
  // broadcast from LDS)
  if (wave == 0) {
    const int col = lane;
    double x[NN];
#pragma unroll
    for (int r = 0; r < NN; ++r) {
      double v = (r == col) ? 1.0 : 0.0;
#pragma unroll
      for (int q = 0; q < r; ++q)
        if (q >= col && r < N) v = fma(-Anew[r + q * N], x[q], v);  // rows r >= N (NN > N) stay out of A
      x[r] = (r >= col && r < N) ? v : 0.0;
    }
    if (col < N) {
#pragma unroll
      for (int r = 0; r < NN; ++r)
        if (r < N) Ainv[r + col * N] = x[r];
    }
  }
  AS_CLK(k4);
  astep_logy2<NN>(Ew, Anew, cs.logy2 + (size_t)c * N * TP, N, TP, T, tid, blockDim.x, logy2offset);
#ifdef CCMM_ABLATION
  __syncthreads();
  AS_CLK(k5);
  AS_ACC(0, k0, k1);
  AS_ACC(1, k1, k2);
  AS_ACC(2, k2, k3);
  AS_ACC(3, k3, k4);
  AS_ACC(4, k4, k5);
  if (c == 0 && tid == 0) atomicAdd(&g_astep_prof[5], 1ull);
#endif
}

// ============================================================== SV: KSC mixture indicators
__constant__ double cKSCprob[7] = {0.00730, 0.10556, 0.00002, 0.04395, 0.34001, 0.24566, 0.25750};
__constant__ double cKSCmean[7] = {-10.12999 - 1.2704, -3.97281 - 1.2704, -8.56686 - 1.2704,
                                   2.77786 - 1.2704,   0.61942 - 1.2704,  1.79518 - 1.2704,
                                   -1.08819 - 1.2704};
__constant__ double cKSCvar[7] = {5.79596, 2.61369, 5.17950, 0.16735, 0.64009, 0.34023, 1.26261};

__global__ void k_sv_mix(Dims d, const int* __restrict__ Tslot, ChainState cs, RngArgs ra) {
  const int c = blockIdx.y;
  const int T = Tslot[cs.slot[c]];
  const int q = blockIdx.x * blockDim.x + threadIdx.x;  // q = i*TP + t
  if (q >= d.N * d.TP) return;
  const int i = q / d.TP, t = q % d.TP;
  const size_t o = (size_t)c * d.N * d.TP + q;
  if (t >= T) {
    cs.svobs[o] = 0.0;
    cs.svir[o] = 0.0;
    cs.kai[o] = 0;
    return;
  }
  const Rng rng = ra.make(c);
  const double u = rng.uniform(CCMM_RNG_SVU, (uint32_t)(i + d.N * t));
  const double y = cs.logy2[o], hp = cs.h[o];
  double cdf[7];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const double vol = sqrt(cKSCvar[k]);
    const double e = (y - hp - cKSCmean[k]) / vol;
    acc += cKSCprob[k] / vol * exp(-0.5 * e * e);
    cdf[k] = acc;
  }
  int s = 1;
#pragma unroll
  for (int k = 0; k < 6; ++k) s += (u > cdf[k] / cdf[6]) ? 1 : 0;
  cs.kai[o] = (int8_t)s;
  cs.svobs[o] = y - cKSCmean[s - 1];
  cs.svir[o] = 1.0 / cKSCvar[s - 1];
}

// ============================================================== small SPD helpers (PHI block)
// Cholesky (left-looking, in place, lower triangle of row-major S) by the
// threads of the whole workgroup (only threads < N work; all reach the barriers).
__device__ void wg_chol_lds(double* S, int N, int NS, int tid, int* bad) {
  for (int col = 0; col < N; ++col) {
    if (tid >= col && tid < N) {
      double s = S[tid * NS + col];
      for (int q = 0; q < col; ++q) s = fma(-S[tid * NS + q], S[col * NS + q], s);
      S[tid * NS + col] = s;
    }
    __syncthreads();
    const double dcc = S[col * NS + col];
    double piv = sqrt(dcc);
    if (!(dcc > 0.0)) {
      *bad = 1;
      piv = 1.0;
    }
    __syncthreads();
    if (tid > col && tid < N) S[tid * NS + col] /= piv;
    if (tid == col) S[col * NS + col] = piv;
    __syncthreads();
  }
}


// ============================================================== PHI inverse-Wishart
// mcmcVAR.m:268-274: Zdraw = randn(N, T+d_PHI); sqrtPHIpost = chol(s_PHI + eta'eta,'lower');
// sqrtZZ = chol(Zdraw*Zdraw'); sqrtPHI_ = sqrtPHIpost / sqrtZZ; PHI_ = sqrtPHI_*sqrtPHI_';
// sqrtPHI_ = chol(PHI_,'lower').
__global__ void k_phi_gen(Dims d, const int* __restrict__ Tslot, int dPHI, ChainState cs,
                          RngArgs ra) {
  const int c = blockIdx.y;
  const int TZ = Tslot[cs.slot[c]] + dPHI;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;  // q = i + N*col (N x TZ column-major)
  if (q >= d.N * TZ) return;
  const Rng rng = ra.make(c);
  cs.Zphi[(size_t)c * d.N * (d.TP + dPHI) + q] = rng.normal(CCMM_RNG_PHI, (uint32_t)q);
}

__global__ __launch_bounds__(256) void k_phi(Dims d, const int* __restrict__ Tslot, int dPHI,
                                             const double* __restrict__ sPHIall, ChainState cs,
                                             int stage_eta) {
  extern __shared__ double sm[];
  const int N = d.N, NS = N + 1, TP = d.TP;
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int T = Tslot[s];
  const int TZ = T + dPHI;
  const int TZmax = TP + dPHI;
  const int tid = threadIdx.x;
  double* Lpost = sm;           // N x NS
  double* Rz = Lpost + N * NS;  // N x NS (lower chol of ZZ', i.e. R')
  double* Sq = Rz + N * NS;     // N x NS
  double* Ph = Sq + N * NS;     // N x NS
  const double* eta = cs.eta + (size_t)c * N * TP;
  const double* Z = cs.Zphi + (size_t)c * N * TZmax;
  const double* sP = sPHIall + (size_t)s * N * N;
  // stage_eta: the SV shocks eta (N x T) go to LDS with odd row stride TP + 1, so the
  // lanes of a wave (different rows r, same t) hit different banks
  const int lde = stage_eta ? TP + 1 : TP;
  const double* etaw = eta;
  if (stage_eta) {
    double* es = Ph + N * NS;
    // sixteen loads per thread issued before their LDS stores (one round trip per sixteen)
    const int nth = blockDim.x;
    for (int q0 = tid; q0 < N * TP; q0 += 16 * nth) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = (q0 + u * nth < N * TP) ? eta[q0 + u * nth] : 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int q = q0 + u * nth;
        if (q < N * TP) {
          const int r = q / TP, t = q - r * TP;
          es[r * lde + t] = v[u];
        }
      }
    }
    __syncthreads();
    etaw = es;
  }
  for (int e = tid; e < N * N; e += blockDim.x) {
    const int r = e / N, col = e % N;
    if (col > r) continue;
    // four independent partial sums: the T-long dot products are serial fma chains on
    // one thread each, so their latency, not the fma count, sets the kernel time
    const double* er = etaw + (size_t)r * lde;
    const double* ec = etaw + (size_t)col * lde;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int t = 0;
    for (; t + 3 < T; t += 4) {
      a0 = fma(er[t], ec[t], a0);
      a1 = fma(er[t + 1], ec[t + 1], a1);
      a2 = fma(er[t + 2], ec[t + 2], a2);
      a3 = fma(er[t + 3], ec[t + 3], a3);
    }
    for (; t < T; ++t) a0 = fma(er[t], ec[t], a0);
    Lpost[r * NS + col] = sP[r + col * N] + ((a0 + a1) + (a2 + a3));
  }
  // stage_eta bit 1: Z (N x TZ, k_phi_gen) follows eta into the same LDS region, one coalesced pass,
  // so that the ZZ' chains read LDS instead of strided HBM rows (~0.2 ms of global-load latency per
  // launch at B = 1); the same products in the same order
  const double* Zw = Z;
  if (stage_eta & 2) {
    double* zs = Ph + N * NS;
    __syncthreads();
    for (int q0 = tid; q0 < N * TZ; q0 += 16 * (int)blockDim.x) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = (q0 + u * (int)blockDim.x < N * TZ) ? Z[q0 + u * blockDim.x] : 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (q0 + u * (int)blockDim.x < N * TZ) zs[q0 + u * blockDim.x] = v[u];
    }
    __syncthreads();
    Zw = zs;
  }
  for (int e = tid; e < N * N; e += blockDim.x) {
    const int r = e / N, col = e % N;
    if (col > r) continue;
    const double* zr = Zw + r;
    const double* zc = Zw + col;
    double b0 = 0.0, b1 = 0.0, b2 = 0.0, b3 = 0.0;
    int q = 0;
    for (; q + 3 < TZ; q += 4) {
      b0 = fma(zr[(size_t)N * q], zc[(size_t)N * q], b0);
      b1 = fma(zr[(size_t)N * (q + 1)], zc[(size_t)N * (q + 1)], b1);
      b2 = fma(zr[(size_t)N * (q + 2)], zc[(size_t)N * (q + 2)], b2);
      b3 = fma(zr[(size_t)N * (q + 3)], zc[(size_t)N * (q + 3)], b3);
    }
    for (; q < TZ; ++q) b0 = fma(zr[(size_t)N * q], zc[(size_t)N * q], b0);
    Rz[r * NS + col] = (b0 + b1) + (b2 + b3);
  }
  __syncthreads();
  int bad = 0;
  wg_chol_lds(Lpost, N, NS, tid, &bad);
  wg_chol_lds(Rz, N, NS, tid, &bad);
  // Sq R = Lpost with R = Rz' upper: row `tid` of Sq
  if (tid < N) {
    const int r = tid;
    for (int col = 0; col < N; ++col) {
      double v = (col <= r) ? Lpost[r * NS + col] : 0.0;
      for (int q = 0; q < col; ++q) v = fma(-Sq[r * NS + q], Rz[col * NS + q], v);
      Sq[r * NS + col] = v / Rz[col * NS + col];
    }
  }
  __syncthreads();
  // PHI = Sq Sq'
  for (int e = tid; e < N * N; e += blockDim.x) {
    const int r = e / N, col = e % N;
    double v = 0.0;
    for (int q = 0; q < N; ++q) v = fma(Sq[r * NS + q], Sq[col * NS + q], v);
    Ph[r * NS + col] = v;
  }
  __syncthreads();
  double* PHI = cs.PHI + (size_t)c * N * N;
  for (int e = tid; e < N * N; e += blockDim.x) {
    const int r = e % N, col = e / N;
    PHI[e] = Ph[r * NS + col];
  }
  __syncthreads();
  wg_chol_lds(Ph, N, NS, tid, &bad);
  double* sqo = cs.sqrtPHI + (size_t)c * N * N;
  for (int e = tid; e < N * N; e += blockDim.x) {
    const int r = e % N, col = e / N;
    sqo[e] = (col <= r) ? Ph[r * NS + col] : 0.0;
  }
  if (bad && tid == 0) atomicOr(&cs.status[c], 16);
}

// ============================================================== draw storage

__global__ void k_store(Dims d, ChainState cs, Store st) {
  const int c = blockIdx.y;
  const int N = d.N, K = d.K, TP = d.TP;
  const int nPAI = K * N, nPHI = N * (N + 1) / 2, nA = N * N, nS = st.Tmax * N;
  const int tot = nPAI + nPHI + nA + nS;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < tot; q += gridDim.x * blockDim.x) {
    if (q < nPAI) {
      const int a = q % K, j = q / K;
      st.PAI[((size_t)c * st.cap + st.m) * nPAI + q] = cs.PAI[((size_t)c * N + j) * d.KP + a];
    } else if (q < nPAI + nPHI) {
      int e = q - nPAI, col = 0;
      while (e >= N - col) {
        e -= N - col;
        ++col;
      }
      const int r = col + e;
      st.PHI[((size_t)c * st.cap + st.m) * nPHI + (q - nPAI)] = cs.PHI[(size_t)c * N * N + r + col * N];
    } else if (q < nPAI + nPHI + nA) {
      const int e = q - nPAI - nPHI;
      st.invA[((size_t)c * st.cap + st.m) * nA + e] = cs.invA[(size_t)c * N * N + e];
    } else {
      const int e = q - nPAI - nPHI - nA;
      const int t = e % st.Tmax, i = e / st.Tmax;
      st.sqrtht[((size_t)c * st.cap + st.m) * nS + e] = cs.sqrtht[((size_t)c * N + i) * TP + t];
    }
  }
}

// running sums of the stored PAI draws m0 <= m < m1 per (chain, entry), in store order; no contraction
// (x * x rounded, then added), the order and rounding of the host loop it replaces
__global__ void k_pai_moments(const double* __restrict__ sPAI, int cap, int m0, int m1, int per, int B,
                              double* __restrict__ sum, double* __restrict__ sumsq) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (size_t)B * per) return;
  const size_t c = q / per, e = q - c * per;
  double s = sum[q], s2 = sumsq[q];
  for (int m = m0; m < m1; ++m) {
    const double x = sPAI[(c * cap + m) * per + e];
    s = __dadd_rn(s, x);
    s2 = __dadd_rn(s2, __dmul_rn(x, x));
  }
  sum[q] = s;
  sumsq[q] = s2;
}

// ============================================================== truncated normal
// drawTruncNormal.m:53-86: inverse CDF, upper truncation at elb.
__device__ __forceinline__ double trunc_normal_dev(double mu, double sig, double elb, double u,
                                                   uint8_t* fl) {
  const double tol = 1e-10;
  const double eps = 2.220446049250313080847e-16;
  sig = fabs(sig);
  if (sig > tol) {
    const double ub = (elb - mu) / sig;
    const double PHIbar = 0.5 * erfc(-sqrt(0.5) * ub);
    double z;
    if (PHIbar > eps) {
      z = -sqrt(2.0) * erfcinv(2.0 * u * PHIbar);
      *fl = 3;
    } else {
      z = ub;
      *fl = 1;
    }
    return mu + sig * z;
  }
  *fl = 0;
  return mu;
}

__global__ void k_truncnorm(int n, const double* mu, const double* sig, double elb, const double* u,
                            double* out, uint8_t* flags) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  uint8_t f;
  out[q] = trunc_normal_dev(mu[q], sig[q], elb, u[q], &f);
  if (flags) flags[q] = f;
}

// ============================================================== diagnostics
// MFMA f64 layout self-test: D = A(16x4) * B(4x16) with the lane maps used above.
// normals of one chain's RNG block (CRN page or Philox), out[q] = normal(block, q): the
// host QR fallback of the coefficient block replays the chain's randn(K, N) (CTA.m:58)
__global__ void k_rng_normals(RngArgs ra, int c, int block, int n, double* __restrict__ out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const Rng rng = ra.make(c);
  out[q] = rng.normal(block, (uint32_t)q);
}

__global__ void k_mfma_selftest(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) + 16 * (l >> 4)], B[(l >> 4) + 4 * (l & 15)],
                                              acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) + 16 * (l & 15)] = acc[r];  // column-major 16x16
}

// D = C + A B with a caller-given accumulator: probes of the instruction's internal
// association and rounding (tools/probe_mfma_order.py, tests/test_gpu_mfma_order.py)
__global__ void k_mfma_selftest_acc(const double* A, const double* B, const double* C, double* D, int nprobe) {
  const int l = threadIdx.x;
  const size_t pr = blockIdx.x;
  if ((int)pr >= nprobe) return;
  A += pr * 64;
  B += pr * 64;
  C += pr * 256;
  D += pr * 256;
  dbl4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = C[((l >> 4) + 4 * r) + 16 * (l & 15)];
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) + 16 * (l >> 4)], B[(l >> 4) + 4 * (l & 15)], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) + 16 * (l & 15)] = acc[r];
}

// ---------------------------------------------------------------- instantiations launched by ccmm_abi.hip
template __global__ void k_resid_multi<8>(Dims, const int*, XSel, ChainState);
template __global__ void k_resid_multi<20>(Dims, const int*, XSel, ChainState);
template __global__ void k_resid_multi<32>(Dims, const int*, XSel, ChainState);
template __global__ void k_astep_w<20>(Dims, const int*, ChainState, RngArgs, double, int, const int*);
template __global__ void k_astep_w<32>(Dims, const int*, ChainState, RngArgs, double, int, const int*);

}  // namespace ccmm
