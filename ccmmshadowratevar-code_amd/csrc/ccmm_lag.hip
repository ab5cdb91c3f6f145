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
//       Linv = inv(L)               right-looking blocked inversion on MFMA (CTA.m:77
//                                   forms the same explicit inverse, Vchol = (L \ I)')
//     output per system (doubles): NTILE tiles of Linv~ (row-major 16 x 16, tile
//     g = column-major enumeration of the lower tiles), then [256]:
//       [0] = 1 / L00, [1 + a] = Linv(1 + a, 0) = -(Linv~ l)_a / L00
//
//   k_cta_solve_lag  per chain, equations j = 1..N in order (CTA.m:60-97):
//       v_t = sum_{i>=j} A(i,j) [E_t A(i,:)'] / sqrtht(t,i)^2        thread per t
//       rhs = iVb_j + X' v                                          D in LDS
//       PAI(:,j) = Linv' (Linv rhs + z_j)   (CTA.m:95-96: V rhs + Vc z with
//                                            V = Vc Vc', Vc = Linv')
//       E(:,j) = Y(:,j) - X PAI(:,j)                                D in LDS
//
// Padded lag columns (a >= Np) map to a spare zero column of D, so they carry zero
// data and the identity prior (iVdiag padding 1): exactly decoupled, x = 0 there.
#include "ccmm_lag.h"

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

// factor a 16 x 16 SPD tile held row-major (ld kGlLd) in LDS by one wave (lanes
// 0..15 = rows); writes L back (zero upper) and rd = 1 / diag(L)
__device__ __forceinline__ int gl_factor_tile(double* Dg, double* rd, int lane) {
  int bad = 0;
  double row[16];
  double mydiag = 1.0;
#pragma unroll
  for (int m = 0; m < 16; ++m) row[m] = (lane < 16 && m <= lane) ? Dg[lane * kGlLd + m] : 0.0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    double dkk = readlane_d(row[kk], kk);
    if (!(dkk > 0.0)) {
      bad = 1;
      dkk = 1.0;
    }
    const double piv = sqrt(dkk);
    const double rp = 1.0 / piv;
    if (lane == kk) {
      row[kk] = piv;
      mydiag = piv;
    }
    if (lane > kk) row[kk] *= rp;
    const double lik = row[kk];
#pragma unroll
    for (int m = kk + 1; m < 16; ++m) {
      const double lmk = readlane_d(lik, m);
      if (lane >= m) row[m] = fma(-lik, lmk, row[m]);
    }
  }
  if (lane < 16) {
#pragma unroll
    for (int m = 0; m < 16; ++m) Dg[lane * kGlLd + m] = (m <= lane) ? row[m] : 0.0;
    rd[lane] = 1.0 / mydiag;
  }
  return bad;
}

// in-place inverse of a lower-triangular 16 x 16 tile in LDS (row-major, ld kGlLd)
// by one wave: lane c < 16 solves L x = e_c (column c of the inverse)
__device__ __forceinline__ void gl_invert_tile(double* S, int lane) {
  double x[16];
  const int c = lane;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    double s = (i == c) ? 1.0 : 0.0;
#pragma unroll
    for (int m = 0; m < i; ++m) s = fma(-S[i * kGlLd + m], x[m], s);
    x[i] = (i >= c) ? s / S[i * kGlLd + i] : 0.0;
  }
  // all lanes have read S (in-order LDS within the wave) before the writes below
  __builtin_amdgcn_wave_barrier();
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) S[i * kGlLd + c] = x[i];
  }
  __builtin_amdgcn_wave_barrier();
}

template <int NT, int W>
__device__ __forceinline__ int gram_lag_body(const GlArgs& g, double* sm, int tid) {
  constexpr int NTILE = gl_ntile(NT);
  constexpr int TPW = gl_tpw(NT);
  constexpr int KL = 16 * NT;
  const int lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  int bad = 0;

  dbl4 acc[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) acc[k] = dbl4{0.0, 0.0, 0.0, 0.0};

  // ------------------------------------------------------------ SYRK of the lag columns
  int off[NT];
#pragma unroll
  for (int b = 0; b < NT; ++b) off[b] = g.colmap[16 * b + lr];
  double bs0 = 0.0, bs1 = 0.0, csum = 0.0;
  const int nks = (g.mode & 1) ? 0 : (g.T + 3) >> 2;
  for (int ks = 0; ks < nks; ++ks) {
    const int t = 4 * ks + lq;
    const double sw = g.swl[t];
    const double* row = g.Dl + t * g.ldd;
    double frag[NT];
#pragma unroll
    for (int b = 0; b < NT; ++b) frag[b] = row[off[b]] * sw;
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      constexpr int dummy = 0;
      (void)dummy;
      if (W + kGlWaves * k < NTILE) {
        const int gi = W + kGlWaves * k;
        acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(frag[gl_ti(NT, gi)], frag[gl_tj(NT, gi)], acc[k],
                                                      0, 0, 0);
      }
    }
    // intercept row b = X~' w: wave W accumulates lag tiles W and W + 8
    if (W < NT) bs0 = fma(frag[W < NT ? W : 0], sw, bs0);
    if (W + kGlWaves < NT) bs1 = fma(frag[W + kGlWaves < NT ? W + kGlWaves : 0], sw, bs1);
    csum = fma(sw, sw, csum);
  }
  bs0 += __shfl_xor(bs0, 16);
  bs0 += __shfl_xor(bs0, 32);
  bs1 += __shfl_xor(bs1, 16);
  bs1 += __shfl_xor(bs1, 32);
  csum += __shfl_xor(csum, 16);
  csum += __shfl_xor(csum, 32);
  __syncthreads();  // D no longer needed: the LDS is reused below

  double* lvec = sm;              // KL   b, then l = b / L00
  double* misc = lvec + KL;       // 8
  double* rdv = misc + 8;         // 2 x 16 (+ spare)
  double* Dg0 = rdv + 64;         // 2 tiles (double-buffered by panel parity)
  double* Pn0 = Dg0 + 2 * kGlTile;  // 2 x NT tiles
  double* Ws = Pn0 + 2 * NT * kGlTile + W * kGlTile;  // this wave's scratch tile
  double* part = Pn0 + 2 * NT * kGlTile + kGlWaves * kGlTile;  // NTILE x 16

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
  // + diag(iV~) - l l'
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int gi = W + kGlWaves * k;
    if (gi < NTILE) {
      const int ti = gl_ti(NT, gi), tj = gl_tj(NT, gi);
      const double lc = lvec[16 * tj + lr] * rL00;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rowi = 16 * ti + lq + 4 * r;
        double v = fma(-(lvec[rowi] * rL00), lc, acc[k][r]);
        if (ti == tj && lq + 4 * r == lr) v += g.iv[1 + rowi];
        acc[k][r] = v;
      }
    }
  }
  __syncthreads();
  if (tid < KL) lvec[tid] *= rL00;  // l
  __syncthreads();

  // ------------------------------------------------------------ Cholesky of M~
  for (int p = 0; p < ((g.mode & 2) ? 0 : NT); ++p) {
    double* Dg = Dg0 + (p & 1) * kGlTile;
    double* Pn = Pn0 + (p & 1) * NT * kGlTile;
    double* rd = rdv + (p & 1) * 16;
    // (1) column p -> LDS
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE && gl_tj(NT, gi) == p) {
        double* dst = (gl_ti(NT, gi) == p) ? Dg : Pn + gl_ti(NT, gi) * kGlTile;
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(lq + 4 * r) * kGlLd + lr] = acc[k][r];
      }
    }
    __syncthreads();
    // (2) diagonal tile
    if (W == 0 && !(g.mode & 256)) bad |= gl_factor_tile(Dg, rd, lane);
    __syncthreads();
    // (3) panel: L_ip = G_ip L_pp^-T, one thread per row
    {
      const int nrows = (g.mode & 512) ? 0 : (NT - 1 - p) * 16;
      for (int e = tid; e < nrows; e += 512) {
        const int ti = p + 1 + (e >> 4), rr = e & 15;
        double* P = Pn + ti * kGlTile + rr * kGlLd;
        double x[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) x[m] = P[m];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          double s = x[m];
#pragma unroll
          for (int q = 0; q < m; ++q) s = fma(-x[q], Dg[m * kGlLd + q], s);
          x[m] = s * rd[m];
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) P[m] = x[m];
      }
    }
    __syncthreads();
    // (4) column p back to registers; trailing update on MFMA
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE && gl_tj(NT, gi) == p) {
        const double* src = (gl_ti(NT, gi) == p) ? Dg : Pn + gl_ti(NT, gi) * kGlTile;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[k][r] = src[(lq + 4 * r) * kGlLd + lr];
      }
    }
    if (p + 1 < NT && !(g.mode & 1024)) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        double pf[NT];
#pragma unroll
        for (int b = 0; b < NT; ++b) pf[b] = (b > p) ? Pn[b * kGlTile + lr * kGlLd + lq + 4 * kk] : 0.0;
#pragma unroll
        for (int k = 0; k < TPW; ++k) {
          const int gi = W + kGlWaves * k;
          if (gi < NTILE && gl_tj(NT, gi) > p)
            acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(-pf[gl_ti(NT, gi)], pf[gl_tj(NT, gi)], acc[k], 0,
                                                          0, 0);
        }
      }
    }
  }

  __syncthreads();  // the last panel's Dg/Pn reads are done before the buffers are reused

  // ------------------------------------------------------------ inverse of L~
  // diagonal tiles in place: slot (p,p) := L_pp^-1
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int gi = W + kGlWaves * k;
    if (gi < NTILE && gl_ti(NT, gi) == gl_tj(NT, gi)) {
#pragma unroll
      for (int r = 0; r < 4; ++r) Ws[(lq + 4 * r) * kGlLd + lr] = acc[k][r];
      __builtin_amdgcn_wave_barrier();
      gl_invert_tile(Ws, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[k][r] = Ws[(lq + 4 * r) * kGlLd + lr];
      __builtin_amdgcn_wave_barrier();
    }
  }
  // right-looking solve of L X = I by tile rows: at step p
  //   X_pj = Linv_pp B_pj (j < p), X_pp = Linv_pp;   B_ij -= L_ip X_pj (i > p, j <= p)
  // slot (i, j) holds L_ij until step j, then B_ij, then (after step i) X_ij.
  for (int p = 0; p < ((g.mode & 4) ? 0 : NT); ++p) {
    double* XD = Dg0 + (p & 1) * kGlTile;          // Linv_pp
    double* LP = Pn0 + (p & 1) * NT * kGlTile;     // L_ip, i > p (slot i)
    double* XR = Pn0 + ((p + 1) & 1) * NT * kGlTile;  // X_pj, j <= p (slot j): other panel buffer
    // (1) Linv_pp and column p of L -> LDS
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE && gl_tj(NT, gi) == p) {
        double* dst = (gl_ti(NT, gi) == p) ? XD : LP + gl_ti(NT, gi) * kGlTile;
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(lq + 4 * r) * kGlLd + lr] = acc[k][r];
      }
    }
    __syncthreads();
    // (2) row p: X_pj = Linv_pp B_pj (j < p); X_pp -> XR as well
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE && gl_ti(NT, gi) == p) {
        const int tj = gl_tj(NT, gi);
        if (tj < p) {
          dbl4 cc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            cc = __builtin_amdgcn_mfma_f64_16x16x4f64(XD[lr * kGlLd + 4 * kk + lq], acc[k][kk], cc, 0, 0, 0);
          acc[k] = cc;
        }
        double* dst = XR + tj * kGlTile;
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(lq + 4 * r) * kGlLd + lr] = acc[k][r];
      }
    }
    __syncthreads();
    // (3) rows below: B_ij -= L_ip X_pj (j < p);  B_ip = -L_ip Linv_pp
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGlWaves * k;
      if (gi < NTILE && gl_ti(NT, gi) > p && gl_tj(NT, gi) <= p) {
        const int ti = gl_ti(NT, gi), tj = gl_tj(NT, gi);
        const double* La = LP + ti * kGlTile;
        const double* Xb = XR + tj * kGlTile;
        dbl4 cc = (tj == p) ? dbl4{0.0, 0.0, 0.0, 0.0} : acc[k];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          cc = __builtin_amdgcn_mfma_f64_16x16x4f64(-La[lr * kGlLd + 4 * kk + lq], Xb[(4 * kk + lq) * kGlLd + lr],
                                                    cc, 0, 0, 0);
        acc[k] = cc;
      }
    }
    // the next step writes the other XD/LP parity; XR of step p+1 is this LP buffer,
    // written only after the next step's first barrier
    __syncthreads();
  }

  // ------------------------------------------------------------ intercept column of Linv
  //   Linv(1+a, 0) = -(Linv~ l)_a / L00: per owned tile, row partial sums over its 16 columns
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int gi = W + kGlWaves * k;
    if (gi < NTILE) {
      const int tj = gl_tj(NT, gi);
      const double lc = lvec[16 * tj + lr];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double v = acc[k][r] * lc;
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if (lr == 0) part[gi * 16 + lq + 4 * r] = v;
      }
    }
  }
  __syncthreads();
  double* o = g.out;
  if (tid < KL) {
    const int ti = tid >> 4, rr = tid & 15;
    double s = 0.0;
    for (int tj = 0; tj <= ti; ++tj) s += part[gl_tile(NT, ti, tj) * 16 + rr];
    o[NTILE * 256 + 1 + tid] = -s * rL00;
  }
  if (tid == 0) o[NTILE * 256] = rL00;
  // ------------------------------------------------------------ Linv~ tiles -> HBM
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
  // D slab and sqrt weights -> LDS
  {
    const double* src = ls.dpool + (size_t)ls.idx[mat] * ls.rows * ls.ldd;
    const int n = ls.rows * ls.ldd;
    for (int q = tid; q < n; q += 512) sm[q] = src[q];
    double* swl = sm + n;
    const double* w = cs.W + (size_t)mat * TP;
    for (int t = tid; t < TP + 4; t += 512) swl[t] = (t < TP) ? w[t] : 0.0;
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
  int bad = 0;
  switch (wave) {
    case 0: bad = gram_lag_body<NT, 0>(g, sm, tid); break;
    case 1: bad = gram_lag_body<NT, 1>(g, sm, tid); break;
    case 2: bad = gram_lag_body<NT, 2>(g, sm, tid); break;
    case 3: bad = gram_lag_body<NT, 3>(g, sm, tid); break;
    case 4: bad = gram_lag_body<NT, 4>(g, sm, tid); break;
    case 5: bad = gram_lag_body<NT, 5>(g, sm, tid); break;
    case 6: bad = gram_lag_body<NT, 6>(g, sm, tid); break;
    case 7: bad = gram_lag_body<NT, 7>(g, sm, tid); break;
    default: __builtin_unreachable();
  }
  if (bad && (tid & 63) == 0) atomicOr(&cs.status[c], 2);
}

// ================================================================== sequential solve
template <int NT, int NMAX>
__global__ __launch_bounds__(kSlThreads) void k_cta_solve_lag(Dims d, const int* __restrict__ Tslot,
                                                              const double* __restrict__ iVb, XSel xs, LagSel ls,
                                                              ChainState cs, RngArgs ra) {
  constexpr int NTILE = gl_ntile(NT);
  constexpr int KL = 16 * NT;
  extern __shared__ double sm[];
  const int N = d.N, TP = d.TP, K = d.K, KP = d.KP;
  const int ldd = ls.ldd, rows = ls.rows;
  double* Dl = sm;
  double* vl = Dl + rows * ldd;      // TP            phases 1-2
  double* part = vl + TP;            // 2 x 256       phase 2
  double* tp = vl;                   // NTILE x 16    phases 3-4 (tile partials)
  double* rl = vl + sl_union(NT, TP);  // 256  rhs, then c = y + z  (K-space)
  double* xl = rl + 256;             // 256  y, then x            (K-space)
  double* Al = xl + 256;             // N x N
  double* red = Al + N * N;          // 16
  int* cm = reinterpret_cast<int*>(red + 16);  // KL
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int T = Tslot[s];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Rng rng = ra.make(c);
  const double* sh = cs.sqrtht + (size_t)c * N * TP;
  const double* Y = xs.ypool + (size_t)xs.yidx[c] * N * TP;
  double* E = cs.E + (size_t)c * N * TP;
  for (int q = tid; q < N * N; q += kSlThreads) Al[q] = cs.A[(size_t)c * N * N + q];
  for (int q = tid; q < KL; q += kSlThreads) cm[q] = ls.colmap[q];
  int cur = -1;

  for (int j = 0; j < N; ++j) {
    const int mat = c * N + j;
    const int slab = ls.idx[mat];
    const double* Lo = cs.G + (size_t)mat * KP * KP;
    const double* Lv = Lo + NTILE * 256;  // [0] 1/L00, [1+a] Linv(1+a,0)
    if (slab != cur) {
      __syncthreads();
      const double* src = ls.dpool + (size_t)slab * rows * ldd;
      for (int q = tid; q < rows * ldd; q += kSlThreads) Dl[q] = src[q];
      cur = slab;
    }
    // ---- (1) v_t (E(:,j) = Y(:,j) stands for PAI(:,j) = 0, CTA.m:63)
    for (int t = tid; t < TP; t += kSlThreads) {
      double acc = 0.0;
      if (t < T && !(ls.mode & 16)) {
        double e[NMAX], ih[NMAX];
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
          if (k < N) {
            e[k] = (k == j) ? Y[(size_t)k * TP + t] : E[(size_t)k * TP + t];
            ih[k] = 1.0 / sh[(size_t)k * TP + t];
          }
        }
#pragma unroll
        for (int i = 0; i < NMAX; ++i) {
          if (i >= j && i < N) {
            double ea = 0.0;
#pragma unroll
            for (int k = 0; k <= i; ++k) ea = fma(e[k], Al[i + k * N], ea);
            acc += Al[i + j * N] * (ea * ih[i]) * ih[i];
          }
        }
      }
      vl[t] = acc;
    }
    __syncthreads();
    // ---- (2) rhs = iVb_j + X' v, two t-halves per column
    {
      const int h = tid >> 8, a = tid & 255;
      const int th = ((T + 1) >> 1);
      const int t0 = h ? th : 0, t1 = h ? T : th;
      double p0 = 0.0, p1 = 0.0;
      if (ls.mode & 32) {
      } else if (a < KL) {
        const double* col = Dl + cm[a];
        int t = t0;
        for (; t + 1 < t1; t += 2) {
          p0 = fma(col[t * ldd], vl[t], p0);
          p1 = fma(col[(t + 1) * ldd], vl[t + 1], p1);
        }
        if (t < t1) p0 = fma(col[t * ldd], vl[t], p0);
      } else if (a == KL) {
        for (int t = t0; t < t1; ++t) p0 += vl[t];
      }
      part[h * 256 + a] = p0 + p1;
    }
    __syncthreads();
    const double* ivb = iVb + ((size_t)s * N + j) * KP;
    if (tid <= KL) {
      const int kx = (tid == KL) ? 0 : 1 + tid;
      rl[kx] = part[tid] + part[256 + tid] + ivb[kx];
    }
    __syncthreads();
    // ---- (3) y = Linv rhs: tile-row partials, one (tile, row) per thread pass
    for (int e = tid; e < ((ls.mode & 64) ? 0 : NTILE * 16); e += kSlThreads) {
      const int gi = e >> 4, rr = e & 15;
      const int ti = gl_ti(NT, gi), tj = gl_tj(NT, gi);
      const double* Lr = Lo + gi * 256 + rr * 16;
      const double* rv = rl + 1 + 16 * tj;
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int n = 0; n < 16; n += 2) {
        s0 = fma(Lr[n], rv[n], s0);
        s1 = fma(Lr[n + 1], rv[n + 1], s1);
      }
      tp[gi * 16 + rr] = s0 + s1;
      (void)ti;
    }
    __syncthreads();
    if (tid < KL) {
      const int ti = tid >> 4, rr = tid & 15;
      double sacc = Lv[1 + tid] * rl[0];
      for (int tj = 0; tj <= ti; ++tj) sacc += tp[gl_tile(NT, ti, tj) * 16 + rr];
      xl[1 + tid] = sacc;
    }
    if (tid == KL) xl[0] = rl[0] * Lv[0];
    __syncthreads();
    // ---- (4) c = y + z_j (randn(K,N) of CTA.m:58, column j); x = Linv' c
    if (tid <= KL) {
      const int kx = (tid == KL) ? 0 : 1 + tid;
      rl[kx] = xl[kx] + ((kx < K) ? rng.normal(CCMM_RNG_PAI, (uint32_t)(kx + K * j)) : 0.0);
    }
    __syncthreads();
    for (int e = tid; e < ((ls.mode & 64) ? 0 : NTILE * 16); e += kSlThreads) {
      const int gi = e >> 4, cc = e & 15;
      const int ti = gl_ti(NT, gi);
      const double* Lc = Lo + gi * 256 + cc;
      const double* cv = rl + 1 + 16 * ti;
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int n = 0; n < 16; n += 2) {
        s0 = fma(Lc[n * 16], cv[n], s0);
        s1 = fma(Lc[(n + 1) * 16], cv[n + 1], s1);
      }
      tp[gi * 16 + cc] = s0 + s1;
    }
    {  // x_0 = c_0 / L00 + sum_a Linv(1+a,0) c_{1+a}
      double pr = (tid < KL) ? Lv[1 + tid] * rl[1 + tid] : 0.0;
      pr = wave_sum(pr);
      if (lane == 0) red[wave] = pr;
    }
    __syncthreads();
    if (tid < KL) {
      const int tj = tid >> 4, cc = tid & 15;
      double sacc = 0.0;
      for (int ti = tj; ti < NT; ++ti) sacc += tp[gl_tile(NT, ti, tj) * 16 + cc];
      xl[1 + tid] = sacc;
    }
    if (tid == KL) {
      double sacc = rl[0] * Lv[0];
      for (int w = 0; w < kSlThreads / 64; ++w) sacc += red[w];
      xl[0] = sacc;
    }
    __syncthreads();
    // ---- (5) PAI(:,j) = x; E(:,j) = Y(:,j) - X x
    double* pai = cs.PAI + ((size_t)c * N + j) * KP;
    for (int k = tid; k < KP; k += kSlThreads) pai[k] = (k < K) ? xl[k] : 0.0;
    for (int t = tid; t < TP; t += kSlThreads) {
      double o = 0.0;
      if (t < T && !(ls.mode & 128)) {
        const double* rowp = Dl + t * ldd;
        double s0 = xl[0], s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int a = 0;
        for (; a + 3 < KL; a += 4) {
          s0 = fma(rowp[cm[a]], xl[1 + a], s0);
          s1 = fma(rowp[cm[a + 1]], xl[2 + a], s1);
          s2 = fma(rowp[cm[a + 2]], xl[3 + a], s2);
          s3 = fma(rowp[cm[a + 3]], xl[4 + a], s3);
        }
        for (; a < KL; ++a) s0 = fma(rowp[cm[a]], xl[1 + a], s0);
        o = Y[(size_t)j * TP + t] - ((s0 + s1) + (s2 + s3));
      }
      E[(size_t)j * TP + t] = o;
    }
    __syncthreads();
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

template <int NT, int NM>
static hipError_t solve_one(hipStream_t st, size_t lds, Dims d, const int* Tslot, const double* iVb, XSel xs,
                            LagSel ls, ChainState cs, RngArgs ra) {
  hipError_t e = hipFuncSetAttribute((const void*)k_cta_solve_lag<NT, NM>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_cta_solve_lag<NT, NM>), dim3(d.B), dim3(kSlThreads), lds, st, d, Tslot, iVb, xs, ls, cs,
                     ra);
  return hipGetLastError();
}

hipError_t lag_launch_solve(int NT, int nmax, hipStream_t st, size_t lds, Dims d, const int* Tslot,
                            const double* iVb, XSel xs, LagSel ls, ChainState cs, RngArgs ra) {
#define SL_CASE(NT_, NM_) \
  if (NT == NT_ && nmax == NM_) return solve_one<NT_, NM_>(st, lds, d, Tslot, iVb, xs, ls, cs, ra);
  SL_CASE(1, 8) SL_CASE(1, 20) SL_CASE(1, 32) SL_CASE(15, 8) SL_CASE(15, 20) SL_CASE(15, 32)
#undef SL_CASE
  return hipErrorInvalidValue;
}

}  // namespace ccmm
