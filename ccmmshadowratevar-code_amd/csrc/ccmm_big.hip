// CTA / CTAsys coefficient block for large systems (CTA.m:57-98, CTAsys.m:57-108):
// K = N p + 1 up to 1536 (the S120 stress configuration N = 120, p = 12, K = 1441),
// N up to 128.  The K x K posterior precisions no longer fit a CU's LDS, so each one
// lives in HBM and the three phases are separate launches batched over all B N systems:
//
//   k_gram_big       G_cj = X' diag(w^(j)) X for the lower 64 x 64 tiles, FP64 MFMA.  One
//                    workgroup = one tile of FOUR systems that share the design X (the
//                    equations of a chain: CTA's X, or one CTAsys slab): the X panels are
//                    staged once in LDS and each wave applies its own equation's weights,
//                    so every loaded byte feeds 4 x 64 x 64 x 2 flops per t.
//   k_chol_big       one workgroup per system: left-looking blocked Cholesky with 64-wide
//                    block columns; the update L(ib,kb) -= sum_mb L(ib,mb) L(kb,mb)' runs on
//                    FP64 MFMA (one row block per wave, L(kb,mb) staged in LDS, L(ib,mb)
//                    in LDS per wave), the 64 x 64 diagonal block is factored by one wave
//                    (readlane broadcasts) and inverted, the panel below is L_kk^{-1}-scaled.
//   k_cta_solve_big  one workgroup (16 waves) per chain, equations in order: v, rhs = iVb +
//                    X'v, blocked forward / back substitution against L in HBM, residual
//                    update.  U = E A' is kept incrementally (rank-one updates of column j)
//                    instead of re-forming E_t A(i,:)' for every (t, i >= j).
#include "ccmm_big.h"

namespace ccmm {

constexpr int kBT = 64;      // tile / block width
constexpr int kBC = 32;      // t rows per staged chunk of the Gram
constexpr int kBLd = 80;     // LDS row stride of staged panels (conflict-free b64 fragment reads)

// ============================================================== Gram (FP64 MFMA)
__global__ __launch_bounds__(256) void k_gram_big(Dims d, const int* __restrict__ Tslot, XSel xs,
                                                  ChainState cs, const int4* __restrict__ groups) {
  __shared__ double Pa[kBC][kBLd];   // a-panel (t, a)
  __shared__ double Pb[kBC][kBLd];   // b-panel (t, b)
  __shared__ double Wl[4][kBC];      // weights of the group's four systems
  const int4 g = groups[blockIdx.y];
  const int mats[4] = {g.x, g.y, g.z, g.w};
  const int c = g.x / d.N;
  const int T = Tslot[cs.slot[c]];
  int tile = blockIdx.x, ti = 0;
  while (tile > ti) {
    tile -= ti + 1;
    ++ti;
  }
  const int tj = tile;
  const int a0 = ti * kBT, b0 = tj * kBT;
  const double* X = xs.pool + (size_t)xs.idx[g.x] * d.KP * d.TP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mymat = mats[wave];
  const int lcol = tid & 63, lt0 = (tid >> 6) * 8;
  dbl4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = dbl4{0.0, 0.0, 0.0, 0.0};
  const int nchunks = (T + kBC - 1) / kBC;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int t0 = ch * kBC;
    {
      const double* xa = X + (size_t)(a0 + lcol) * d.TP + t0 + lt0;
      const double* xb = X + (size_t)(b0 + lcol) * d.TP + t0 + lt0;
      double va[8], vb[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        va[q] = xa[q];
        vb[q] = xb[q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        Pa[lt0 + q][lcol] = va[q];
        Pb[lt0 + q][lcol] = vb[q];
      }
      if (tid < 4 * kBC) {
        const int e = tid >> 5, t = tid & 31;
        Wl[e][t] = mats[e] >= 0 ? cs.W[(size_t)mats[e] * d.TP + t0 + t] : 0.0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kBC / 4; ++kk) {
      const int kr = kk * 4 + (lane >> 4);
      const double wv = Wl[wave][kr];
      double fa[4], fb[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        fb[x] = Pb[kr][x * 16 + (lane & 15)];       // MFMA A operand: rows = b
        fa[x] = Pa[kr][x * 16 + (lane & 15)] * wv;  // MFMA B operand: cols = a (weighted)
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[x], fa[y], acc[x][y], 0, 0, 0);
    }
    __syncthreads();
  }
  if (mymat < 0) return;
  // D[row = b][col = a]: lane holds rows (lane >> 4) + 4 r of block x, column lane & 15 of block y
  double* G = cs.G + (size_t)mymat * d.KP * d.KP;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = b0 + x * 16 + (lane >> 4) + 4 * r;
        const int a = a0 + y * 16 + (lane & 15);
        G[(size_t)b * d.KP + a] = acc[x][y][r];
      }
}

// ============================================================== Cholesky (per system)
// In place on G_cj + diag(iV_j) (CTA.m:73-74): the lower triangle becomes L, rdiag = 1 / L_kk.
// LDS: Bs = L(kb, k0:k0+32) staged, As = L(ib_w, k0:k0+32) per wave; after the update the
// As region holds Li = L_kk^{-1} and Lk holds the factored diagonal block.
constexpr int kCK = 32;  // k columns per staged chunk of the update
constexpr int kLiLd = 65;
__global__ __launch_bounds__(256) void k_chol_big(Dims d, const int* __restrict__ slotIV,
                                                  const double* __restrict__ iVdiag, ChainState cs,
                                                  double* __restrict__ rdiag) {
  __shared__ double Bs[kCK][kBLd];       // Bs[k][j] = L(kb*64 + j, k0 + k)
  __shared__ double As[4][kCK][kBLd];    // As[w][k][i] = L(ib_w*64 + i, k0 + k)   (80 KB)
  __shared__ double Lk[kBT][kLiLd];      // Lk[i][k] = L_kk(i, k)
  double* Li = &As[0][0][0];             // Li[j * kLiLd + k] = (L_kk^{-1})(j, k)  (aliases As)
  const int mat = blockIdx.x;
  const int c = mat / d.N, j = mat % d.N;
  const int KP = d.KP;
  const int nb = KP / kBT;
  double* A = cs.G + (size_t)mat * KP * KP;
  const double* iv = iVdiag + ((size_t)slotIV[c] * d.N + j) * KP;
  double* rd = rdiag + (size_t)mat * KP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int a = tid; a < KP; a += 256) A[(size_t)a * KP + a] += iv[a];
  __syncthreads();
  int bad = 0;
  for (int kb = 0; kb < nb; ++kb) {
    const int kcol = kb * kBT;
    // ---- 1. update of block column kb, four row blocks at a time (one per wave)
    for (int ib0 = kb; ib0 < nb; ib0 += 4) {
      const int ib = ib0 + wave;
      const bool act = ib < nb;
      const int irow = ib * kBT;
      dbl4 acc[4][4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = irow + x * 16 + (lane >> 4) + 4 * r;
            const int jj = kcol + y * 16 + (lane & 15);
            acc[x][y][r] = act ? A[(size_t)jj * KP + i] : 0.0;
          }
      for (int k0 = 0; k0 < kcol; k0 += kCK) {
        for (int e = tid; e < kCK * kBT; e += 256) {
          const int k = e >> 6, r = e & 63;
          Bs[k][r] = A[(size_t)(k0 + k) * KP + kcol + r];
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int ibw = ib0 + w;
            As[w][k][r] = (ibw < nb) ? A[(size_t)(k0 + k) * KP + ibw * kBT + r] : 0.0;
          }
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < kCK / 4; ++ks) {
          const int k = ks * 4 + (lane >> 4);
          double fa[4], fb[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            fa[x] = -As[wave][k][x * 16 + (lane & 15)];  // MFMA A: row i, col k (negated)
            fb[x] = Bs[k][x * 16 + (lane & 15)];         // MFMA B: B[k][col j] = L(j, k)
          }
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y)
              acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[x], fb[y], acc[x][y], 0, 0, 0);
        }
        __syncthreads();
      }
      if (act) {
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = irow + x * 16 + (lane >> 4) + 4 * r;
              const int jj = kcol + y * 16 + (lane & 15);
              A[(size_t)jj * KP + i] = acc[x][y][r];
            }
      }
    }
    __syncthreads();
    // ---- 2. factor the diagonal block (wave 0, lane = row; readlane broadcasts)
    if (wave == 0) {
      double row[kBT];
      double mydiag = 1.0;
#pragma unroll
      for (int m = 0; m < kBT; ++m) row[m] = (m <= lane) ? A[(size_t)(kcol + m) * KP + kcol + lane] : 0.0;
#pragma unroll
      for (int kk = 0; kk < kBT; ++kk) {
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
        for (int m = kk + 1; m < kBT; ++m) {
          const double lmk = readlane_d(lik, m);
          if (lane >= m) row[m] = fma(-lik, lmk, row[m]);
        }
      }
#pragma unroll
      for (int m = 0; m < kBT; ++m) {
        const double v = (m <= lane) ? row[m] : 0.0;
        Lk[lane][m] = v;
        if (m <= lane) A[(size_t)(kcol + m) * KP + kcol + lane] = v;
      }
      rd[kcol + lane] = 1.0 / mydiag;
      // column `lane` of L_kk^{-1} by forward substitution, kept in LDS (no unrolled state)
      for (int i = 0; i < kBT; ++i) {
        double s = (i == lane) ? 1.0 : 0.0;
        for (int k = lane; k < i; ++k) s = fma(-Lk[i][k], Li[k * kLiLd + lane], s);
        Li[i * kLiLd + lane] = (i >= lane) ? s / Lk[i][i] : 0.0;
      }
    }
    __syncthreads();
    // ---- 3. panel below: L(r, kb) = C(r, kb) L_kk^{-T} on MFMA, 64-row tiles per wave
    for (int rt = kb + 1 + wave; rt < nb; rt += 4) {
      const int r0 = rt * kBT;
      dbl4 acc[4][4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
      for (int ks = 0; ks < kBT / 4; ++ks) {
        const int k = ks * 4 + (lane >> 4);
        double fa[4], fb[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          fa[x] = A[(size_t)(kcol + k) * KP + r0 + x * 16 + (lane & 15)];  // C(r, k)
          fb[x] = Li[(x * 16 + (lane & 15)) * kLiLd + k];                   // Linv(jj, k)
        }
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[x], fb[y], acc[x][y], 0, 0, 0);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = r0 + x * 16 + (lane >> 4) + 4 * r;
            const int jj = kcol + y * 16 + (lane & 15);
            A[(size_t)jj * KP + row] = acc[x][y][r];
          }
    }
    __syncthreads();
  }
  if (bad && lane == 0) atomicOr(&cs.status[c], 2);
}

// ============================================================== sequential solve (per chain)
constexpr int kBSLd = 65;
__global__ __launch_bounds__(1024) void k_cta_solve_big(Dims d, const int* __restrict__ Tslot,
                                                        const double* __restrict__ iVb, XSel xs,
                                                        ChainState cs, const double* __restrict__ rdiag,
                                                        RngArgs ra, double* __restrict__ Ubuf) {
  extern __shared__ double sm[];
  const int N = d.N, KP = d.KP, TP = d.TP, K = d.K;
  double* v = sm;                 // TP
  double* yv = v + TP;            // KP
  double* rdl = yv + KP;          // KP
  double* Ls = rdl + KP;          // 64 x kBSLd
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int T = Tslot[s];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NT = 1024, NW = 16;
  const Rng rng = ra.make(c);
  const double* Ac = cs.A + (size_t)c * N * N;
  const double* sh = cs.sqrtht + (size_t)c * N * TP;
  const double* Y = xs.ypool + (size_t)xs.yidx[c] * N * TP;
  double* E = cs.E + (size_t)c * N * TP;
  double* U = Ubuf + (size_t)c * N * TP;
  // U = E A' (E: residuals of the current PAI, k_resid)
  for (int q = tid; q < N * TP; q += NT) {
    const int i = q / TP, t = q - i * TP;
    double u = 0.0;
    if (t < T)
      for (int k = 0; k <= i; ++k) u = fma(E[(size_t)k * TP + t], Ac[i + k * N], u);
    U[q] = u;
  }
  __syncthreads();
  for (int j = 0; j < N; ++j) {
    const int mat = c * N + j;
    const double* X = xs.pool + (size_t)xs.idx[mat] * KP * TP;
    const double* L = cs.G + (size_t)mat * KP * KP;
    // ---- E(:,j) = Y(:,j) (PAI(:,j) = 0, CTA.m:63); U(:,i) += dE A(i,j), i >= j; v_t
    for (int t = tid; t < TP; t += NT) {
      double acc = 0.0;
      if (t < T) {
        const double yj = Y[(size_t)j * TP + t];
        const double dl = yj - E[(size_t)j * TP + t];
        E[(size_t)j * TP + t] = yj;
        for (int i = j; i < N; ++i) {
          const double aij = Ac[i + j * N];
          const double u = fma(dl, aij, U[(size_t)i * TP + t]);
          U[(size_t)i * TP + t] = u;
          const double hi = sh[(size_t)i * TP + t];
          acc += aij * (u / hi) / hi;
        }
      }
      v[t] = acc;
    }
    for (int a = tid; a < KP; a += NT) rdl[a] = rdiag[(size_t)mat * KP + a];
    __syncthreads();
    // ---- rhs = iVb_j + X' v (wave per column)
    const double* ivb = iVb + ((size_t)s * N + j) * KP;
    for (int a = wave; a < KP; a += NW) {
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
      if (a < K) {
        const double* xa = X + (size_t)a * TP;
        int t = lane;
        for (; t + 192 < TP; t += 256) {
          p0 = fma(xa[t], v[t], p0);
          p1 = fma(xa[t + 64], v[t + 64], p1);
          p2 = fma(xa[t + 128], v[t + 128], p2);
          p3 = fma(xa[t + 192], v[t + 192], p3);
        }
        for (; t < TP; t += 64) p0 = fma(xa[t], v[t], p0);
      }
      const double p = wave_sum((p0 + p1) + (p2 + p3));
      if (lane == 0) yv[a] = ivb[a] + p;
    }
    __syncthreads();
    const int nb = (K + 63) / 64;
    // ---- forward substitution L y = rhs (64 x 64 diagonal blocks by wave 0, GEMV by all)
    for (int b = 0; b < nb; ++b) {
      const int r0 = b * 64;
      for (int e = tid; e < 64 * 64; e += NT) {
        const int i = e & 63, k = e >> 6;
        Ls[i * kBSLd + k] = (k <= i) ? L[(size_t)(r0 + k) * KP + r0 + i] : 0.0;
      }
      __syncthreads();
      if (wave == 0) {
        double yi = yv[r0 + lane];
        const int kend = min(64, K - r0);
        for (int k = 0; k < kend; ++k) {
          const double yk = readlane_d(yi, k) * rdl[r0 + k];
          yi = (lane == k) ? yk : ((lane > k) ? fma(-Ls[lane * kBSLd + k], yk, yi) : yi);
        }
        yv[r0 + lane] = yi;
      }
      __syncthreads();
      for (int r = r0 + 64 + tid; r < KP; r += NT) {
        double a0 = 0.0, a1 = 0.0;
#pragma unroll 8
        for (int k = 0; k < 64; k += 2) {
          a0 = fma(L[(size_t)(r0 + k) * KP + r], yv[r0 + k], a0);
          a1 = fma(L[(size_t)(r0 + k + 1) * KP + r], yv[r0 + k + 1], a1);
        }
        yv[r] -= a0 + a1;
      }
      __syncthreads();
    }
    // ---- + z_j (randn(K,N) of CTA.m:58, column j)
    for (int a = tid; a < K; a += NT) yv[a] += rng.normal(CCMM_RNG_PAI, (uint32_t)(a + K * j));
    __syncthreads();
    // ---- back substitution L' x = y
    for (int b = nb - 1; b >= 0; --b) {
      const int r0 = b * 64;
      for (int e = tid; e < 64 * 64; e += NT) {
        const int i = e & 63, k = e >> 6;
        Ls[i * kBSLd + k] = (k <= i) ? L[(size_t)(r0 + k) * KP + r0 + i] : 0.0;
      }
      __syncthreads();
      if (wave == 0) {
        double ci = yv[r0 + lane];
        const int kend = min(64, K - r0);
        for (int k = kend - 1; k >= 0; --k) {
          const double xk = readlane_d(ci, k) * rdl[r0 + k];
          ci = (lane == k) ? xk : ((lane < k) ? fma(-Ls[k * kBSLd + lane], xk, ci) : ci);
        }
        if (lane < kend) yv[r0 + lane] = ci;
      }
      __syncthreads();
      // x(r) -= sum_k L(r0+k, r) x(r0+k) for r < r0: the rows of the transposed block are
      // columns r of L, k contiguous -> one wave per row r (coalesced over k)
      for (int r = wave; r < r0; r += NW) {
        const double p = wave_sum(L[(size_t)r * KP + r0 + lane] * yv[r0 + lane]);
        if (lane == 0) yv[r] -= p;
      }
      __syncthreads();
    }
    // ---- PAI(:,j) = x ; E(:,j) = Y(:,j) - X x ; U(:,i) += (E_new - Y_j) A(i,j), i >= j
    double* pai = cs.PAI + ((size_t)c * N + j) * KP;
    for (int a = tid; a < KP; a += NT) {
      const double val = (a < K) ? yv[a] : 0.0;
      pai[a] = val;
      yv[a] = val;
    }
    __syncthreads();
    for (int t = tid; t < T; t += NT) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      int a = 0;
      for (; a + 3 < K; a += 4) {
        a0 = fma(X[(size_t)a * TP + t], yv[a], a0);
        a1 = fma(X[(size_t)(a + 1) * TP + t], yv[a + 1], a1);
        a2 = fma(X[(size_t)(a + 2) * TP + t], yv[a + 2], a2);
        a3 = fma(X[(size_t)(a + 3) * TP + t], yv[a + 3], a3);
      }
      for (; a < K; ++a) a0 = fma(X[(size_t)a * TP + t], yv[a], a0);
      const double xp = (a0 + a1) + (a2 + a3);
      E[(size_t)j * TP + t] = Y[(size_t)j * TP + t] - xp;
      for (int i = j; i < N; ++i) U[(size_t)i * TP + t] = fma(-xp, Ac[i + j * N], U[(size_t)i * TP + t]);
    }
    __syncthreads();
  }
}

// ============================================================== host launchers
size_t big_solve_lds_bytes(const Dims& d) {
  return (size_t)(d.TP + 2 * d.KP + 64 * kBSLd) * sizeof(double);
}

hipError_t big_launch_cta(hipStream_t st, const Dims& d, const int* Tslot, const int* slotIV,
                          const double* iVdiag, const double* iVb, XSel xs, ChainState cs,
                          const int4* groups, int ngroups, double* rdiag, RngArgs ra, double* Ubuf,
                          int phase_mask) {
  const int nt = d.KP / kBT;
  if (phase_mask & 1)
    hipLaunchKernelGGL(k_gram_big, dim3(nt * (nt + 1) / 2, ngroups), dim3(256), 0, st, d, Tslot, xs, cs,
                       groups);
  if (phase_mask & 2)
    hipLaunchKernelGGL(k_chol_big, dim3(d.nmat), dim3(256), 0, st, d, slotIV, iVdiag, cs, rdiag);
  if (phase_mask & 4) {
    const size_t lds = big_solve_lds_bytes(d);
    hipError_t e = hipFuncSetAttribute((const void*)k_cta_solve_big,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cta_solve_big, dim3(d.B), dim3(1024), lds, st, d, Tslot, iVb, xs, cs, rdiag,
                       ra, Ubuf);
  }
  return hipGetLastError();
}

}  // namespace ccmm
