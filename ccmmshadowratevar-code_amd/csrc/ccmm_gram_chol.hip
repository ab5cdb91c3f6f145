// Fused weighted Gram + Cholesky of one CTA system per workgroup (CTA.m:69-78):
//
//   G = X' diag(w) X + diag(iV_j)      (SYRK on v_mfma_f64_16x16x4_f64)
//   L = chol(G)                        (right-looking, 16-wide panels, in registers)
//
// The lower triangle of G (16*NT <= 288, NT(NT+1)/2 tiles of 16 x 16; NT = 18 serves the hybrid
// model's K = 277 inside a KP = 320 system buffer, the rows past 16*NT staying zero) never
// leaves the register file: 8 waves, wave W owns tiles g = W + 8k of the
// column-major enumeration of the lower tiles, one dbl4 MFMA accumulator per tile
// (lane l holds G[ti*16 + (l>>4) + 4r][tj*16 + (l&15)], r = 0..3).  The body is
// specialised per wave (switch on the wave id), so every tile index is a
// compile-time constant and the MFMA operands are picked from a per-k-step
// array of 16 block fragments without runtime register indexing.
//
// SYRK: X rows are streamed in chunks of 16, scaled by sqrt(w_t) into an LDS
// panel Z (t x a); per 4-row k-step every wave reads the NT block fragments it
// needs (fragment b = Z[k][16b + l&15]) and issues its MFMAs back to back.
// Cholesky, for each 16-panel p:
//   (1) the owner of tile (p,p) hands it to LDS, wave 0 factors it (lane = row,
//       readlane broadcasts) and writes L_pp;
//   (2) owners of tiles (i,p), i > p, hand them to LDS; one thread per row
//       solves X L_pp' = G_ip;
//   (3) every wave updates its live tiles (i,j), p < j <= i: G_ij -= L_ip L_jp'
//       (MFMA, operands from the LDS panel; dead tiles in a live group of four
//       get a zero operand instead of a branch).
// Output, as k_chol: L (lower) and L' (upper) in the system's KP x KP buffer, 1/L_kk.
#include "ccmm_sweep.h"

namespace ccmm {


template <int NT, int W>
__device__ __forceinline__ int gram_chol_body(const GcArgs& g, double* sm, int tid) {
  constexpr int TPW = gc_tpw(NT);
  constexpr int NTILE = NT * (NT + 1) / 2;
  const int lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int KP = g.KP, TP = g.TP;

  dbl4 acc[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) acc[k] = dbl4{0.0, 0.0, 0.0, 0.0};

  // ------------------------------------------------------------ SYRK
  constexpr int LDZ = gc_ldz(NT);
  double* Z0 = sm;
  double* Z1 = sm + kGcTC * LDZ;
  constexpr int NLOAD = (kGcTC * 16 * NT + 511) / 512;
  const int nch = (g.mode & 1) ? 0 : (g.T + kGcTC - 1) / kGcTC;
  double vals[NLOAD];
  auto load_chunk = [&](int ch) {
    const int t0 = ch * kGcTC;
#pragma unroll
    for (int q = 0; q < NLOAD; ++q) {
      const int e = tid + 512 * q;
      const int t = e & 15, a = e >> 4;
      vals[q] = (a < 16 * NT) ? g.X[(size_t)a * TP + t0 + t] * g.w[t0 + t] : 0.0;
    }
  };
  auto store_chunk = [&](double* Z) {
#pragma unroll
    for (int q = 0; q < NLOAD; ++q) {
      const int e = tid + 512 * q;
      const int t = e & 15, a = e >> 4;
      if (a < 16 * NT) Z[t * LDZ + a] = vals[q];
    }
  };
  if (nch > 0) {
    load_chunk(0);
    store_chunk(Z0);
  }
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    double* Zc = (ch & 1) ? Z1 : Z0;
    double* Zn = (ch & 1) ? Z0 : Z1;
    const bool more = ch + 1 < nch;
    if (more) load_chunk(ch + 1);
#pragma unroll
    for (int kk = 0; kk < kGcTC / 4; ++kk) {
      const double* zr = Zc + (kk * 4 + lq) * LDZ + lr;
      double frag[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) frag[b] = zr[16 * b];
#pragma unroll
      for (int k = 0; k < TPW; ++k) {
        constexpr int dummy = 0;
        (void)dummy;
        if (W + kGcWaves * k < NTILE) {
          const int gi = W + kGcWaves * k;
          acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(frag[gc_ti(NT, gi)], frag[gc_tj(NT, gi)],
                                                        acc[k], 0, 0, 0);
        }
      }
    }
    if (more) store_chunk(Zn);
    __syncthreads();
  }
  // + diag(iV_j)
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int gi = W + kGcWaves * k;
    if (gi < NTILE && gc_ti(NT, gi) == gc_tj(NT, gi)) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (lq + 4 * r == lr) acc[k][r] += g.iv[gc_ti(NT, gi) * 16 + lr];
    }
  }

  // ------------------------------------------------------------ Cholesky
  double* Dg = sm;                // 16 x kGcLdp   L_pp
  double* Pn = sm + 16 * kGcLdp;  // NT slots of 16 x kGcLdp   L_ip
  int bad = 0;
  const int npanel = (g.mode & 2) ? 0 : NT;
  for (int p = 0; p < npanel; ++p) {
    // (1) diagonal tile -> LDS
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGcWaves * k;
      if (gi < NTILE && gc_ti(NT, gi) == p && gc_tj(NT, gi) == p) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Dg[(lq + 4 * r) * kGcLdp + lr] = acc[k][r];
      }
    }
    __syncthreads();
    if (W == 0 && !(g.mode & 16)) {
      double row[16];
      double mydiag = 1.0;
#pragma unroll
      for (int m = 0; m < 16; ++m) row[m] = (lane < 16 && m <= lane) ? Dg[lane * kGcLdp + m] : 0.0;
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
        const int i = p * 16 + lane;
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          const double v = (m <= lane) ? row[m] : 0.0;
          Dg[lane * kGcLdp + m] = v;
          if (m <= lane) {
            g.L[(size_t)(p * 16 + m) * KP + i] = v;  // L(i, 16p+m)
            g.L[(size_t)i * KP + p * 16 + m] = v;    // L' (upper)
          }
        }
        g.rd[i] = 1.0 / mydiag;
      }
    }
    // (2) panel tiles (i,p), i > p -> LDS
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int gi = W + kGcWaves * k;
      if (gi < NTILE && gc_tj(NT, gi) == p && gc_ti(NT, gi) > p) {
        double* P = Pn + gc_ti(NT, gi) * 16 * kGcLdp;
#pragma unroll
        for (int r = 0; r < 4; ++r) P[(lq + 4 * r) * kGcLdp + lr] = acc[k][r];
      }
    }
    __syncthreads();
    {
      const int nrows = (g.mode & 8) ? 0 : (NT - 1 - p) * 16;
      for (int e = tid; e < nrows; e += 512) {
        const int ti = p + 1 + (e >> 4), rr = e & 15;
        double* P = Pn + ti * 16 * kGcLdp + rr * kGcLdp;
        double x[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) x[m] = P[m];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          double sacc = x[m];
#pragma unroll
          for (int q = 0; q < m; ++q) sacc = fma(-x[q], Dg[m * kGcLdp + q], sacc);
          x[m] = sacc / Dg[m * kGcLdp + m];
        }
        const int i = ti * 16 + rr;
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          P[m] = x[m];
          g.L[(size_t)(p * 16 + m) * KP + i] = x[m];
          g.L[(size_t)i * KP + p * 16 + m] = x[m];
        }
      }
    }
    __syncthreads();
    // (3) trailing update, groups of 4 tiles
    if (p + 1 < NT && !(g.mode & 4)) {
#pragma unroll
      for (int g0 = 0; g0 < TPW; g0 += 4) {
        // live iff tj > p; tj is non-decreasing in k, so test the last slot of the group
        constexpr int dummy = 0;
        (void)dummy;
        int tjmax = -1;
#pragma unroll
        for (int k = g0; k < g0 + 4 && k < TPW; ++k)
          if (W + kGcWaves * k < NTILE) tjmax = gc_tj(NT, W + kGcWaves * k);
        if (tjmax > p) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            double pf[NT];
#pragma unroll
            for (int b = 0; b < NT; ++b)
              pf[b] = Pn[(b > p ? b : p + 1) * 16 * kGcLdp + lr * kGcLdp + lq + kk * 4];
#pragma unroll
            for (int k = g0; k < g0 + 4 && k < TPW; ++k) {
              const int gi = W + kGcWaves * k;
              if (gi < NTILE) {
                const bool live = gc_tj(NT, gi) > p;
                const double a = live ? -pf[gc_ti(NT, gi)] : 0.0;
                acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, pf[gc_tj(NT, gi)], acc[k], 0, 0, 0);
              }
            }
          }
        }
      }
    }
    __syncthreads();
  }
  return bad;
}

template <int NT>
__global__ __launch_bounds__(512, 1) void k_gram_chol(Dims d, const int* __restrict__ Tslot,
                                                      XSel xs, ChainState cs,
                                                      const double* __restrict__ iVdiag,
                                                      double* __restrict__ rdiag, int mode) {
  extern __shared__ double sm[];
  const int mat = blockIdx.x;
  const int c = mat / d.N, j = mat % d.N;
  const int s = cs.slot[c];
  GcArgs g;
  g.mode = mode;
  g.T = Tslot[s];
  g.TP = d.TP;
  g.KP = d.KP;
  g.X = xs.pool + (size_t)xs.idx[mat] * d.KP * d.TP;
  g.w = cs.W + (size_t)mat * d.TP;
  g.iv = iVdiag + ((size_t)s * d.N + j) * d.KP;
  g.L = cs.G + (size_t)mat * d.KP * d.KP;
  g.rd = rdiag + (size_t)mat * d.KP;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bad = 0;
  switch (wave) {
    case 0: bad = gram_chol_body<NT, 0>(g, sm, tid); break;
    case 1: bad = gram_chol_body<NT, 1>(g, sm, tid); break;
    case 2: bad = gram_chol_body<NT, 2>(g, sm, tid); break;
    case 3: bad = gram_chol_body<NT, 3>(g, sm, tid); break;
    case 4: bad = gram_chol_body<NT, 4>(g, sm, tid); break;
    case 5: bad = gram_chol_body<NT, 5>(g, sm, tid); break;
    case 6: bad = gram_chol_body<NT, 6>(g, sm, tid); break;
    case 7: bad = gram_chol_body<NT, 7>(g, sm, tid); break;
    default: __builtin_unreachable();
  }
  if (bad && (tid & 63) == 0) atomicOr(&cs.status[c], 2);
}

// ---------------------------------------------------------------- instantiations launched by ccmm_abi.hip
template __global__ void k_gram_chol<4>(Dims, const int*, XSel, ChainState, const double*, double*, int);
template __global__ void k_gram_chol<8>(Dims, const int*, XSel, ChainState, const double*, double*, int);
template __global__ void k_gram_chol<12>(Dims, const int*, XSel, ChainState, const double*, double*, int);
template __global__ void k_gram_chol<16>(Dims, const int*, XSel, ChainState, const double*, double*, int);

}  // namespace ccmm
