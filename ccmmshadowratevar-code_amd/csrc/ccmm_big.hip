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

#include <cstdlib>

namespace ccmm {

constexpr int kBT = 64;      // tile / block width
constexpr int kBC = 32;      // t rows per staged chunk of the Gram
constexpr int kBLd = 80;     // LDS row stride of staged panels (conflict-free b64 fragment reads)

// ============================================================== Gram (FP64 MFMA)
__global__ __launch_bounds__(256) void k_gram_big(Dims d, const int* __restrict__ Tslot, XSel xs,
                                                  ChainState cs, const int4* __restrict__ groups, ColX cx) {
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
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mymat = mats[wave];
  const int lcol = tid & 63, lt0 = (tid >> 6) * 8;
  // this thread's two staged columns a0 + lcol and b0 + lcol (X itself or its lag twin; the twin's
  // rows t >= T hold data where X holds zeros, but their weights are 0)
  const double *xa0, *xb0;
  if (cx.pool) {
    const double* D = cx.pool + (size_t)xs.idx[g.x] * cx.slab;
    xa0 = D + cx.off[a0 + lcol];
    xb0 = D + cx.off[b0 + lcol];
  } else {
    const double* X = xs.pool + (size_t)xs.idx[g.x] * d.KP * d.TP;
    xa0 = X + (size_t)(a0 + lcol) * d.TP;
    xb0 = X + (size_t)(b0 + lcol) * d.TP;
  }
  // 16 x 16 sub-tiles (x: b rows, y: a columns) that hold no lower-triangle entry of a real
  // coefficient -- the diagonal tile's upper half and the padded rows / columns >= K, whose X rows
  // are zero -- are not multiplied: they stay +0 (what the zero products sum to; the Cholesky and
  // the solve read only the lower triangle)
  unsigned need = 0;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
      if (b0 + 16 * x < d.K && a0 + 16 * y < d.K && !(ti == tj && y < x)) need |= 1u << (4 * x + y);
  need = __builtin_amdgcn_readfirstlane(need);
  dbl4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = dbl4{0.0, 0.0, 0.0, 0.0};
  const int nchunks = (T + kBC - 1) / kBC;
  // chunk ch + 1's panel rows and weights are loaded into registers while chunk ch multiplies
  double va[8], vb[8], wn = 0.0;
  auto load_chunk = [&](int t0) __attribute__((always_inline)) {
    const double* xa = xa0 + t0 + lt0;
    const double* xb = xb0 + t0 + lt0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      va[q] = xa[q];
      vb[q] = xb[q];
    }
    if (tid < 4 * kBC) {
      const int e = tid >> 5, t = tid & 31;
      wn = mats[e] >= 0 ? cs.W[(size_t)mats[e] * d.TP + t0 + t] : 0.0;
    }
  };
  load_chunk(0);
  for (int ch = 0; ch < nchunks; ++ch) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      Pa[lt0 + q][lcol] = va[q];
      Pb[lt0 + q][lcol] = vb[q];
    }
    if (tid < 4 * kBC) Wl[tid >> 5][tid & 31] = wn;
    __syncthreads();
    if (ch + 1 < nchunks) load_chunk((ch + 1) * kBC);
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
          if (need & (1u << (4 * x + y)))
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
// Update phase: each wave owns one 64-row block; its MFMA A fragments come straight from
// HBM into registers one 16-column chunk ahead of use, the shared L(kb, k) chunk is
// double-buffered in LDS (one barrier per chunk).  Factor phase: the LDS holds the
// diagonal block and its inverse instead (a union: 66.5 KB, two systems per CU).
constexpr int kCK = 8;  // k columns per pipelined chunk of the update
constexpr int kLiLd = 65;
__global__ __launch_bounds__(256, 2) void k_chol_big(Dims d, const int* __restrict__ slotIV,
                                                     const double* __restrict__ iVdiag, ChainState cs,
                                                     double* __restrict__ rdiag,
                                                     double* __restrict__ Dinv, int skip) {
  // skip: timing-only phase ablation (CCMM_CHOL_SKIP; results invalid): 1 update, 2 factor,
  // 4 panel; inside the factor phase 8 the 16 x 16 tile factor + inverse, 16 the inverse's
  // off-diagonal tiles, 32 the trailing tile updates
  __shared__ double smu[2 * kBT * kLiLd];  // update: Bs[2][kCK][kBLd]; factor: Lk | Li
  double* Lk = smu;                        // Lk[i * kLiLd + k] = L_kk(i, k)
  double* Li = smu + kBT * kLiLd;          // Li[j * kLiLd + k] = (L_kk^{-1})(j, k)
  const int mat = blockIdx.x;
  const int c = mat / d.N, j = mat % d.N;
  const int KP = d.KP;
  const int nb = KP / kBT;
  double* A = cs.G + (size_t)mat * KP * KP;
  const double* iv = iVdiag + ((size_t)slotIV[c] * d.N + j) * KP;
  double* rd = rdiag + (size_t)mat * KP;
  const int tid0 = threadIdx.x, wave = tid0 >> 6;
  for (int a = tid0; a < KP; a += 256) A[(size_t)a * KP + a] += iv[a];
  __syncthreads();
  int bad = 0;
  for (int kb = 0; kb < nb; ++kb) {
    // lane ids made opaque per block column: the fragment addresses derived from them are then
    // recomputed where used instead of ~100 of them being hoisted out of this loop and spilled
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, lr = lane & 15, lk = lane >> 4;
    const int kcol = kb * kBT;
    const int nch = kcol / kCK;
    // ---- 1. update of block column kb, four row blocks at a time (one per wave); block column 0
    //         has no update (its pass would store back the values it loaded)
    for (int ib0 = kb; ib0 < nb && kb > 0 && !(skip & 1); ib0 += 4) {
      const int ib = min(ib0 + wave, nb - 1);  // idle waves shadow the last block, store nothing
      const bool act = ib0 + wave < nb;
      const int irow = ib * kBT;
      dbl4 acc[4][4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[x][y][r] = -A[(size_t)(kcol + y * 16 + lr) * KP + irow + x * 16 + lk + 4 * r];  // -C: the
      // products add into the negated block (no negated copy of the A fragments), negated back on store
      if (nch > 0) {
        // the shared L(kb, k) chunk is double-buffered in LDS and each wave's own A fragments are
        // register double-buffered: chunk ch + 1's loads are in flight while chunk ch multiplies.
        // A wave without a row block (act false) stages its share of the chunk but multiplies
        // nothing, and the diagonal block's strictly upper 16 x 16 sub-tiles (never read) are
        // skipped: the SIMD's MFMA pipe goes to the co-resident system's waves instead.
        const bool diag = ib == kb;
        // 16-row sub-blocks wholly in the padding (rows >= K: zero data, identity prior, L rows
        // e_r) take no products: their update is by zero rows of L (the stored value is the same)
        const int xr = __builtin_amdgcn_readfirstlane(min(4, max(0, (d.K - irow + 15) / 16)));
        double bv[kCK * kBT / 256];
        auto load_b = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
          for (int q = 0; q < kCK * kBT / 256; ++q) {
            const int e = tid + 256 * q;
            bv[q] = A[(size_t)(k0 + (e >> 6)) * KP + kcol + (e & 63)];
          }
        };
        auto store_b = [&](double* Bn) __attribute__((always_inline)) {
#pragma unroll
          for (int q = 0; q < kCK * kBT / 256; ++q) {
            const int e = tid + 256 * q;
            Bn[(e >> 6) * kBLd + (e & 63)] = bv[q];
          }
        };
        double ac[kCK], an[kCK];
        auto load_a = [&](double (&dst)[kCK], int kc) __attribute__((always_inline)) {
          if (act) {
#pragma unroll
            for (int q = 0; q < kCK; ++q)
              dst[q] = A[(size_t)(kc + (q >> 2) * 4 + lk) * KP + irow + (q & 3) * 16 + lr];
          }
        };
        load_b(0);
        load_a(ac, 0);
        store_b(smu);
        __syncthreads();
        for (int ch = 0; ch < nch; ++ch) {
          const bool more = ch + 1 < nch;
          if (more) {
            load_b((ch + 1) * kCK);
            load_a(an, (ch + 1) * kCK);
          }
          if (act) {
            const double* Bs = smu + (ch & 1) * kCK * kBLd;
#pragma unroll
            for (int ks = 0; ks < kCK / 4; ++ks) {
              double fb[4];
#pragma unroll
              for (int y = 0; y < 4; ++y) fb[y] = Bs[(ks * 4 + lk) * kBLd + y * 16 + lr];
#pragma unroll
              for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y)
                  if (x < xr && !(diag && y > x))
                    acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[ks * 4 + x], fb[y], acc[x][y], 0, 0, 0);
            }
          }
          if (more) store_b(smu + ((ch + 1) & 1) * kCK * kBLd);
          __syncthreads();
#pragma unroll
          for (int q = 0; q < kCK; ++q) ac[q] = an[q];
        }
      }
      if (act) {
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              A[(size_t)(kcol + y * 16 + lr) * KP + irow + x * 16 + lk + 4 * r] = -acc[x][y][r];
      }
    }
    __syncthreads();
    // ---- 2. factor the diagonal block and invert it, as a 4 x 4 grid of 16 x 16 tiles:
    //         right-looking over tile columns q, the 16 x 16 tile (q, q) factored and inverted
    //         by wave 0 (lane = row, readlane broadcasts), the tiles below it scaled by
    //         L_qq^-T and the trailing tiles updated on MFMA by all waves; then the inverse's
    //         off-diagonal tiles Li_rq = -L_rr^-1 sum_k L_rk Li_kq by distance r - q on MFMA
    if (!(skip & 2)) {
      {  // the diagonal block's 16 entries per thread loaded before the first LDS store (one round trip)
        double lv[kBT * kBT / 256];
#pragma unroll
        for (int u = 0; u < kBT * kBT / 256; ++u) {
          const int e = tid + 256 * u, i = e & 63, k = e >> 6;
          lv[u] = (k <= i) ? A[(size_t)(kcol + k) * KP + kcol + i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kBT * kBT / 256; ++u) {
          const int e = tid + 256 * u, i = e & 63, k = e >> 6;
          Lk[i * kLiLd + k] = lv[u];
          Li[i * kLiLd + k] = 0.0;
        }
      }
      __syncthreads();
      for (int q = 0; q < 4; ++q) {
        if (wave == 0 && !(skip & 8)) {
          double* Tq = Lk + 16 * q * kLiLd + 16 * q;
          double row[16];
          double rdg = 1.0;  // 1 / L_ii of this lane's row
#pragma unroll
          for (int m = 0; m < 16; ++m) row[m] = (lane < 16 && m <= lane) ? Tq[lane * kLiLd + m] : 0.0;
#pragma unroll
          for (int kk = 0; kk < 16; ++kk) {
            double dkk = readlane_d(row[kk], kk);
            if (!(dkk > 0.0)) {
              bad = 1;
              dkk = 1.0;
            }
            // 1 / sqrt(d) by the deterministic iteration rsqrt_det (no IEEE sqrt / division on the
            // serial pivot chain, and reproducible off the device: oracle/cta_big_mirror.c);
            // L_kk = d / sqrt(d)
            const double rp = rsqrt_det(dkk);
            if (lane == kk) {
              row[kk] = dkk * rp;
              rdg = rp;
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
            for (int m = 0; m < 16; ++m) Tq[lane * kLiLd + m] = (m <= lane) ? row[m] : 0.0;
            rd[kcol + 16 * q + lane] = rdg;
          }
          // column c = lane of L_qq^-1 by forward substitution, L_im and 1 / L_ii read from
          // lane i's registers (no LDS round trip or division on the serial row chain)
          {
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
              x[i] = (i >= c) ? (s0 + s1) * readlane_d(rdg, i) : 0.0;
            }
            if (lane < 16) {
              double* Lq = Li + 16 * q * kLiLd + 16 * q;
#pragma unroll
              for (int i = 0; i < 16; ++i) Lq[i * kLiLd + c] = x[i];
            }
          }
        }
        __syncthreads();
        // tiles below: L_rq = A_rq L_qq^-T  (A operand A_rq(i, k), B operand Linv_qq(j, k))
        if (wave < 3 - q) {
          const int r = q + 1 + wave;
          dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const double a = Lk[(16 * r + lr) * kLiLd + 16 * q + 4 * kk + lk];
            const double b = Li[(16 * q + lr) * kLiLd + 16 * q + 4 * kk + lk];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
          }
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) Lk[(16 * r + lk + 4 * r4) * kLiLd + 16 * q + lr] = acc[r4];
        }
        __syncthreads();
        // trailing tiles A_rs -= L_rq L_sq'  (q < s <= r <= 3)
        if (q < 3 && !(skip & 32)) {
          int pr = 0;
          for (int r = q + 1; r < 4; ++r)
            for (int s2 = q + 1; s2 <= r; ++s2, ++pr) {
              if ((pr & 3) != wave) continue;
              dbl4 acc;
#pragma unroll
              for (int r4 = 0; r4 < 4; ++r4) acc[r4] = Lk[(16 * r + lk + 4 * r4) * kLiLd + 16 * s2 + lr];
#pragma unroll
              for (int kk = 0; kk < 4; ++kk) {
                const double a = Lk[(16 * r + lr) * kLiLd + 16 * q + 4 * kk + lk];
                const double b = Lk[(16 * s2 + lr) * kLiLd + 16 * q + 4 * kk + lk];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-a, b, acc, 0, 0, 0);
              }
#pragma unroll
              for (int r4 = 0; r4 < 4; ++r4) Lk[(16 * r + lk + 4 * r4) * kLiLd + 16 * s2 + lr] = acc[r4];
            }
          __syncthreads();
        }
      }
      // inverse tiles below the diagonal, by distance (each wave one tile per distance)
      for (int dist = 1; dist < 4 && !(skip & 16); ++dist) {
        if (wave < 4 - dist) {
          const int qq = wave, r = wave + dist;
          dbl4 sacc = dbl4{0.0, 0.0, 0.0, 0.0};  // S = sum_k L_rk Li_kq, k = q .. r - 1
          for (int kt = qq; kt < r; ++kt) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
              const double a = Lk[(16 * r + lr) * kLiLd + 16 * kt + 4 * kk + lk];
              const double b = Li[(16 * kt + 4 * kk + lk) * kLiLd + 16 * qq + lr];
              sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, sacc, 0, 0, 0);
            }
          }
          dbl4 x = dbl4{0.0, 0.0, 0.0, 0.0};  // -Linv_rr S: the accumulator is the B operand
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const double a = Li[(16 * r + lr) * kLiLd + 16 * r + 4 * kk + lk];
            x = __builtin_amdgcn_mfma_f64_16x16x4f64(-a, sacc[kk], x, 0, 0, 0);
          }
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) Li[(16 * r + lk + 4 * r4) * kLiLd + 16 * qq + lr] = x[r4];
        }
        __syncthreads();
      }
      for (int e = tid; e < kBT * kBT; e += 256) {
        const int i = e & 63, k = e >> 6;
        if (k <= i) A[(size_t)(kcol + k) * KP + kcol + i] = Lk[i * kLiLd + k];
      }
    }
    __syncthreads();
    // the diagonal block's inverse, row-major 64 x 64, for the solve's block substitutions
    {
      double* Dk = Dinv + ((size_t)mat * nb + kb) * kBT * kBT;
      for (int e = tid; e < kBT * kBT; e += 256) Dk[e] = Li[(e >> 6) * kLiLd + (e & 63)];
    }
    // ---- 3. panel below: L(r, kb) = C(r, kb) L_kk^{-T} on MFMA, 64-row tiles per wave;
    //         the tile's C fragments are loaded in four bursts of 16 per lane
    for (int rt = kb + 1 + wave; rt < nb && !(skip & 4); rt += 4) {
      const int r0 = rt * kBT;
      const int xr = __builtin_amdgcn_readfirstlane(min(4, max(0, (d.K - r0 + 15) / 16)));  // as in the update
      dbl4 acc[4][4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
      for (int half = 0; half < 4; ++half) {  // not unrolled: the later bursts' loads would be
        double fa[16];                        // hoisted and spill the accumulators
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int k = half * 16 + (q >> 2) * 4 + lk;
          fa[q] = A[(size_t)(kcol + k) * KP + r0 + (q & 3) * 16 + lr];
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int k = half * 16 + ks * 4 + lk;
          double fb[4];
#pragma unroll
          for (int y = 0; y < 4; ++y) fb[y] = Li[(y * 16 + lr) * kLiLd + k];
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y)
              if (x < xr) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[ks * 4 + x], fb[y], acc[x][y], 0, 0, 0);
        }
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            A[(size_t)(kcol + y * 16 + lr) * KP + r0 + x * 16 + lk + 4 * r] = acc[x][y][r];
    }
    __syncthreads();
  }
  if (bad && (tid0 & 63) == 0) atomicOr(&cs.status[c], 2);
}

// ============================================================== sequential solve (per chain)
// One workgroup of 16 waves per chain.  Every phase of an equation keeps many independent
// loads in flight per lane (the phases are latency- and bandwidth-bound through one CU):
//   v / U      thread per t, the i loop unrolled by 4
//   X' v       four columns per wave at a time, lanes over t, DPP wave sums
//   L y = r    64-row diagonal blocks by wave 0, the rows below by a thread each
//   L' x = y   left-looking: for block b the columns c of L below the block are contiguous,
//              so lanes run over their rows and a DPP sum gives (L' x)_c
//   X x        the K columns split in 8 slices x T in 64-row chunks, partial sums in LDS
constexpr int kBSLd = 65;
constexpr int kResSlices = 8;
// staged twin (KP <= kStageMaxKP): the X'v and residual phases read the lag twin from LDS, 256 months
// (plus the p - 1 presample rows their lags reach) at a time, instead of one L2 load per product
constexpr int kStageMonths = 256;
constexpr int kStageMaxKP = 320;
__host__ __device__ inline int big_stage_rows(int p) { return kStageMonths + p; }
__host__ inline size_t big_stage_lds_doubles(const Dims& d, const ColX& cx) {
  return (size_t)cx.ncol * big_stage_rows(d.p) + (d.KP + 1) / 2;  // + the KP int offsets
}
__global__ __launch_bounds__(1024) void k_cta_solve_big(Dims d, const int* __restrict__ Tslot,
                                                        const double* __restrict__ iVb, XSel xs,
                                                        ChainState cs, const double* __restrict__ rdiag,
                                                        RngArgs ra, double* __restrict__ Ubuf,
                                                        const double* __restrict__ Dinv, int skip, ColX cx) {
  // skip: timing-only phase ablation (CCMM_SOLVE_SKIP; results invalid): 1 v/U, 2 X'v,
  // 4 forward, 8 backward, 16 residual
  extern __shared__ double sm[];
  const int N = d.N, KP = d.KP, TP = d.TP, K = d.K;
  double* v = sm;                    // TP
  double* yv = v + TP;               // KP
  double* rdl = yv + KP;             // KP
  double* Ls = rdl + KP;             // 64 x kBSLd
  double* part = Ls + 64 * kBSLd;    // kResSlices x TP
  // staged twin: ncol x SR doubles, then the LDS offset of every design column
  const bool staged = cx.pool && cx.ncol > 0;
  const int SR = big_stage_rows(d.p);
  double* Ds = part + kResSlices * TP;
  int* loff = reinterpret_cast<int*>(Ds + (staged ? cx.ncol * SR : 0));
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int T = Tslot[s];
  const int tid0 = threadIdx.x;
  constexpr int NT = 1024, NW = 16;
  const Rng rng = ra.make(c);
  const double* Ac = cs.A + (size_t)c * N * N;
  const double* sh = cs.sqrtht + (size_t)c * N * TP;
  const double* Y = xs.ypool + (size_t)xs.yidx[c] * N * TP;
  double* E = cs.E + (size_t)c * N * TP;
  double* U = Ubuf + (size_t)c * N * TP;
  // U = E A' (E: residuals of the current PAI, k_resid)
  for (int q = tid0; q < N * TP; q += NT) {
    const int i = q / TP, t = q - i * TP;
    double u = 0.0;
    if (t < T)
      for (int k = 0; k <= i; ++k) u = fma(E[(size_t)k * TP + t], Ac[i + k * N], u);
    U[q] = u;
  }
  if (staged)
    for (int a = tid0; a < KP; a += NT) {
      const int o = cx.off[a], col = o / cx.ld;
      loff[a] = col * SR + (o - col * cx.ld);
    }
  __syncthreads();
  const int nb = (K + 63) / 64;
  // months [t0, t0 + 256) of the chain's twin -> Ds (rows t0 .. t0 + SR - 1 of every column); the
  // thread's loads are all issued before its LDS stores
  auto stage = [&](const double* Dg, int t0, int tid) __attribute__((always_inline)) {
    const int n = cx.ncol * SR;
    for (int e0 = tid; e0 < n; e0 += 8 * NT) {
      double val[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * NT, col = e / SR, r = e - col * SR;
        val[u] = (e < n && t0 + r < cx.ld) ? Dg[(size_t)col * cx.ld + t0 + r] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u * NT < n) Ds[e0 + u * NT] = val[u];
    }
  };
  for (int j = 0; j < N; ++j) {
    // per-equation opaque thread id: the lane-derived addresses of the phases below are formed
    // where they are used instead of being hoisted out of the equation loop (and spilled)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
    const int mat = c * N + j;
    // column a of the design: X + a TP, or its lag twin's column (same values for t < T; every
    // read below at t >= T is multiplied by v_t = 0 or not made)
    const double* X = cx.pool ? cx.pool + (size_t)xs.idx[mat] * cx.slab : xs.pool + (size_t)xs.idx[mat] * KP * TP;
    auto xcol = [&](int a) __attribute__((always_inline)) -> const double* {
      return cx.pool ? X + cx.off[a] : X + (size_t)a * TP;
    };
    const double* L = cs.G + (size_t)mat * KP * KP;
    // ---- E(:,j) = Y(:,j) (PAI(:,j) = 0, CTA.m:63); U(:,i) += dE A(i,j), i >= j; v_t
    for (int t = tid; t < TP && !(skip & 1); t += NT) {
      double acc = 0.0;
      if (t < T) {
        const double yj = Y[(size_t)j * TP + t];
        const double dl = yj - E[(size_t)j * TP + t];
        E[(size_t)j * TP + t] = yj;
        int i = j;
        for (; i + 7 < N; i += 8) {
          double u[8], h[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            u[q] = U[(size_t)(i + q) * TP + t];
            h[q] = sh[(size_t)(i + q) * TP + t];
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const double aij = Ac[i + q + j * N];
            u[q] = fma(dl, aij, u[q]);
            U[(size_t)(i + q) * TP + t] = u[q];
            acc += aij * (u[q] / h[q]) / h[q];
          }
        }
        for (; i < N; ++i) {
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
    // ---- rhs = iVb_j + X' v: four columns per wave at a time
    const double* ivb = iVb + ((size_t)s * N + j) * KP;
    if (staged && !(skip & 2)) {
      // the twin staged 256 months at a time; wave w keeps the sums of columns w*4 + 64 r + q (r < 5)
      // across the pieces, each lane adding its months t = lane + 64 u in increasing order: every
      // column's sum is formed in the order of the unstaged loop below
      double pr[kStageMaxKP / 64][4];
#pragma unroll
      for (int r = 0; r < kStageMaxKP / 64; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) pr[r][q] = 0.0;
      for (int t0 = 0; t0 < TP; t0 += kStageMonths) {
        __syncthreads();
        stage(X, t0, tid);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kStageMaxKP / 64; ++r) {
          const int a0 = wave * 4 + 64 * r;
          if (a0 < KP) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const double* col = Ds + loff[min(a0 + q, K - 1)] - t0;
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const int t = t0 + lane + 64 * u;
                if (t < TP) pr[r][q] = fma(col[t], v[t], pr[r][q]);
              }
            }
          }
        }
      }
#pragma unroll
      for (int r = 0; r < kStageMaxKP / 64; ++r) {
        const int a0 = wave * 4 + 64 * r;
        if (a0 < KP) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const double tot = wave_sum_dpp(a0 + q < K ? pr[r][q] : 0.0);
            if (lane == 0 && a0 + q < KP) yv[a0 + q] = ivb[a0 + q] + tot;
          }
        }
      }
    }
    for (int a0 = wave * 4; a0 < KP && !(skip & 2) && !staged; a0 += NW * 4) {
      double p[4] = {0.0, 0.0, 0.0, 0.0};
      const double* xc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) xc[q] = xcol(min(a0 + q, K - 1));
      int t = lane;
      for (; t + 64 * 3 < TP; t += 64 * 4) {  // 16 loads in flight per lane
        double xv[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q) xv[u][q] = xc[q][t + 64 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const double vt = v[t + 64 * u];
#pragma unroll
          for (int q = 0; q < 4; ++q) p[q] = fma(xv[u][q], vt, p[q]);
        }
      }
      for (; t < TP; t += 64) {
        const double vt = v[t];
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = fma(xc[q][t], vt, p[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double tot = wave_sum_dpp(a0 + q < K ? p[q] : 0.0);
        if (lane == 0 && a0 + q < KP) yv[a0 + q] = ivb[a0 + q] + tot;
      }
    }
    __syncthreads();
    // ---- forward substitution L y = rhs: per 64-row block y_b = Linv_bb (r_b) (the stored
    //      diagonal-block inverse, a 64 x 64 GEMV on wave 0), then the rows below
    //      r_r -= L(r, b) y_b (a thread per row, two bursts of 32 loads); the next block's
    //      inverse is prefetched into registers while the current one is applied
    const double* Dm = Dinv + (size_t)mat * nb * 4096;
    double dpre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dpre[q] = Dm[tid + NT * q];
    for (int b = 0; b < nb && !(skip & 4); ++b) {
      const int r0 = b * 64;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = tid + NT * q;
        Ls[(e >> 6) * kBSLd + (e & 63)] = dpre[q];
      }
      __syncthreads();
      if (b + 1 < nb)
#pragma unroll
        for (int q = 0; q < 4; ++q) dpre[q] = Dm[(size_t)(b + 1) * 4096 + tid + NT * q];
      if (wave == 0) {
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 16
        for (int k = 0; k < 64; ++k) a4[k & 3] = fma(Ls[lane * kBSLd + k], yv[r0 + k], a4[k & 3]);
        const double yi = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        wave_lds_sync();
        yv[r0 + lane] = yi;
      }
      __syncthreads();
      for (int r = r0 + 64 + tid; r < KP; r += NT) {
        double acc4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // two bursts of 32 loads in flight per thread
          double lv[32];
#pragma unroll
          for (int k = 0; k < 32; ++k) lv[k] = L[(size_t)(r0 + 32 * h + k) * KP + r];
#pragma unroll
          for (int k = 0; k < 32; ++k) acc4[k & 3] = fma(lv[k], yv[r0 + 32 * h + k], acc4[k & 3]);
        }
        yv[r] -= (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
      }
      __syncthreads();
    }
    // ---- + z_j (randn(K,N) of CTA.m:58, column j)
    for (int a = tid; a < K; a += NT) yv[a] += rng.normal(CCMM_RNG_PAI, (uint32_t)(a + K * j));
    __syncthreads();
    // ---- back substitution L' x = y, left-looking by 64-column blocks: (L' x)_c over the
    //      rows below the block (columns of L are contiguous), then x_b = Linv_bb' (y_b - s_b)
    if (!(skip & 8)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) dpre[q] = Dm[(size_t)(nb - 1) * 4096 + tid + NT * q];
    }
    for (int b = nb - 1; b >= 0 && !(skip & 8); --b) {
      const int r0 = b * 64;
      const int rb = r0 + 64;  // rows below the block: rb .. KP-1 (x there is final)
      {
        const int cq = wave * 4;
        double pq[4] = {0.0, 0.0, 0.0, 0.0};
        int r = rb + lane;
        for (; r + 64 * 3 < KP; r += 64 * 4) {  // 16 loads in flight per lane
          double lv[4][4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int q = 0; q < 4; ++q) lv[u][q] = L[(size_t)(r0 + cq + q) * KP + r + 64 * u];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const double xr = yv[r + 64 * u];
#pragma unroll
            for (int q = 0; q < 4; ++q) pq[q] = fma(lv[u][q], xr, pq[q]);
          }
        }
        for (; r < KP; r += 64) {
          const double xr = yv[r];
#pragma unroll
          for (int q = 0; q < 4; ++q) pq[q] = fma(L[(size_t)(r0 + cq + q) * KP + r], xr, pq[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double tot = wave_sum_dpp(pq[q]);
          if (lane == 0) part[cq + q] = tot;   // part is free until the residual phase
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = tid + NT * q;
        Ls[(e >> 6) * kBSLd + (e & 63)] = dpre[q];
      }
      __syncthreads();
      if (b > 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) dpre[q] = Dm[(size_t)(b - 1) * 4096 + tid + NT * q];
      if (wave == 0) {
        const double ri = yv[r0 + lane] - part[lane];
        part[64 + lane] = ri;
        wave_lds_sync();
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 16
        for (int k = 0; k < 64; ++k) a4[k & 3] = fma(Ls[k * kBSLd + lane], part[64 + k], a4[k & 3]);
        yv[r0 + lane] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
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
    if (staged && !(skip & 16)) {
      // the same items from the staged twin: each 256-month piece holds two chunk pairs, so the
      // piece's 16 items (8 slices x 2 pairs) are one per wave; each month's sum as below
      const int per = (K + kResSlices - 1) / kResSlices;
      for (int t0 = 0; t0 < TP; t0 += kStageMonths) {
        __syncthreads();
        stage(X, t0, tid);
        __syncthreads();
        const int slc = wave % kResSlices;
        const int t = t0 + (wave / kResSlices) * 128 + lane, t2 = t + 64;
        if (t < TP) {
          const int a_lo = slc * per, a_hi = min(K, a_lo + per);
          const int tc = max(min(t, T - 1) - t0, 0), tc2 = max(min(t2, T - 1) - t0, 0);  // unused when >= T
          double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
          double b0 = 0.0, b1 = 0.0, b2 = 0.0, b3 = 0.0;
          int a = a_lo;
          for (; a + 15 < a_hi; a += 16) {
            double xv[16], xw[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              const double* xc = Ds + loff[a + q];
              xv[q] = xc[tc];
              xw[q] = xc[tc2];
            }
#pragma unroll
            for (int q = 0; q < 16; q += 4) {
              a0 = fma(xv[q], yv[a + q], a0);
              a1 = fma(xv[q + 1], yv[a + q + 1], a1);
              a2 = fma(xv[q + 2], yv[a + q + 2], a2);
              a3 = fma(xv[q + 3], yv[a + q + 3], a3);
              b0 = fma(xw[q], yv[a + q], b0);
              b1 = fma(xw[q + 1], yv[a + q + 1], b1);
              b2 = fma(xw[q + 2], yv[a + q + 2], b2);
              b3 = fma(xw[q + 3], yv[a + q + 3], b3);
            }
          }
          for (; a < a_hi; ++a) {
            const double* xc = Ds + loff[a];
            a0 = fma(xc[tc], yv[a], a0);
            b0 = fma(xc[tc2], yv[a], b0);
          }
          part[slc * TP + t] = (t < T) ? (a0 + a1) + (a2 + a3) : 0.0;
          if (t2 < TP) part[slc * TP + t2] = (t2 < T) ? (b0 + b1) + (b2 + b3) : 0.0;
        }
      }
    } else {
      // items = (slice, pair of 64-month chunks): each lane forms the slice's sum for months t and
      // t + 64 with 32 loads in flight (the sum of each month in the same order as one month per item)
      const int nchunk = (T + 63) / 64, npair = (nchunk + 1) / 2;
      const int per = (K + kResSlices - 1) / kResSlices;
      for (int item = wave; item < npair * kResSlices && !(skip & 16); item += NW) {
        const int slc = item % kResSlices, tpr = item / kResSlices;
        const int t = tpr * 128 + lane, t2 = t + 64;
        const int a_lo = slc * per, a_hi = min(K, a_lo + per);
        const int tc = min(t, T - 1), tc2 = min(t2, T - 1);  // clamped reads; results of t >= T unused
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        double b0 = 0.0, b1 = 0.0, b2 = 0.0, b3 = 0.0;
        int a = a_lo;
        for (; a + 15 < a_hi; a += 16) {
          double xv[16], xw[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const double* xc = xcol(a + q);
            xv[q] = xc[tc];
            xw[q] = xc[tc2];
          }
#pragma unroll
          for (int q = 0; q < 16; q += 4) {
            a0 = fma(xv[q], yv[a + q], a0);
            a1 = fma(xv[q + 1], yv[a + q + 1], a1);
            a2 = fma(xv[q + 2], yv[a + q + 2], a2);
            a3 = fma(xv[q + 3], yv[a + q + 3], a3);
            b0 = fma(xw[q], yv[a + q], b0);
            b1 = fma(xw[q + 1], yv[a + q + 1], b1);
            b2 = fma(xw[q + 2], yv[a + q + 2], b2);
            b3 = fma(xw[q + 3], yv[a + q + 3], b3);
          }
        }
        for (; a < a_hi; ++a) {
          const double* xc = xcol(a);
          a0 = fma(xc[tc], yv[a], a0);
          b0 = fma(xc[tc2], yv[a], b0);
        }
        if (t < TP) part[slc * TP + t] = (t < T) ? (a0 + a1) + (a2 + a3) : 0.0;
        if (t2 < TP) part[slc * TP + t2] = (t2 < T) ? (b0 + b1) + (b2 + b3) : 0.0;
      }
    }
    __syncthreads();
    // E(:,j) and the rank-one update of U(:, i >= j), U's entries loaded eight at a time (one round
    // trip per eight instead of one per entry)
    for (int t = tid; t < T; t += NT) {
      double xp = 0.0;
#pragma unroll
      for (int q = 0; q < kResSlices; ++q) xp += part[q * TP + t];
      E[(size_t)j * TP + t] = Y[(size_t)j * TP + t] - xp;
      int i = j;
      for (; i + 7 < N; i += 8) {
        double u[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) u[q] = U[(size_t)(i + q) * TP + t];
#pragma unroll
        for (int q = 0; q < 8; ++q) U[(size_t)(i + q) * TP + t] = fma(-xp, Ac[i + q + j * N], u[q]);
      }
      for (; i < N; ++i) U[(size_t)i * TP + t] = fma(-xp, Ac[i + j * N], U[(size_t)i * TP + t]);
    }
    __syncthreads();
  }
}

// ============================================================== host launchers
size_t big_solve_lds_bytes(const Dims& d) {
  return (size_t)(d.TP + 2 * d.KP + 64 * kBSLd + kResSlices * d.TP) * sizeof(double);
}

hipError_t big_launch_cta(hipStream_t st, const Dims& d, const int* Tslot, const int* slotIV,
                          const double* iVdiag, const double* iVb, XSel xs, ChainState cs,
                          const int4* groups, int ngroups, double* rdiag, RngArgs ra, double* Ubuf,
                          double* Dinv, int phase_mask, ColX cx) {
  static const int skip = env_ablation("CCMM_SOLVE_SKIP", 0);
  static const int cskip = env_ablation("CCMM_CHOL_SKIP", 0);
  const int nt = d.KP / kBT;
  if (phase_mask & 1)
    hipLaunchKernelGGL(k_gram_big, dim3(nt * (nt + 1) / 2, ngroups), dim3(256), 0, st, d, Tslot, xs, cs,
                       groups, cx);
  if (phase_mask & 2)
    hipLaunchKernelGGL(k_chol_big, dim3(d.nmat), dim3(256), 0, st, d, slotIV, iVdiag, cs, rdiag, Dinv,
                       cskip);
  if (phase_mask & 4) {
    // the staged twin when the design fits kStageMaxKP and its LDS fits beside the rest
    ColX cs_x = cx;
    size_t lds = big_solve_lds_bytes(d);
    const size_t lds_st = lds + big_stage_lds_doubles(d, cx) * sizeof(double);
    if (!cx.pool || d.KP > kStageMaxKP || lds_st > 160 * 1024) cs_x.ncol = 0;
    else lds = lds_st;
    hipError_t e = hipFuncSetAttribute((const void*)k_cta_solve_big,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cta_solve_big, dim3(d.B), dim3(1024), lds, st, d, Tslot, iVb, xs, cs, rdiag,
                       ra, Ubuf, Dinv, skip, cs_x);
  }
  return hipGetLastError();
}

}  // namespace ccmm
