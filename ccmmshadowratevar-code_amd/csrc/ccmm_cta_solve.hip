// Sequential part of the triangular CTA draw (CTA.m:60-97 / CTAsys.m:62-108),
// one workgroup (4 waves) per chain, equations j = 1..N in order.
//
// Per equation:
//   v_t   = sum_{i>=j} A(i,j) [E_t A(i,:)'] / sqrtht(t,i)^2   (X_j'Y_j = X' v)      thread per t
//   rhs   = iVb_j + X' v                                     wave per column, 12 loads/lane in flight
//   L y = rhs ; L' x = y + z_j                               blocked: 64x64 diagonal block in LDS
//                                                            solved by wave 0 (readlane broadcasts),
//                                                            off-diagonal GEMV by all 4 waves
//   PAI(:,j) = x ; E(:,j) = Y(:,j) - X x                     thread per t
// L (lower) and L' (upper) both live in the system's KP x KP buffer written by
// k_chol; rdiag holds 1/L_kk.
#include "ccmm_sweep.h"

namespace ccmm {


template <int NMAX>
__global__ __launch_bounds__(256) void k_cta_solve2(Dims d, const int* __restrict__ Tslot,
                                                    const double* __restrict__ iVb, XSel xs,
                                                    ChainState cs, const double* __restrict__ rdiag,
                                                    RngArgs ra) {
  extern __shared__ double sm[];
  const int N = d.N, KP = d.KP, TP = d.TP, K = d.K;
  double* v = sm;                       // TP
  double* yv = v + TP;                  // KP
  double* rdl = yv + KP;                // KP
  double* Ls = rdl + KP;                // 64 x kSolveLd
  double* Al = Ls + 64 * kSolveLd;      // N x N (column-major A)
  double* Ael = Al + N * N;             // N x N Aelb (CTAsysAswitching), when cs.Aelb
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int T = Tslot[s];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Rng rng = ra.make(c);
  const double* sh = cs.sqrtht + (size_t)c * N * TP;
  const double* Y = xs.ypool + (size_t)xs.yidx[c] * N * TP;
  double* E = cs.E + (size_t)c * N * TP;
  for (int q = tid; q < N * N; q += 256) Al[q] = cs.A[(size_t)c * N * N + q];
  if (cs.Aelb)
    for (int q = tid; q < N * N; q += 256) Ael[q] = cs.Aelb[(size_t)c * N * N + q];
  __syncthreads();

  for (int j = 0; j < N; ++j) {
    const int mat = c * N + j;
    const double* X = xs.pool + (size_t)xs.idx[mat] * KP * TP;
    const double* L = cs.G + (size_t)mat * KP * KP;
    // ---- 1+2: E(:,j) = Y(:,j) (PAI(:,j) = 0, CTA.m:63), then v_t
    for (int t = tid; t < TP; t += 256) {
      double acc = 0.0;
      if (t < T) {
        double e[NMAX], ih[NMAX];
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
          if (k < N) {
            e[k] = (k == j) ? Y[(size_t)k * TP + t] : E[(size_t)k * TP + t];
            ih[k] = 1.0 / sh[(size_t)k * TP + t];
          }
        }
        E[(size_t)j * TP + t] = Y[(size_t)j * TP + t];
        const double* Am = (cs.atELB && cs.atELB[(size_t)c * TP + t]) ? Ael : Al;  // CTAsysAswitching.m:76-77
#pragma unroll
        for (int i = 0; i < NMAX; ++i) {
          if (i >= j && i < N) {
            double ea = 0.0;
#pragma unroll
            for (int k = 0; k <= i; ++k) ea = fma(e[k], Am[i + k * N], ea);
            acc += Am[i + j * N] * (ea * ih[i]) * ih[i];
          }
        }
      } else {
        E[(size_t)j * TP + t] = 0.0;
      }
      v[t] = acc;
    }
    for (int a = tid; a < KP; a += 256) rdl[a] = rdiag[(size_t)mat * KP + a];
    __syncthreads();
    // ---- 3: rhs = iVb_j + X' v   (wave per column)
    const double* ivb = iVb + ((size_t)s * N + j) * KP;
    for (int a = wave; a < KP; a += 4) {
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
    // ---- 4: forward substitution L y = rhs (blocked)
    for (int b = 0; b < nb; ++b) {
      const int r0 = b * 64;
      for (int e = tid; e < 64 * 64; e += 256) {
        const int i = e & 63, k = e >> 6;
        Ls[i * kSolveLd + k] = (k <= i) ? L[(size_t)(r0 + k) * KP + r0 + i] : 0.0;
      }
      __syncthreads();
      if (wave == 0) {
        double yi = yv[r0 + lane];
        const int kend = min(64, K - r0);
        for (int k = 0; k < kend; ++k) {
          const double yk = readlane_d(yi, k) * rdl[r0 + k];
          yi = (lane == k) ? yk : ((lane > k) ? fma(-Ls[lane * kSolveLd + k], yk, yi) : yi);
        }
        yv[r0 + lane] = yi;
      }
      __syncthreads();
      for (int r = r0 + 64 + tid; r < KP; r += 256) {
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
    // ---- 5: + z_j  (randn(K,N) of CTA.m:58, column j)
    for (int a = tid; a < K; a += 256) yv[a] += rng.normal(CCMM_RNG_PAI, (uint32_t)(a + K * j));
    __syncthreads();
    // ---- 6: back substitution L' x = y (blocked, upper storage U(r,k) = L(k,r))
    for (int b = nb - 1; b >= 0; --b) {
      const int r0 = b * 64;
      for (int e = tid; e < 64 * 64; e += 256) {
        const int i = e & 63, k = e >> 6;
        Ls[i * kSolveLd + k] = (k <= i) ? L[(size_t)(r0 + k) * KP + r0 + i] : 0.0;
      }
      __syncthreads();
      if (wave == 0) {
        double ci = yv[r0 + lane];
        const int kend = min(64, K - r0);
        for (int k = kend - 1; k >= 0; --k) {
          const double xk = readlane_d(ci, k) * rdl[r0 + k];
          ci = (lane == k) ? xk : ((lane < k) ? fma(-Ls[k * kSolveLd + lane], xk, ci) : ci);
        }
        if (lane < kend) yv[r0 + lane] = ci;
      }
      __syncthreads();
      for (int r = tid; r < r0; r += 256) {
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
    // ---- 7: PAI(:,j) = x ; E(:,j) = Y(:,j) - X x
    double* pai = cs.PAI + ((size_t)c * N + j) * KP;
    for (int a = tid; a < KP; a += 256) {
      const double val = (a < K) ? yv[a] : 0.0;
      pai[a] = val;
      yv[a] = val;
    }
    __syncthreads();
    for (int t = tid; t < T; t += 256) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      int a = 0;
      for (; a + 3 < K; a += 4) {
        a0 = fma(X[(size_t)a * TP + t], yv[a], a0);
        a1 = fma(X[(size_t)(a + 1) * TP + t], yv[a + 1], a1);
        a2 = fma(X[(size_t)(a + 2) * TP + t], yv[a + 2], a2);
        a3 = fma(X[(size_t)(a + 3) * TP + t], yv[a + 3], a3);
      }
      for (; a < K; ++a) a0 = fma(X[(size_t)a * TP + t], yv[a], a0);
      E[(size_t)j * TP + t] = Y[(size_t)j * TP + t] - ((a0 + a1) + (a2 + a3));
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- instantiations launched by ccmm_abi.hip
template __global__ void k_cta_solve2<8>(Dims, const int*, const double*, XSel, ChainState, const double*, RngArgs);
template __global__ void k_cta_solve2<20>(Dims, const int*, const double*, XSel, ChainState, const double*, RngArgs);
template __global__ void k_cta_solve2<32>(Dims, const int*, const double*, XSel, ChainState, const double*, RngArgs);

}  // namespace ccmm
