// Generalized impulse responses by antithetic simulation (generateGIRF2linear.m,
// generateGIRF2blockhybrid.m:199-259, generateGIRF2hybrid.m:191-251, simVAR /
// simVARshadowrateBlockHybrid / simVARhybrid, antitheticSim):
// per MCMC draw, nsim shock paths x 4 antithetic shock sets x 3 scenarios (no shock,
// +shock11, -shock11 on variable 1 at horizon 1), each simulated over H horizons, averaged.
//
// The simulation is a batched GEMM per horizon: with the state of S = 16 simulations as
// the columns of X (rows: constant, p lags of y in a ring, p lags of the Ny actual rates in
// a ring (block hybrid), the horizon's structural shocks u), y_h = F X_h where the rows of
// F are the companion's y rows [PAIshadow' | PAIactual' | invA].  F is constant: each wave
// holds its 16-equation tile of F as v_mfma_f64_16x16x4f64 A-fragments in registers for
// the whole kernel; X lives in LDS and the ring shift is an index rotation.
//
//   grid (path chunks of 4, scenario, MCMC draw), 64 x ceil(N/16) threads
//   per horizon: SV step + shocks -> LDS | MFMA y = F X (4 accumulators) | ring update
//   (block hybrid: actual-rate states max(shadow, ELB)) | per-equation partial sums of
//   the 16 simulations (yields floored at the ELB) -> HBM
//   k_girf_reduce: sum the chunks in order, / (4 nsim), cumcode cumsum / np
#include "ccmm_girf.h"
#include "ccmm_internal.h"

namespace ccmm {

namespace {

constexpr int kGS = 16;  // simulations per workgroup: 4 paths x 4 antithetic shock sets

struct GirfDev {
  int M, N, p, H, nsim, bh, Ny, KX, KT, nchunk;
  int ldP;                // rows of PAI per equation: K (linear, block hybrid), K + Ny p (hybrid)
  const double* PAI;      // [M][N][ldP]
  const double* invA;     // [M][N][N]
  const double* sqrtPHI;  // [M][N][N] lower
  const double* SV0;      // [M][N]
  const double* Xj;       // [M][ldX] Xjumpoff (block hybrid: K + p Ny states)
  int ldX;
  const uint8_t* actual;  // [N] (block hybrid)
  const int* yidx;        // [Ny] ring variables (block hybrid: yields, hybrid: shadow rates)
  const uint8_t* yfloor;  // [N] floored at the ELB in the output (ndxYIELDS), bh != 0
  double elb, shock11;
  const double* z;        // [M][nsim][H][N] or nullptr (Philox)
  const double* svz;      // [M][nsim][H][N] or nullptr
  uint64_t seed;
  double* part;           // [M][3][nchunk][H][N]
};

// state row of companion coordinate k at ring head `head` (tabulated per head in LDS)
__device__ __forceinline__ int girf_row(int k, int head, const GirfDev& g) {
  const int Np = g.N * g.p;
  if (k == 0 || k >= g.KX) return k;
  if (k <= Np) {
    const int l = (k - 1) / g.N, j = k - 1 - l * g.N;
    int s = head - l;
    s += (s < 0) ? g.p : 0;
    return 1 + s * g.N + j;
  }
  const int q = k - 1 - Np, l = q / g.Ny, j = q - l * g.Ny;
  int s = head - l;
  s += (s < 0) ? g.p : 0;
  return 1 + Np + s * g.Ny + j;
}

template <int KS>
__global__ __launch_bounds__(128) void k_girf(GirfDev g) {
  extern __shared__ double sm[];
  const int chunk = blockIdx.x, scen = blockIdx.y, mm = blockIdx.z;
  const int N = g.N, p = g.p, H = g.H, K = 1 + N * p, Np = N * p;
  const int tid = threadIdx.x, lane = tid & 63, et = tid >> 6;
  const int nks = (g.KT + 3) / 4;
  double* X = sm;                            // [nks * 4][kGS]
  double* logsv = X + (size_t)nks * 4 * kGS; // [4][N]
  double* ybuf = logsv + 4 * N;              // [N][kGS]
  double* nrm = ybuf + N * kGS;              // [2][4][N]: svz, z of this horizon
  int* rowtab = (int*)(nrm + 8 * N);         // [p][nks * 4]: state row of coordinate k at head
  const int ldP = g.ldP;
  const double* PAI = g.PAI + (size_t)mm * N * ldP;
  const double* invA = g.invA + (size_t)mm * N * N;
  const double* sqP = g.sqrtPHI + (size_t)mm * N * N;
  const double* SV0 = g.SV0 + (size_t)mm * N;
  const double* Xj = g.Xj + (size_t)mm * g.ldX;
  const double s11 = scen == 0 ? 0.0 : (scen == 1 ? g.shock11 : -g.shock11);
  // F tile of this wave in registers: A[eq = 16 et + (lane & 15)][k = 4 ks + (lane >> 4)]
  double af[KS];
  {
    const int eq = 16 * et + (lane & 15);
    const bool act = g.bh == 1 && eq < N && g.actual[eq];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 4 * ks + (lane >> 4);
      double v = 0.0;
      if (eq < N && ks < nks) {
        if (k < K) {
          v = PAI[(size_t)eq * ldP + k];
          if (act && k > 0)
            for (int y = 0; y < g.Ny; ++y) v = (g.yidx[y] == (k - 1) % N) ? 0.0 : v;
        } else if (k < g.KX) {
          const int q = k - K, l = q / g.Ny, y = q - l * g.Ny;
          // hybrid (generateGIRF2hybrid.m:226-227): the PAI rows of the actual-rate lags;
          // block hybrid (generateGIRF2blockhybrid.m:226-234): PAIactual of the yield lags
          v = (g.bh == 2) ? PAI[(size_t)eq * ldP + K + q] : (act ? PAI[(size_t)eq * ldP + 1 + l * N + g.yidx[y]] : 0.0);
        } else if (k < g.KX + N) {
          v = invA[eq + (size_t)(k - g.KX) * N];
        }
      }
      af[ks] = v;
    }
  }
  // initial states (head = 0: lag l+1 in ring slot (-l) mod p), replicated over the 16 sims
  for (int q = tid; q < nks * 4 * kGS; q += blockDim.x) {
    const int r = q / kGS;
    double v = 0.0;
    if (r == 0) {
      v = Xj[0];
    } else if (r <= Np) {
      const int s = (r - 1) / N, j = r - 1 - s * N, l = (s == 0) ? 0 : p - s;
      v = Xj[1 + l * N + j];
    } else if (r < g.KX) {
      const int s = (r - 1 - Np) / g.Ny, j = r - 1 - Np - s * g.Ny, l = (s == 0) ? 0 : p - s;
      v = Xj[K + l * g.Ny + j];
    }
    X[q] = v;
  }
  for (int q = tid; q < 4 * N; q += blockDim.x) logsv[q] = 0.0;
  for (int q = tid; q < p * nks * 4; q += blockDim.x) rowtab[q] = girf_row(q % (nks * 4), q / (nks * 4), g);
  Rng rng;
  rng.crn = nullptr;
  rng.seed = g.seed;
  rng.chain = (uint32_t)mm;
  rng.sweep = 0;
  int head = 0;
  __syncthreads();
  for (int h = 0; h < H; ++h) {
    // (1) this horizon's normals of the 4 paths (one per thread), then the SV step and the
    //     shocks of the 16 sims (sim = 4 set + path)
    for (int q = tid; q < 4 * N; q += blockDim.x) {
      const int pl = q / N, i = q - pl * N;
      const int nn = chunk * 4 + pl;
      double zs = 0.0, zz = 0.0;
      if (nn < g.nsim) {
        const size_t base = ((size_t)nn * H + h) * N;
        zs = g.svz ? g.svz[(size_t)mm * g.nsim * H * N + base + i] : rng.normal(10, (uint32_t)(base + i));
        zz = g.z ? g.z[(size_t)mm * g.nsim * H * N + base + i] : rng.normal(9, (uint32_t)(base + i));
      }
      nrm[q] = zs;
      nrm[4 * N + q] = zz;
    }
    __syncthreads();
    for (int q = tid; q < 4 * N; q += blockDim.x) {
      const int pl = q / N, i = q - pl * N;
      const int nn = chunk * 4 + pl;
      double u[4] = {0.0, 0.0, 0.0, 0.0};
      if (nn < g.nsim) {
        double inc = 0.0;
        for (int j = 0; j <= i; ++j) inc = fma(sqP[i + (size_t)j * N], nrm[pl * N + j], inc);
        const double ls = logsv[q] + inc;
        logsv[q] = ls;
        const double sv = exp(ls * 0.5);
        const double zi = nrm[4 * N + q];
        const double a = zi * sv * SV0[i], b = zi / sv * SV0[i];
        const double add = (i == 0 && h == 0) ? s11 : 0.0;
        u[0] = a + add;
        u[1] = -a + add;
        u[2] = b + add;
        u[3] = -b + add;
      }
      for (int v = 0; v < 4; ++v) X[(size_t)(g.KX + i) * kGS + v * 4 + pl] = u[v];
    }
    __syncthreads();
    // (2) y = F X on MFMA (4 independent accumulation chains)
    dbl4 acc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) acc[a] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int* rt = rowtab + head * nks * 4 + (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks < nks) {
        const double b = X[rt[4 * ks] * kGS + (lane & 15)];
        acc[ks & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[ks], b, acc[ks & 3], 0, 0, 0);
      }
    }
    __syncthreads();
    // (3) ring update: slot head+1 takes y (and the actual rates max(y, ELB))
    const int nh = (head + 1 == p) ? 0 : head + 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int eq = 16 * et + (lane >> 4) + 4 * r, sim = lane & 15;
      const double y = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
      if (eq < N) {
        X[(size_t)(1 + nh * N + eq) * kGS + sim] = y;
        double yo = y;
        if (g.bh) {
          const double ya = y < g.elb ? g.elb : y;
          for (int q = 0; q < g.Ny; ++q)
            if (g.yidx[q] == eq) X[(size_t)(1 + Np + nh * g.Ny + q) * kGS + sim] = ya;
          if (g.yfloor[eq]) yo = ya;  // yields floored at the ELB in the output (:386-390)
        }
        ybuf[eq * kGS + sim] = yo;
      }
    }
    head = nh;
    __syncthreads();
    // (4) partial sums over the chunk's valid sims, fixed order
    if (tid < N) {
      double s = 0.0;
      for (int sim = 0; sim < kGS; ++sim)
        if (chunk * 4 + (sim & 3) < g.nsim) s += ybuf[tid * kGS + sim];
      g.part[((((size_t)mm * 3 + scen) * g.nchunk + chunk) * H + h) * N + tid] = s;
    }
  }
}

// Specialised form for compile-time p, N4 = ceil4(N), NY4 = ceil4(Ny): the state rows are laid
// out so that every 4-row k-step lies inside one lag block (blocks padded to N4 / NY4, the
// constant last), hence the B-operand row of k-step ks is (ring slot of its lag) * N4 + 4 kk
// + lq with ks -> (lag, kk) known at compile time: no table lookups, the LDS loads of the whole
// k-loop are independent of the MFMA results and can be issued ahead.
//   rows: [P x N4 lag ring][P x NY4 actual-rate ring][N4 shocks][4: constant 1, 0, 0, 0]
template <int P, int N4, int NY4>
__global__ __launch_bounds__(128) void k_girf_fast(GirfDev g) {
  constexpr int LAGR = P * N4, ACTR = P * NY4, SHR = LAGR + ACTR, CR = SHR + N4, KR = CR + 4;
  constexpr int KS = KR / 4;
  constexpr int NYD = NY4 > 0 ? NY4 : 1;  // divisor (the actual-rate branches are dead when NY4 = 0)
  extern __shared__ double sm[];
  const int chunk = blockIdx.x, scen = blockIdx.y, mm = blockIdx.z;
  const int N = g.N, H = g.H, K = 1 + N * P;
  const int tid = threadIdx.x, lane = tid & 63, et = tid >> 6, lq = lane >> 4;
  double* X = sm;                            // [KR][kGS]
  double* logsv = X + KR * kGS;              // [4][N]
  double* ybuf = logsv + 4 * N;              // [N][kGS]
  double* nrm = ybuf + N * kGS;              // [2][4][N]
  const int ldP = g.ldP;
  const double* PAI = g.PAI + (size_t)mm * N * ldP;
  const double* invA = g.invA + (size_t)mm * N * N;
  const double* sqP = g.sqrtPHI + (size_t)mm * N * N;
  const double* SV0 = g.SV0 + (size_t)mm * N;
  const double* Xj = g.Xj + (size_t)mm * g.ldX;
  const double s11 = scen == 0 ? 0.0 : (scen == 1 ? g.shock11 : -g.shock11);
  double af[KS];
  {
    const int eq = 16 * et + (lane & 15);
    const bool act = g.bh == 1 && eq < N && g.actual[eq];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 4 * ks + lq;
      double v = 0.0;
      if (eq < N) {
        if (k < LAGR) {
          const int l = k / N4, j = k - l * N4;
          if (j < N) {
            v = PAI[(size_t)eq * ldP + 1 + l * N + j];
            if (act)
              for (int y = 0; y < g.Ny; ++y) v = (g.yidx[y] == j) ? 0.0 : v;
          }
        } else if (k < SHR) {
          const int q = k - LAGR, l = q / NYD, jy = q - l * NYD;
          if (jy < g.Ny)
            v = (g.bh == 2) ? PAI[(size_t)eq * ldP + K + l * g.Ny + jy]
                            : (act ? PAI[(size_t)eq * ldP + 1 + l * N + g.yidx[jy]] : 0.0);
        } else if (k < CR) {
          if (k - SHR < N) v = invA[eq + (size_t)(k - SHR) * N];
        } else if (k == CR) {
          v = PAI[(size_t)eq * ldP];
        }
      }
      af[ks] = v;
    }
  }
  for (int q = tid; q < KR * kGS; q += blockDim.x) {
    const int r = q / kGS;
    double v = 0.0;
    if (r < LAGR) {
      const int s = r / N4, j = r - s * N4, l = (s == 0) ? 0 : P - s;
      if (j < N) v = Xj[1 + l * N + j];
    } else if (r < SHR) {
      const int s = (r - LAGR) / NYD, j = r - LAGR - s * NYD, l = (s == 0) ? 0 : P - s;
      if (j < g.Ny) v = Xj[K + l * g.Ny + j];
    } else if (r == CR) {
      v = Xj[0];
    }
    X[q] = v;
  }
  for (int q = tid; q < 4 * N; q += blockDim.x) logsv[q] = 0.0;
  Rng rng;
  rng.crn = nullptr;
  rng.seed = g.seed;
  rng.chain = (uint32_t)mm;
  rng.sweep = 0;
  int head = 0;
  __syncthreads();
  for (int h = 0; h < H; ++h) {
    for (int q = tid; q < 4 * N; q += blockDim.x) {
      const int pl = q / N, i = q - pl * N;
      const int nn = chunk * 4 + pl;
      double zs = 0.0, zz = 0.0;
      if (nn < g.nsim) {
        const size_t base = ((size_t)nn * H + h) * N;
        zs = g.svz ? g.svz[(size_t)mm * g.nsim * H * N + base + i] : rng.normal(10, (uint32_t)(base + i));
        zz = g.z ? g.z[(size_t)mm * g.nsim * H * N + base + i] : rng.normal(9, (uint32_t)(base + i));
      }
      nrm[q] = zs;
      nrm[4 * N + q] = zz;
    }
    __syncthreads();
    for (int q = tid; q < 4 * N; q += blockDim.x) {
      const int pl = q / N, i = q - pl * N;
      const int nn = chunk * 4 + pl;
      double u[4] = {0.0, 0.0, 0.0, 0.0};
      if (nn < g.nsim) {
        double inc = 0.0;
        for (int j = 0; j <= i; ++j) inc = fma(sqP[i + (size_t)j * N], nrm[pl * N + j], inc);
        const double ls = logsv[q] + inc;
        logsv[q] = ls;
        const double sv = exp(ls * 0.5);
        const double zi = nrm[4 * N + q];
        const double a = zi * sv * SV0[i], b = zi / sv * SV0[i];
        const double add = (i == 0 && h == 0) ? s11 : 0.0;
        u[0] = a + add;
        u[1] = -a + add;
        u[2] = b + add;
        u[3] = -b + add;
      }
      for (int v = 0; v < 4; ++v) X[(size_t)(SHR + i) * kGS + v * 4 + pl] = u[v];
    }
    __syncthreads();
    dbl4 acc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) acc[a] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int hd = __builtin_amdgcn_readfirstlane(head);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k0 = 4 * ks;
      int rb;
      if (k0 < LAGR) {
        const int l = k0 / N4;
        const int sl = (hd - l < 0) ? hd - l + P : hd - l;
        rb = sl * N4 + (k0 - l * N4);
      } else if (k0 < SHR) {
        const int l = (k0 - LAGR) / NYD;
        const int sl = (hd - l < 0) ? hd - l + P : hd - l;
        rb = LAGR + sl * NYD + (k0 - LAGR - l * NYD);
      } else {
        rb = k0;
      }
      const double b = X[(rb + lq) * kGS + (lane & 15)];
      acc[ks & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[ks], b, acc[ks & 3], 0, 0, 0);
    }
    __syncthreads();
    const int nh = (head + 1 == P) ? 0 : head + 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int eq = 16 * et + lq + 4 * r, sim = lane & 15;
      const double y = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
      if (eq < N) {
        X[(size_t)(nh * N4 + eq) * kGS + sim] = y;
        double yo = y;
        if (g.bh) {
          const double ya = y < g.elb ? g.elb : y;
          for (int q = 0; q < g.Ny; ++q)
            if (g.yidx[q] == eq) X[(size_t)(LAGR + nh * NYD + q) * kGS + sim] = ya;
          if (g.yfloor[eq]) yo = ya;
        }
        ybuf[eq * kGS + sim] = yo;
      }
    }
    head = nh;
    __syncthreads();
    if (tid < N) {
      double s = 0.0;
      for (int sim = 0; sim < kGS; ++sim)
        if (chunk * 4 + (sim & 3) < g.nsim) s += ybuf[tid * kGS + sim];
      g.part[((((size_t)mm * 3 + scen) * g.nchunk + chunk) * H + h) * N + tid] = s;
    }
  }
}

__global__ void k_girf_reduce(int M, int N, int H, int nchunk, int nsim, const double* __restrict__ part,
                              const uint8_t* __restrict__ cumcode, double np_, double* out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;  // (i, scen, mm)
  if (q >= N * 3 * M) return;
  const int i = q % N, sc = (q / N) % 3, mm = q / (3 * N);
  const double inv = 1.0 / (4.0 * nsim);
  double run = 0.0;
  for (int h = 0; h < H; ++h) {
    double s = 0.0;
    for (int c = 0; c < nchunk; ++c) s += part[((((size_t)mm * 3 + sc) * nchunk + c) * H + h) * N + i];
    double v = s * inv;
    if (cumcode && cumcode[i]) {
      run += v;
      v = run / np_;
    }
    out[(((size_t)mm * 3 + sc) * H + h) * N + i] = v;  // N x H x 3 x M
  }
}

}  // namespace

size_t girf_lds_bytes(int N, int p, int KT) {
  const int nks = (KT + 3) / 4;
  return ((size_t)nks * 4 * kGS + 12 * N + (size_t)N * kGS) * sizeof(double) + (size_t)p * nks * 4 * sizeof(int);
}

hipError_t girf_launch(hipStream_t st, const GirfArgs& a) {
  GirfDev g{};
  g.M = a.M; g.N = a.N; g.p = a.p; g.H = a.H; g.nsim = a.nsim; g.bh = a.bh; g.Ny = a.bh ? a.Ny : 0;
  const int K = 1 + a.N * a.p;
  g.KX = K + g.Ny * a.p;
  g.ldP = (a.bh == 2) ? g.KX : K;
  g.yfloor = a.yfloor;
  g.KT = g.KX + a.N;
  g.nchunk = (a.nsim + 3) / 4;
  g.PAI = a.PAI; g.invA = a.invA; g.sqrtPHI = a.sqrtPHI; g.SV0 = a.SV0; g.Xj = a.Xj; g.ldX = a.ldX;
  g.actual = a.actual; g.yidx = a.yidx; g.elb = a.elb; g.shock11 = a.shock11; g.z = a.z; g.svz = a.svz;
  g.seed = a.seed; g.part = a.part;
  const int nks = (g.KT + 3) / 4;
  const size_t lds = girf_lds_bytes(a.N, a.p, g.KT);
  const dim3 grid(g.nchunk, 3, a.M), block(64 * ((a.N + 15) / 16));
  auto go = [&](auto kern) -> hipError_t {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, grid, block, lds, st, g);
    return hipGetLastError();
  };
  hipError_t e;
  const int N4 = (a.N + 3) / 4 * 4, NY4 = (g.Ny + 3) / 4 * 4;
  const size_t lds_fast = ((size_t)(a.p * (N4 + NY4) + N4 + 4) * kGS + 12 * a.N + (size_t)a.N * kGS) * sizeof(double);
  auto go_fast = [&](auto kern) -> hipError_t {
    hipError_t e2 = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_fast);
    if (e2 != hipSuccess) return e2;
    hipLaunchKernelGGL(kern, grid, block, lds_fast, st, g);
    return hipGetLastError();
  };
  if (!a.force_generic && a.p == 12 && N4 == 20 && NY4 == 8) e = go_fast(k_girf_fast<12, 20, 8>);
  else if (!a.force_generic && a.p == 12 && N4 == 20 && NY4 == 4) e = go_fast(k_girf_fast<12, 20, 4>);
  else if (!a.force_generic && a.p == 12 && N4 == 20 && NY4 == 0) e = go_fast(k_girf_fast<12, 20, 0>);
  else if (nks <= 32) e = go(k_girf<32>);
  else if (nks <= 64) e = go(k_girf<64>);
  else if (nks <= 96) e = go(k_girf<96>);
  else return hipErrorInvalidValue;
  if (e != hipSuccess) return e;
  const int nt = a.N * 3 * a.M;
  hipLaunchKernelGGL(k_girf_reduce, dim3((nt + 255) / 256), dim3(256), 0, st, a.M, a.N, a.H, g.nchunk, a.nsim,
                     a.part, a.cumcode, a.np_, a.out);
  return hipGetLastError();
}

}  // namespace ccmm
