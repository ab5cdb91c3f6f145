// Per-vintage post-processing of the OOS driver on the device
// (goVARshadowrateBlockHybrid.m:349-480): for every series of kept draws (forecast paths
// per variable and horizon, their cumulated form, the shadow-rate paths, the VAR
// coefficients) the mean, the median, MATLAB prctile quantiles, std(., 1) and the CRPS of
// the empirical distribution at the realised value (crpsDraws).
//
//   gather   the series' draws from the chain set's stores into contiguous segments
//            (draw d = (chain, kept draw, forecast draw); cumsum over horizons for the
//            cumcode variables, :353-355)
//   sort     rocPRIM segmented radix sort of the segments (doubles, all 64 key bits)
//   stats    one workgroup per series on the sorted segment: order statistics give the
//            median and quantiles exactly; the sums (mean, variance, CRPS) are reduced in
//            a fixed order
//
// prctile: position vi = n q - 0.5 (0-based, q = pct / 100), clamped to [0, n - 1], linear
// interpolation as numpy's _lerp (method "hazen" = MATLAB's definition: the i-th sorted
// value sits at percentile 100 (i - 0.5) / n).
// CRPS (crpsDraws, em-matlabbox, source absent): mean|x - y| - 1/n^2 sum_i (2i - n - 1) x_(i).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "ccmm_post.h"

namespace ccmm {

namespace {

__device__ __forceinline__ double block_sum_256(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// numpy's _lerp with every operation rounded separately (the TU is built with
// -ffp-contract=off), so the quantiles are bit-identical to numpy.percentile(method="hazen")
__device__ __forceinline__ double lerp_np(double a, double b, double t) {
  const double d = b - a;
  return (t >= 0.5) ? b - d * (1.0 - t) : a + d * t;
}

// numpy's _compute_virtual_index: n q + (alpha + q (1 - alpha - beta)) - 1, alpha = beta = 0.5
__device__ __forceinline__ double hazen_index(int n, double pc) {
  const double q = pc / 100.0;
  return ((double)n * q + 0.5) - 1.0;
}

__global__ __launch_bounds__(256) void k_post_stats(int S, int n, const double* __restrict__ sorted,
                                                    const double* __restrict__ realized, int nq,
                                                    const double* __restrict__ pct, double* mean,
                                                    double* median, double* quant, size_t ldq, double* sd,
                                                    double* crps) {
  __shared__ double red[256];
  const int s = blockIdx.x;
  if (s >= S) return;
  const double* x = sorted + (size_t)s * n;
  const int tid = threadIdx.x;
  double a = 0.0;
  for (int i = tid; i < n; i += 256) a += x[i];
  const double mu = block_sum_256(a, red) / n;
  double v = 0.0;
  for (int i = tid; i < n; i += 256) {
    const double dlt = x[i] - mu;
    v = fma(dlt, dlt, v);
  }
  const double var = block_sum_256(v, red) / n;
  if (crps) {
    const double y = realized ? realized[s] : __builtin_nan("");
    double e = 0.0, g = 0.0;
    for (int i = tid; i < n; i += 256) {
      e += fabs(x[i] - y);
      g = fma(2.0 * (i + 1) - n - 1.0, x[i], g);
    }
    e = block_sum_256(e, red);
    g = block_sum_256(g, red);
    if (tid == 0) crps[s] = e / n - g / ((double)n * n);
  }
  if (tid == 0) {
    if (mean) mean[s] = mu;
    if (sd) sd[s] = sqrt(var);
  }
  auto pq = [&](double pc) {
    const double vi = hazen_index(n, pc);
    const double fl = floor(vi);
    int lo = (int)fl, hi = lo + 1;
    double gam = vi - fl;
    if (vi < 0.0) {
      lo = hi = 0;
      gam = 0.0;
    }
    if (lo >= n - 1) {
      lo = hi = n - 1;
      gam = 0.0;
    }
    return lerp_np(x[lo], x[hi], gam);
  };
  // median: the middle value, or the mean of the middle pair (MATLAB median, numpy median)
  if (median && tid == 0) median[s] = (n & 1) ? x[n / 2] : (x[n / 2 - 1] + x[n / 2]) / 2.0;
  if (quant)
    for (int q = tid; q < nq; q += 256) quant[(size_t)q * ldq + s] = pq(pct[q]);
}

// forecast paths: chain c's record of kept draw m, forecast draw job, horizon h, variable i
// at src[c * cap Nd H N + ((m Nd + job) H + h) N + i]; series s = r + nr h over the selected
// rows (rows[r], nr of them); draw d = (cc, m, job), job fastest.  Variables with flo[i] != 0
// are floored first, y(y < fl) = fl (mcmcVARshadowrate.m:642-645, 676-681: NaN stays NaN)
__global__ void k_gather_fcst(const double* __restrict__ src, int chain0, int C, int M, int Nd, int H,
                              int N, int cap, const int* __restrict__ rows, int nr,
                              const uint8_t* __restrict__ cum, const uint8_t* __restrict__ flo, double fl,
                              double* dst) {
  const int n = C * M * Nd;
  const int S = nr * H;
  const size_t total = (size_t)n * nr;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (size_t)gridDim.x * blockDim.x) {
    const int d = (int)(q % n), r = (int)(q / n);
    const int job = d % Nd, m = (d / Nd) % M, cc = d / (Nd * M);
    const int i = rows[r];
    const double* base = src + ((size_t)(chain0 + cc) * cap * Nd + (size_t)m * Nd + job) * H * N + i;
    const bool c = cum && cum[i];
    const bool f = flo && flo[i];
    double run = 0.0;
    for (int h = 0; h < H; ++h) {
      double val = base[(size_t)h * N];
      if (f && val < fl) val = fl;
      run = c ? run + val : val;
      dst[(size_t)(r + nr * h) * n + d] = run;
    }
    (void)S;
  }
}

// stored coefficient draws: chain c's kept draw m at src[(c cap + m) KN + e]; series e
__global__ void k_gather_pai(const double* __restrict__ src, int chain0, int C, int M, int cap, int KN,
                             double* dst) {
  const int n = C * M;
  const size_t total = (size_t)n * KN;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (size_t)gridDim.x * blockDim.x) {
    const int e = (int)(q % KN), d = (int)(q / KN);
    const int m = d % M, cc = d / M;
    dst[(size_t)e * n + d] = src[((size_t)(chain0 + cc) * cap + m) * KN + e];
  }
}

__global__ void k_offsets(int S, int n, int* off) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s <= S) off[s] = s * n;
}

#define PCHECK(x)                                              \
  do {                                                         \
    hipError_t e_ = (x);                                       \
    if (e_ != hipSuccess) return e_;                           \
  } while (0)

}  // namespace

// rocPRIM's segmented sort counts items in 32 bits: the series are sorted in batches of at most
// INT_MAX items (each batch's segment offsets s n fit an int)
static size_t series_per_sort(int S, int n) {
  return std::max<size_t>(1, std::min<size_t>((size_t)S, (size_t)INT_MAX / (size_t)n));
}

size_t post_workspace_bytes(int S, int n) {
  size_t tb = 0;
  if (S <= 0 || n <= 0) return 256;
  const size_t per = series_per_sort(S, n);
  (void)rocprim::segmented_radix_sort_keys((void*)nullptr, tb, (const double*)nullptr, (double*)nullptr,
                                           (unsigned int)(per * n), (unsigned int)per, (const int*)nullptr,
                                           (const int*)nullptr, 0, 64, (hipStream_t)0);
  return tb + (per + 1) * sizeof(int) + 256;
}

hipError_t post_summaries(hipStream_t st, int S, int n, const double* draws, double* sorted, void* ws,
                          size_t ws_bytes, const double* realized, int nq, const double* pct, double* mean,
                          double* median, double* quant, double* sd, double* crps) {
  if (S <= 0 || n <= 0) return hipSuccess;
  const size_t per = series_per_sort(S, n);
  int* off = (int*)ws;
  void* tmp = (char*)ws + (((per + 1) * sizeof(int) + 255) / 256) * 256;
  size_t tb = ws_bytes - ((char*)tmp - (char*)ws);
  auto at = [](double* p, size_t o) { return p ? p + o : nullptr; };
  for (size_t s0 = 0; s0 < (size_t)S; s0 += per) {
    const int Sc = (int)std::min(per, (size_t)S - s0);
    hipLaunchKernelGGL(k_offsets, dim3((Sc + 256) / 256), dim3(256), 0, st, Sc, n, off);
    PCHECK(hipGetLastError());
    PCHECK(rocprim::segmented_radix_sort_keys(tmp, tb, draws + s0 * n, sorted + s0 * n,
                                              (unsigned int)((size_t)Sc * n), (unsigned int)Sc, off, off + 1, 0, 64,
                                              st));
    hipLaunchKernelGGL(k_post_stats, dim3(Sc), dim3(256), 0, st, Sc, n, sorted + s0 * n,
                       realized ? realized + s0 : nullptr, nq, pct, at(mean, s0), at(median, s0), at(quant, s0),
                       (size_t)S, at(sd, s0), at(crps, s0));
    PCHECK(hipGetLastError());
  }
  return hipSuccess;
}

hipError_t post_gather_fcst(hipStream_t st, const double* src, int chain0, int C, int M, int Nd, int H, int N,
                            int cap, const int* rows, int nr, const uint8_t* cum, const uint8_t* flo, double fl,
                            double* dst) {
  const size_t total = (size_t)C * M * Nd * nr;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_gather_fcst, dim3(blocks), dim3(256), 0, st, src, chain0, C, M, Nd, H, N, cap, rows,
                     nr, cum, flo, fl, dst);
  return hipGetLastError();
}

hipError_t post_gather_pai(hipStream_t st, const double* src, int chain0, int C, int M, int cap, int KN,
                           double* dst) {
  const size_t total = (size_t)C * M * KN;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_gather_pai, dim3(blocks), dim3(256), 0, st, src, chain0, C, M, cap, KN, dst);
  return hipGetLastError();
}

}  // namespace ccmm
