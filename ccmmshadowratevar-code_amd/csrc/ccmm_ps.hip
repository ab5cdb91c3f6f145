// Acceptance-sampling branch of the ELB step (mcmcVARshadowrateBlockHybrid.m:438-466):
// Nproposals unconstrained draws of the censored shadow-rate cells from their joint
// Gaussian given the VAR (the em-matlabbox precision sampler VARTVPSVprecisionsamplerNaN,
// restated in oracle/ccmm_oracle_bh.precision_sampler_nan), the first proposal whose
// censored cells all lie below the ELB is accepted, else the Gibbs draw serves the sweep.
//
// The joint precision P of the n censored cells (month-major, variables in index order,
// the vec order of elb.yNaN) is block-banded: cells more than p months apart do not
// interact.  k_elb_cond already evaluates its blocks per censored month (the month's
// precision and the unit responses of the past neighbours) and, for the PS model, the
// linear term b (Yhatactual as an intercept, :423).  Then
//
//   k_ps_chol_w per chain, one wave (W <= 64): banded Cholesky P = L L' with the window rows in
//              registers (band storage L(i + j, i), j < W) and the forward solve ybar = L^-1 b;
//              k_ps_chol (W x W window in LDS) for wider bands
//   k_ps_prop  per (chain, 256 proposals): x_k = L'^-1 (ybar + z_k) by back substitution,
//              one proposal per thread with its last W values in registers (a shift
//              window, static indices), acceptance = all x < ELB (a
//              proposal stops at its first cell above the ELB), the smallest accepted index
//              by an LDS then a global atomic min
//   k_ps_apply per chain: recompute the accepted proposal into the chain's shadow rates
//              (k_elb_gibbs skips those chains), bookkeeping of :453-460
#include "ccmm_elb.h"

namespace ccmm {


// ---------------------------------------------------------------- banded Cholesky
// One thread per band row (64 threads, 128 for band widths above 64: Ns = 5 with p = 12)
__global__ __launch_bounds__(128) void k_ps_chol(Dims d, ElbDev e, PsDev ps, ChainState cs) {
  extern __shared__ double sm[];
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int lane = threadIdx.x, nth = blockDim.x;
  const int Ns = e.Ns, p = e.p, N = d.N, W = ps.W;
  const int nc = e.ncens[s];
  double* win = sm;                 // W x W: A(row, col) at [(row % W) W + col % W]
  double* lv = win + W * W;         // W: the current column of L
  double* bb = lv + W;              // W: forward-solve right-hand sides, slot i % W
  int* info = (int*)(bb + W);       // nmax: (censored-month index << 3) | variable
  __shared__ int sn;
  if (lane == 0) {
    int n = 0;
    for (int ci = 0; ci < nc; ++ci) {
      const int t = e.cens[(size_t)s * e.elbTmax + ci];
      for (int a = 0; a < Ns; ++a)
        if (e.sNaN[((size_t)s * e.elbTmax + t) * Ns + a]) info[n++] = (ci << 3) | a;
    }
    sn = n;
  }
  __syncthreads();
  const int n = sn;
  for (int i = lane; i < n; i += nth) {
    const int ci = info[i] >> 3, a = info[i] & 7;
    ps.cell[(size_t)c * ps.nmax + i] = e.cens[(size_t)s * e.elbTmax + ci] * Ns + a;
  }
  if (lane == 0) ps.n[c] = n;
  if (n == 0) return;
  const double* recs = e.cond + (size_t)c * e.elbTmax * e.condStride;
  const int xo = elb_cond_ps_off(Ns, p);
  // P(i, j), i >= j, from the month records (ccmm_elb.hip: P | b_PS | gP)
  auto pentry = [&](int i, int j) -> double {
    const int ci = info[i] >> 3, ai = info[i] & 7, cj = info[j] >> 3, aj = info[j] & 7;
    const int kp = e.cens[(size_t)s * e.elbTmax + ci] - e.cens[(size_t)s * e.elbTmax + cj];
    const double* x = recs + (size_t)ci * e.condStride + xo;
    if (kp == 0) return x[ai * Ns + aj];
    if (kp > p) return 0.0;
    return -x[Ns * Ns + Ns + ((kp - 1) * Ns + aj) * Ns + ai];
  };
  // b(i) = AA_m' (cc - AA_o y_o) of the censored cell: k_elb_cond's b_PS is the gradient at
  // censored cells = 0 with every observed cell (the month's uncensored shadow rates included)
  // at its value, so it is the whole linear term
  auto rhs = [&](int i) -> double {
    const int ci = info[i] >> 3, ai = info[i] & 7;
    return recs[(size_t)ci * e.condStride + xo + Ns * Ns + ai];
  };
  for (int q = lane; q < W * W; q += nth) {
    const int r = q / W, cc = q % W;
    win[q] = (cc <= r && r < n) ? pentry(r, cc) : 0.0;
  }
  if (lane < W) bb[lane] = lane < n ? rhs(lane) : 0.0;
  __syncthreads();
  double* Lg = ps.L + (size_t)c * ps.nmax * W;
  bool fail = false;
  for (int k = 0; k < n; ++k) {
    const int r = lane;
    const double v = (r < W && k + r < n) ? win[((k + r) % W) * W + k % W] : 0.0;
    const double dkk = win[(k % W) * W + k % W];  // row 0's v, read by every wave
    fail |= !(dkk > 0.0);
    const double lkk = sqrt(fabs(dkk) > 0.0 ? fabs(dkk) : 1.0);
    const double l = (r == 0) ? lkk : v / lkk;
    if (r < W) {
      Lg[(size_t)k * W + r] = l;
      lv[r] = l;
    }
    const double yk = bb[k % W] / lkk;
    if (r == 0) ps.ybar[(size_t)c * ps.nmax + k] = yk;
    __syncthreads();
    if (r >= 1 && r < W && k + r < n) {
      bb[(k + r) % W] -= l * yk;
      double* row = win + ((k + r) % W) * W;
      for (int cc = 1; cc <= r; ++cc) row[(k + cc) % W] -= l * lv[cc];
    }
    __syncthreads();
    // row k + W enters the window (its entries left of column k + 1 are outside the band)
    const int nr = k + W;
    if (nr < n) {
      if (r < W) win[(nr % W) * W + (nr - r) % W] = pentry(nr, nr - r);
      if (r == 0) bb[nr % W] = rhs(nr);
    }
    __syncthreads();
  }
  if (fail) {  // not positive definite: no proposals, the Gibbs draw serves the sweep
    if (lane == 0) {
      ps.n[c] = 0;
      atomicOr(&cs.status[c], CCMM_STATUS_PS_GIBBS);  // informational (k_phi sets bit 16 concurrently)
    }
  }
}

// ---------------------------------------------------------------- banded Cholesky, register window
// Band widths W <= 64 (the reference's Ns = 3 with p = 12: 39, padded to 48; S120's Ns = 4: 64).
// One wave per chain.  Lane q owns the window row i = q (mod W): its band entries sit in registers
// indexed by the column's distance to the pivot column k (reg[cc] = A(i, k + cc)), so every index
// is static.  A step broadcasts the pivot column L(k + r, k) through LDS once, every lane applies
// its row's rank-1 update and shifts its row one column left, and the lane whose row k just
// finished takes row k + W from an LDS chunk of assembled rows.  Entries right of a row's diagonal
// (cc > i - k) hold values no step reads.  Per column: one LDS write and W - 1 broadcast reads, two
// wave-scope syncs, against k_ps_chol's three workgroup barriers and a W x W read-modify-write of
// the window in LDS (and its serial assembly of the cell list).  Same band storage, same updates
// (fma(-L(i,k), L(j,k), A(i,j)) and bb -= L(i,k) yk) in the same order per entry.

template <int W>
__global__ __launch_bounds__(64) void k_ps_chol_w(Dims d, ElbDev e, PsDev ps, ChainState cs) {
  static_assert(W >= 2 && W <= 64, "one wave: W <= 64");
  extern __shared__ double sm[];
  double* prow = sm;                  // kPsChunk x W: P(i, i - W + 1 + cc) of row i at [(i - base) W + cc]
  double* pb = prow + kPsChunk * W;   // kPsChunk: b(i) of the chunk's rows
  double* sL = pb + kPsChunk;         // W: pivot column L(k + r, k) at [r]
  int* scens = (int*)(sL + W);        // elbTmax: month of censored month ci
  int* info = scens + e.elbTmax;      // nmax: (censored-month index << 3) | variable
  const int c = blockIdx.x;
  const int s = cs.slot[c];
  const int lane = threadIdx.x;
  const int Ns = e.Ns, p = e.p;
  const int nc = e.ncens[s];
  for (int ci = lane; ci < nc; ci += 64) scens[ci] = e.cens[(size_t)s * e.elbTmax + ci];
  __syncthreads();
  // cell list, month-major (variables in index order): per-month counts and a wave prefix sum
  int n = 0;
  for (int b0 = 0; b0 < nc; b0 += 64) {
    const int ci = b0 + lane;
    unsigned m = 0;
    if (ci < nc) {
      const uint8_t* f = e.sNaN + ((size_t)s * e.elbTmax + scens[ci]) * Ns;
      for (int a = 0; a < Ns; ++a) m |= f[a] ? (1u << a) : 0u;
    }
    const int cnt = __popc(m);
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    int off = n + incl - cnt;
    for (int a = 0; a < Ns; ++a)
      if ((m >> a) & 1u) info[off++] = (ci << 3) | a;
    n += __shfl(incl, 63, 64);
  }
  __syncthreads();
  for (int i = lane; i < n; i += 64) ps.cell[(size_t)c * ps.nmax + i] = scens[info[i] >> 3] * Ns + (info[i] & 7);
  if (lane == 0) ps.n[c] = n;
  if (n == 0) return;
  const double* recs = e.cond + (size_t)c * e.elbTmax * e.condStride;
  const int xo = elb_cond_ps_off(Ns, p);
  auto pentry = [&](int i, int j) -> double {  // P(i, j), i >= j (as k_ps_chol)
    const int ci = info[i] >> 3, ai = info[i] & 7, cj = info[j] >> 3, aj = info[j] & 7;
    const int kp = scens[ci] - scens[cj];
    const double* x = recs + (size_t)ci * e.condStride + xo;
    if (kp == 0) return x[ai * Ns + aj];
    if (kp > p) return 0.0;
    return -x[Ns * Ns + Ns + ((kp - 1) * Ns + aj) * Ns + ai];
  };
  auto fill = [&](int base) {  // band rows base .. base + kPsChunk - 1 and their b
    for (int q = lane; q < kPsChunk * W; q += 64) {
      const int i = base + q / W, cc = q % W, j = i - W + 1 + cc;
      prow[q] = (i < n && j >= 0) ? pentry(i, j) : 0.0;
    }
    const int i = base + lane;
    pb[lane] = i < n ? recs[(size_t)(info[i] >> 3) * e.condStride + xo + Ns * Ns + (info[i] & 7)] : 0.0;
  };
  int base = 0;
  fill(0);
  __syncthreads();
  double reg[W];
  double bbv = 0.0;
  // step 0: lane q < W holds row q (columns 0..q; 0 right of the diagonal and for rows >= n)
#pragma unroll
  for (int cc = 0; cc < W; ++cc)
    reg[cc] = (lane < W && cc <= lane) ? prow[lane * W + cc - lane + W - 1] : 0.0;
  if (lane < W) bbv = pb[lane];
  int r = lane < W ? lane : W;  // the lane's row relative to the pivot row (W: idle lane)
  double* Lg = ps.L + (size_t)c * ps.nmax * W;
  double* yb = ps.ybar + (size_t)c * ps.nmax;
  bool fail = false;
  int sk = 0;  // the pivot row's lane, k mod W
  for (int k = 0; k < n; ++k) {
    const double dkk = readlane_d(reg[0], sk);
    fail |= !(dkk > 0.0);
    const double lkk = sqrt(fabs(dkk) > 0.0 ? fabs(dkk) : 1.0);
    const double l = (r == 0) ? lkk : (r < W ? reg[0] / lkk : 0.0);
    const double yk = readlane_d(bbv, sk) / lkk;
    if (r < W) {
      Lg[(size_t)k * W + r] = l;
      sL[r] = l;
    }
    if (lane == sk) yb[k] = yk;
    wave_lds_sync();
#pragma unroll
    for (int cc = 1; cc < W; ++cc) reg[cc] = fma(-l, sL[cc], reg[cc]);
    bbv = fma(-l, yk, bbv);
#pragma unroll
    for (int cc = 0; cc < W - 1; ++cc) reg[cc] = reg[cc + 1];
    reg[W - 1] = 0.0;
    const int inew = k + W;  // enters on lane sk, whose row k is finished
    if (inew - base >= kPsChunk && inew < n) {
      base += kPsChunk;
      wave_lds_sync();
      fill(base);
    }
    wave_lds_sync();
    if (lane == sk) {
      if (inew < n) {
#pragma unroll
        for (int cc = 0; cc < W; ++cc) reg[cc] = prow[(inew - base) * W + cc];
        bbv = pb[inew - base];
      } else {
#pragma unroll
        for (int cc = 0; cc < W; ++cc) reg[cc] = 0.0;
        bbv = 0.0;
      }
    }
    r = (r == 0) ? W - 1 : (r < W ? r - 1 : W);
    sk = (sk + 1 == W) ? 0 : sk + 1;
  }
  if (fail && lane == 0) {  // not positive definite: no proposals, the Gibbs draw serves the sweep
    ps.n[c] = 0;
    atomicOr(&cs.status[c], CCMM_STATUS_PS_GIBBS);  // informational (k_phi sets bit 16 concurrently)
  }
}

// x = L'^-1 (ybar + z_k): one proposal by back substitution, the W - 1 values x_{i+1..i+W-1}
// in registers (win[j - 1] = x_{i + j}, shifted down one slot per step so every index is
// static).  The W - 1 products of a cell go to four interleaved accumulators (j mod 4), so the
// cell's dependent chain is W / 4 fused multiply-adds, not W - 1.  Lc: the chain's band factor.
// out != nullptr writes x into the chain's shadow
// rates.  Returns whether every cell lies below the ELB (a rejected proposal stops at its first cell
// at or above it unless out is set).
//
// Normals: with CRN, randn(nmiss, Nproposals) column-major (cell i of proposal k: i + n k).  With
// Philox, cell i of proposal k takes normal i + n2 k, n2 = n rounded up to even, so that every lane
// of a wave sees the same parity at the same cell and both values of a Box-Muller pair (normals
// 2P and 2P + 1: one log, one sqrt, one sincospi) serve two consecutive cells; the next pair is
// formed while the current pair's two cells are substituted (software-pipelined by one pair).
template <int W>
__device__ inline bool ps_backsub(const double* __restrict__ Lc, const double* __restrict__ yb, int n,
                                  const Rng& rng, int k, double elb, double* out, const int* cell,
                                  const double* zs = nullptr) {
  double win[W - 1];
#pragma unroll
  for (int j = 0; j < W - 1; ++j) win[j] = 0.0;
  bool ok = true;
  // one cell: returns false when the proposal is rejected and nothing more is needed
  auto step = [&](int i, double z) -> bool {
    const double* li = Lc + (size_t)i * W;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int j = 1; j < W; ++j) acc[j & 3] = fma(li[j], win[j - 1], acc[j & 3]);
    const double v = ((yb[i] + z) - ((acc[1] + acc[2]) + (acc[3] + acc[0]))) / li[0];
#pragma unroll
    for (int j = W - 2; j >= 1; --j) win[j] = win[j - 1];
    win[0] = v;
    ok = ok && (v < elb);
    if (out) {
      out[cell[i]] = v;
      return true;
    }
    return ok;  // rejected (a cell at or above the ELB): the rest of this proposal is never read
  };
  if (zs) {  // the proposal's normals, formed beforehand (ps_normals)
    for (int i = n - 1; i >= 0; --i)
      if (!step(i, zs[i])) break;
    return ok;
  }
  if (rng.crn) {
    for (int i = n - 1; i >= 0; --i)
      if (!step(i, rng.normal(CCMM_RNG_PS, (uint32_t)(i + n * k)))) break;
    return ok;
  }
  const uint32_t base = (uint32_t)((n + (n & 1)) * k);  // even: the cells' parities are wave-uniform
  auto pair = [&](uint32_t P, double& lo, double& hi) {  // normals 2P (cos) and 2P + 1 (sin)
    const u32x4 r = rng.raw(CCMM_RNG_PS, P);
    const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
    const double rad = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    lo = rad * cs;
    hi = rad * sn;
  };
  // cell i's normal index base + i; the top cell opens pair (base + n - 1) >> 1.  Pairs run two
  // ahead of the substitution: the pair of cells i - 4, i - 5 is formed while cells i, i - 1 are
  // substituted (a pair's log / sqrt / sincos outlasts two cells' substitution)
  int i = n - 1;
  uint32_t P = (base + (uint32_t)i) >> 1;
  double lo, hi, lo1 = 0.0, hi1 = 0.0;
  pair(P, lo, hi);
  if (i >= 1) pair(P - 1, lo1, hi1);
  if (((base + (uint32_t)i) & 1u) == 0u) {  // n odd: the top cell is the even half of its pair
    if (!step(i, lo)) return ok;
    --i;
    --P;
    lo = lo1;
    hi = hi1;
    if (i >= 3) pair(P - 1, lo1, hi1);
  }
  // now cell i is the odd half (hi) of pair P and cell i - 1 its even half (lo); pair P - 1 is in
  // (lo1, hi1) when cells i - 2, i - 3 exist
  while (i >= 0) {
    double lo2 = 0.0, hi2 = 0.0;
    if (i >= 5) pair(P - 2, lo2, hi2);
    if (!step(i, hi)) break;
    if (!step(i - 1, lo)) break;
    i -= 2;
    --P;
    lo = lo1;
    hi = hi1;
    lo1 = lo2;
    hi1 = hi2;
  }
  return ok;
}

// The normals of cell i and of cell i - 1 of proposal k, as ps_backsub takes them (i odd: the two
// halves of one Box-Muller pair under Philox), for a parallel fill: lanes take cells in pairs.
__device__ inline void ps_normal_pair(const Rng& rng, int n, int k, int i, double& zi, double& zim1) {
  if (rng.crn) {
    zi = rng.normal(CCMM_RNG_PS, (uint32_t)(i + n * k));
    zim1 = (i >= 1) ? rng.normal(CCMM_RNG_PS, (uint32_t)(i - 1 + n * k)) : 0.0;
    return;
  }
  const uint32_t idx = (uint32_t)((n + (n & 1)) * k) + (uint32_t)i;
  const u32x4 r = rng.raw(CCMM_RNG_PS, idx >> 1);
  const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
  const double rad = sqrt(-2.0 * log(u1));
  double sn, cs;
  sincospi(2.0 * u2, &sn, &cs);
  // idx odd: cell i is the pair's sin half and cell i - 1 its cos half; idx even (only the top cell
  // when n is odd): cell i is the cos half
  zi = (idx & 1u) ? rad * sn : rad * cs;
  zim1 = rad * cs;
}

// proposals k = blockIdx.x * 256 + threadIdx.x of chain blockIdx.y.  The band rows of L are read with
// wave-uniform addresses (scalar loads through the constant cache); staging L in LDS instead measured
// slower (0.34 -> 0.37 ms at B = 1: 48 vector LDS reads per cell against three scalar loads)
template <int W>
__global__ __launch_bounds__(256) void k_ps_prop(ElbDev e, PsDev ps, RngArgs ra) {
  const int c = blockIdx.y;
  const int n = ps.n[c];
  if (n == 0) return;
  const int k = blockIdx.x * 256 + threadIdx.x;
  __shared__ int kmin;
  if (threadIdx.x == 0) kmin = INT_MAX;
  __syncthreads();
  if (k < ps.NP) {
    const Rng rng = ra.make(c);
    // proposal 1 also lands in its censored cells of `first` (whose other cells hold the window's data)
    const bool keep = k == 0 && ps.first != nullptr;
    const bool ok = ps_backsub<W>(ps.L + (size_t)c * ps.nmax * W, ps.ybar + (size_t)c * ps.nmax, n, rng, k,
                                  ps.elb, keep ? ps.first + (size_t)c * ps.per : nullptr,
                                  keep ? ps.cell + (size_t)c * ps.nmax : nullptr);
    if (ok) atomicMin(&kmin, k);
  }
  __syncthreads();
  if (threadIdx.x == 0 && kmin != INT_MAX) atomicMin(ps.acc + c, kmin);
}

// One wave per chain: the accepted proposal's normals are formed by all lanes (Box-Muller pairs in
// parallel) into LDS, then lane 0 substitutes it into the chain's shadow rates (the serial chain
// then waits on the substitution only, not on a log / sqrt / sincos per two cells)
template <int W>
__global__ __launch_bounds__(64) void k_ps_apply(ElbDev e, PsDev ps, RngArgs ra, int kept) {
  extern __shared__ double zl[];  // [nmax]
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = ps.n[c];
  const int kmin = ps.acc[c];
  if (n == 0 || kmin == INT_MAX) {
    if (lane == 0) {
      ps.acc[c] = INT_MAX;
      if (n == 0 && ps.first)  // no proposals this sweep (precision not positive definite)
        for (int q = 0; q < ps.per; ++q) ps.first[(size_t)c * ps.per + q] = __builtin_nan("");
      ps.flag[c] = 0;
      if (ps.state) __hip_atomic_store(&ps.state[c], ps.epoch << 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const Rng rng = ra.make(c);
  // cells in pairs from the top: (n - 1, n - 2), ... (n odd under Philox: the top cell alone first)
  const bool lone = !rng.crn && (n & 1);
  if (lone && lane == 0) {
    double zi, zj;
    ps_normal_pair(rng, n, kmin, n - 1, zi, zj);
    zl[n - 1] = zi;
  }
  const int top = lone ? n - 2 : n - 1;  // cell top is a pair's upper half
  for (int q = lane; 2 * q <= top; q += 64) {
    const int i = top - 2 * q;
    double zi, zj;
    ps_normal_pair(rng, n, kmin, i, zi, zj);
    zl[i] = zi;
    if (i >= 1) zl[i - 1] = zj;
  }
  __syncthreads();
  if (lane == 0) {
    ps.acc[c] = INT_MAX;
    (void)ps_backsub<W>(ps.L + (size_t)c * ps.nmax * W, ps.ybar + (size_t)c * ps.nmax, n, rng, kmin, ps.elb,
                        e.Scur + (size_t)c * e.elbTmax * e.Ns, ps.cell + (size_t)c * ps.nmax, zl);
    ps.flag[c] = kmin + 1;
    ps.count[2 * c + (kept ? 1 : 0)] += 1;
    if (ps.state) __hip_atomic_store(&ps.state[c], ps.epoch << 1 | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// missingrate_all(thisMCMCdraw,:,:) = missingrate (mcmcVARshadowrate.m:498): proposal 1 of a PS
// sweep, NaN for a Gibbs sweep (:406) and beyond the vintage's window
__global__ void k_ps_first_store(const double* first, const int* elbT, const int* slot, double* out, int per,
                                 int Ns, int cap, int m) {
  const int c = blockIdx.x;
  const int T = elbT[slot[c]];
  double* o = out + ((size_t)c * cap + m) * per;
  for (int q = threadIdx.x; q < per; q += blockDim.x)
    o[q] = (first && q / Ns < T) ? first[(size_t)c * per + q] : __builtin_nan("");
}

// stackAccept(thisMCMCdraw) = ndxAccept (:457), 0 when the sweep fell back to Gibbs
__global__ void k_ps_store(const int* flag, int* out, int B, int cap, int m) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < B) out[(size_t)c * cap + m] = flag ? flag[c] : 0;
}

// ---------------------------------------------------------------- instantiations launched by ccmm_abi.hip
template __global__ void k_ps_chol_w<16>(Dims, ElbDev, PsDev, ChainState);
template __global__ void k_ps_chol_w<32>(Dims, ElbDev, PsDev, ChainState);
template __global__ void k_ps_chol_w<48>(Dims, ElbDev, PsDev, ChainState);
template __global__ void k_ps_chol_w<64>(Dims, ElbDev, PsDev, ChainState);
#define CCMM_PS_INST(W)                                                 \
  template __global__ void k_ps_prop<W>(ElbDev, PsDev, RngArgs);        \
  template __global__ void k_ps_apply<W>(ElbDev, PsDev, RngArgs, int);
CCMM_PS_INST(16)
CCMM_PS_INST(32)
CCMM_PS_INST(48)
CCMM_PS_INST(64)
CCMM_PS_INST(80)
#undef CCMM_PS_INST

}  // namespace ccmm
