/*
 * ccmm.h — C ABI of libccmm, the MI355X-native Gibbs sweep of the CCMM
 * shadow-rate BVAR-SV (Carriero, Clark, Marcellino & Mertens).
 *
 * Drop-in boundary.  Each entry point replaces one MATLAB function (or loop)
 * of the reference (Allisterh/CCMMshadowrateVAR-code @ 2025-01-27); the
 * reference file:line it replaces is cited beside it.  The MATLAB signatures
 * stay unchanged: a MEX gateway marshals mxArrays into these
 * calls.  Plain C types only: pointers to column-major fp64 host arrays
 * (MATLAB layout), int sizes, and opaque handles.
 *
 * Conventions
 *  - Every matrix argument is column-major, exactly the MATLAB array shape
 *    quoted in the comment ("T x N" means T rows, N columns).  Batched
 *    arguments append the chain index as the slowest dimension ("x B").
 *  - Return codes: 0 = OK; > 0 = warning (mirrors MATLAB warning(): e.g.
 *    CCMM_WARN_QR_FALLBACK, CTA.m:82); < 0 = error (mirrors error(): e.g.
 *    CCMM_ERR_DIM, gibbsdrawShadowrates.m:51).  ccmm_last_error() returns a
 *    thread-local message for the last non-zero return on this thread.
 *  - Host buffers belong to the caller and are never freed by the library.
 *    Device buffers, RNG state and scratch belong to the context / chain set.
 *  - Reentrancy: one context is bound to one device and serialises its calls
 *    on its own HIP stream; distinct contexts may be driven from distinct
 *    threads or processes (one per GPU).
 *  - Random numbers: every drawing entry point takes either a CRN array (the
 *    host-injected common random numbers, in the reference's draw order and
 *    shape) or NULL, in which case the library draws from its counter-based
 *    Philox4x32-10 generator keyed by (seed, chain, sweep, block).
 */
#ifndef CCMM_H
#define CCMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCMM_ABI_VERSION 4  /* 4: ccmm_batch_out.shadowratePSRFchains, kernel options, status bit 64 */

/* return codes */
#define CCMM_OK 0
#define CCMM_WARN_QR_FALLBACK 1    /* CTA.m:80-92 "switching to QR routine" */
#define CCMM_WARN_ELBT0 2          /* mcmcVARshadowrateBlockHybrid.m:203-205 */
#define CCMM_WARN_MVNCDF 3         /* censored log score with more than 12 series at the ELB: score NaN (4..12: deterministic lattice estimate inside MATLAB mvncdf's QMC tolerance 1e-4) */
#define CCMM_ERR_DIM (-1)          /* gibbsdrawShadowrates.m:50-52 "dimension mismatch" */
#define CCMM_ERR_ARG (-2)          /* invalid argument / unsupported size */
#define CCMM_ERR_HIP (-3)          /* HIP runtime failure */
#define CCMM_ERR_NOTSPD (-4)       /* Cholesky failure in a block without fallback */
#define CCMM_ERR_STATE (-5)        /* call order violated (e.g. sweep before set_data) */

/* per-chain status bits (ccmm_chains_get_status) */
#define CCMM_STATUS_QR 1            /* CTA Cholesky failed, the host QR branch of CTA.m:80-92 redrew the chain (valid) */
#define CCMM_STATUS_CTA 2           /* CTA Cholesky pivot <= 0 without the QR repair (invalid draws) */
#define CCMM_STATUS_ASTEP 4         /* A-step Cholesky pivot <= 0 (invalid draws) */
#define CCMM_STATUS_SV 8            /* SV sampler pivot <= 0 (invalid draws) */
#define CCMM_STATUS_PHI 16          /* PHI Cholesky pivot <= 0 (invalid draws) */
#define CCMM_STATUS_HANDOFF 32      /* a device hand-off between workgroups / waves reached its spin cap (invalid) */
#define CCMM_STATUS_PS_GIBBS 64     /* the PS precision was not positive definite: the Gibbs draw served the
                                       sweep, as the reference's fallback (:462-463) does (valid) */
#define CCMM_STATUS_INFO (CCMM_STATUS_QR | CCMM_STATUS_PS_GIBBS)  /* informational bits */

/* model ids for the sweep-level API */
#define CCMM_MODEL_LINEAR 0        /* mcmcVAR.m */
#define CCMM_MODEL_BLOCKHYBRID 1   /* mcmcVARshadowrateBlockHybrid.m */
#define CCMM_MODEL_HYBRID 2        /* mcmcVARhybridGibbs.m: K = N*p + 1 + Ns*p, X = [1, lags, Xffrlags] */
#define CCMM_MODEL_SHADOWRATE 3    /* mcmcVARshadowrate.m: shadow-rate design for every equation, ELB step
                                      as the block hybrid, the linear model's predictive density */

/* RNG block ids (Philox counter word 3); also the order of the per-sweep CRN blocks */
#define CCMM_RNG_PAI 1   /* randn(K,N)            CTA.m:58 / CTAsys.m:58 */
#define CCMM_RNG_A 2     /* 19x randn(ii-1,1)     mcmcVAR.m:251 */
#define CCMM_RNG_SVU 3   /* rand(N,T)             SV mixture indicators */
#define CCMM_RNG_SVZ 4   /* randn(N,T+1)          SV joint draw h_0..h_T */
#define CCMM_RNG_PHI 5   /* randn(N,T+d_PHI)      mcmcVAR.m:268 */
#define CCMM_RNG_ELB 6   /* rand(Ns,elbT,101)     gibbsdrawShadowrates.m:173 */
#define CCMM_RNG_FCST 7  /* randn(N,H*Nd) then randn(N,H,Nd)  mcmcVAR.m:302,306 */
#define CCMM_RNG_PS 8    /* randn(nmiss,Nproposals)  PS proposals, mcmcVARshadowrateBlockHybrid.m:439-441 */

typedef struct ccmm_ctx ccmm_ctx;
typedef struct ccmm_chains ccmm_chains;

/* ---------------------------------------------------------------- context */
int ccmm_abi_version(void);
const char* ccmm_last_error(void);
/* Environment.  A default build reads NO environment variable: kernel forms and schedules are the
 * explicit options below.  Timing-only ablation variables (CCMM_CHOL_SKIP, CCMM_SOLVE_SKIP, CCMM_SV_SKIP,
 * CCMM_GC_MODE, CCMM_LAG_MODE, CCMM_BIG_MASK, CCMM_ELB_MODE, the ablation bits of CCMM_SV_MODE,
 * CCMM_FCST_MODE, CCMM_POISON) leave the draws invalid and, like the options' CCMM_* defaults, are read
 * only by a build with -DCCMM_ABLATION (`make ablation`: libccmm_ablation.so); ccmm_ablation_build()
 * returns 1 there.  ccmm_env_ignored() returns how many CCMM_* variables the library knows are set and
 * ignored (names comma-separated in buf, len bytes with the terminator; buf may be NULL), and
 * ccmm_chains_create() leaves the same list in ccmm_last_error() as a warning. */
int ccmm_ablation_build(void);
int ccmm_env_ignored(char* buf, int len);
/* Kernel options: choices between kernel forms and schedules, set explicitly per context (inherited by
 * the chain sets created on it afterwards and used by the block-level drop-ins) or per chain set.
 * Schedules give bit-identical draws: solve_split (-1 auto, 0, 1), solve_async (0/1), sv_nwg (0 auto,
 * 1, 2, 4), elb_waves (1, 4, 8), elb_oct (0, 1 auto, 2), elb_async (0/1), elb_parts (0 auto, 1, 2, 4:
 * workgroups per chain of the ELB wavefront), fcst_reg (0/1), phi_overlap (0/1), qr_fallback (0/1),
 * big_lagx (0/1: the large path reads the column-major lag twin of a lag-structured X; set before
 * ccmm_chains_set_data).
 * Forms run the same algorithm in another summation order (or the QR branch): lag (0/1), large_path
 * (0/1; set before ccmm_chains_set_data), astep_serial, ps_chol_lds, sv_mfma (0/1), force_qr,
 * girf_generic.  CCMM_ERR_ARG for an unknown name or a value out of range. */
int ccmm_option_count(void);
const char* ccmm_option_name(int i);
/* The value a new context starts from (host only): the built-in default in a default build, whatever the
 * environment holds; the ablation build's CCMM_* override. */
int ccmm_option_default(const char* name, int* value);
int ccmm_device_count(void);
/* Create a context bound to HIP device `device`.  Returns NULL on failure. */
ccmm_ctx* ccmm_create(int device);
void ccmm_destroy(ccmm_ctx* ctx);
int ccmm_synchronize(ccmm_ctx* ctx);
int ccmm_set_option(ccmm_ctx* ctx, const char* name, int value);
int ccmm_get_option(ccmm_ctx* ctx, const char* name, int* value);

/* --------------------------------------------------- block-level drop-ins */

/* Triangular (CTA) draw of the VAR coefficients, batched over B chains.
 * Replaces CTA.m:1-98 (called at mcmcVAR.m:228, mcmcVARhybridGibbs.m:376) and
 * CTAsys.m:1-108 (called at mcmcVARshadowrateBlockHybrid.m:343).
 *   Y      T x N (x B if y_per_chain)
 *   X      T x K x nx (x B if x_per_chain); equation j uses slab (nx==1 ? 0 : j)
 *          nx == 1 is CTA, nx == N is CTAsys
 *   A      N x N x B   unit lower triangular A_
 *   sqrtht T x N x B
 *   iVdiag K x N       diagonal of the block-diagonal prior precision iV (mcmcVAR.m:186)
 *   iVb    K x N       iVb_prior reshaped to K x N
 *   PAI    K x N x B   in: previous draw (columns j+1..N used by CTAsys); out: new draw
 *   z      K x N x B   randn(K,N) of CTA.m:58, or NULL (Philox, block CCMM_RNG_PAI, sweep 0)
 *   status B           per-chain status (0 ok, 1 QR fallback used), may be NULL
 * A chain whose posterior precision fails the device Cholesky is redrawn on the host by
 * the QR branch of CTA.m:80-92 (Householder QR of Kailath's array; same previous draw and
 * normals); the call then returns CCMM_WARN_QR_FALLBACK.  CCMM_ERR_NOTSPD only when the
 * QR factor itself is singular.
 * Supports 1 <= N <= 128, K <= 1536. */
int ccmm_cta(ccmm_ctx* ctx, int B, int T, int N, int K,
             const double* Y, int y_per_chain,
             const double* X, int nx, int x_per_chain,
             const double* A, const double* sqrtht,
             const double* iVdiag, const double* iVb,
             double* PAI, const double* z, int* status);

/* CTAsysAswitching.m:1-123 (the Aelb shadow-rate model's coefficient block): as ccmm_cta with
 * CTAsys designs, but the months with atELB[t] != 0 use the second A matrix Aelb in the residual
 * map and the weights (CTAsysAswitching.m:61-80: kron(Aelb_(j:N,j), XatELB) stacked over
 * kron(A_(j:N,j), XawayELB)).  Aelb N x N x B, atELB T bytes (logical, shared by the chains).
 * The QR branch (:82-93) is the host fallback of ccmm_cta with the same two-matrix map.
 * Supports N <= 32, K <= 256. */
int ccmm_cta_aswitching(ccmm_ctx* ctx, int B, int T, int N, int K,
                        const double* Y, int y_per_chain,
                        const double* X, int nx, int x_per_chain,
                        const double* A, const double* Aelb, const uint8_t* atELB,
                        const double* sqrtht, const double* iVdiag, const double* iVb,
                        double* PAI, const double* z, int* status);

/* A-matrix draw, flat prior (mcmcVAR.m:236-254 == mcmcVARshadowrateBlockHybrid.m:354-372).
 *   RESID T x N x B, sqrtht T x N x B, z (N(N-1)/2) x B or NULL
 *   A out N x N x B (unit lower), invA out N x N x B (A_\I, mcmcVAR.m:254) */
int ccmm_astep(ccmm_ctx* ctx, int B, int T, int N, const double* RESID, const double* sqrtht,
               const double* z, double* A, double* invA);

/* Stochastic-volatility block: KSC 7-component mixture indicators and joint
 * draw of the random-walk log variances with correlated shocks.  Replaces the
 * em-matlabbox call StochVolKSCcorrsqrt (mcmcVAR.m:261,
 * mcmcVARshadowrateBlockHybrid.m:379, mcmcVARhybridGibbs.m:405).
 *   logy2T N x T x B (logy2'), hprevT N x T x B (Vol_states'), sqrtPHI N x N x B lower,
 *   h0mean N, h0vcvsqrt N x N, u N x T x B or NULL, z N x (T+1) x B or NULL
 *   hT out N x T x B, h0 out N x B, shocksT out N x T x B, kai2 out N x T x B (int8, 1..7) */
int ccmm_sv_ksc(ccmm_ctx* ctx, int B, int T, int N, const double* logy2T, const double* hprevT,
                const double* sqrtPHI, const double* h0mean, const double* h0vcvsqrt,
                const double* u, const double* z, double* hT, double* h0, double* shocksT,
                int8_t* kai2);

/* Inverse-Wishart draw of the SV shock covariance (mcmcVAR.m:268-274).
 *   eta T x N x B, sPHI N x N, dPHI, Zdraw N x (T+dPHI) x B or NULL
 *   sqrtPHI out N x N x B (lower Cholesky of PHI_), PHI out N x N x B */
int ccmm_phi_iw(ccmm_ctx* ctx, int B, int T, int N, const double* eta, const double* sPHI,
                int dPHI, const double* Zdraw, double* sqrtPHI, double* PHI);

/* Gibbs draw of the ELB-censored shadow rates given the VAR state space, batched over B
 * independent calls.  Replaces gibbsdrawShadowrates.m:1-245 (called at
 * mcmcVARshadowrateBlockHybrid.m:436,462,494 and mcmcVARhybridGibbs.m:481,513).
 *   ndxS   Ny (logical)            sNaN  Ns x elbT (logical; censored cells)
 *   Y      Ny x elbT x B           the window, previous shadow values in censored cells
 *   STATE0 K x B (K = Ny p + 1)    YHAT0 Ny x elbT x B or NULL (zeros)
 *   C      K x K x B  (elb.A)      Psi   K x Ny x B (elb.B: invA in rows 2..Ny+1)
 *   SVol   Ny x elbT x B           u     Ns x elbT x (burnin + Ndraws) x B uniforms
 *                                        (rand(rndStream, Ns, elbT, .), :173) or NULL (Philox)
 *   out    Ns x elbT x Ndraws x B  flags Ns x elbT x (burnin + Ndraws) x B (drawTruncNormal
 *                                        branches, as ccmm_draw_trunc_normal) or NULL
 * Ndraws must be 1 (the reference's only use).  Evaluated in the stable residual form of the
 * device ELB step (ccmm_elb.hip): the same conditional moments as the QR formulation of
 * gibbsdrawShadowrates.m:74-145 in exact arithmetic, on the structural matrix A = Psi(2:Ny+1, :)^-1.
 * Any invertible impact matrix: a lower-triangular one (every reference caller passes invA,
 * mcmcVARshadowrateBlockHybrid.m:418) by forward substitution, a general one by Gauss-Jordan with
 * partial pivoting and the conditionals on the full A.  CCMM_ERR_ARG when Psi(2:Ny+1, :) is
 * singular; CCMM_ERR_DIM: sum(ndxS) != Ns (gibbsdrawShadowrates.m:50-52). */
int ccmm_gibbs_shadowrates(ccmm_ctx* ctx, int B, int Ny, int elbT, int Ns, int p, const uint8_t* ndxS,
                           const uint8_t* sNaN, const double* Y, const double* STATE0,
                           const double* YHAT0, const double* C, const double* Psi, const double* SVol,
                           double elbBound, int Ndraws, int burnin, const double* u, double* out,
                           uint8_t* flags);

/* gibbsdrawShadowratesB3 (gibbsdrawShadowratesB3.m:1-231, the 12-argument signature
 * (Y, STATE0, ndxS, sNaN, p, A, B, SVol, elbBound, Ndraws, burnin, rndStream)), batched over B calls:
 * the same Gibbs passes with the VAR run on Y itself (intercept in the state, STATElag starting at
 * STATE0, no deterministic Y0 path: :171-185) and an impact matrix that may vary by month.
 *   A      K x K x B (the companion with intercept)
 *   Bmat   K x Ny x elbT x B when B3d != 0 (B(:,:,t), :49-62), else K x Ny x B (repeated over t);
 *          rows 2..Ny+1 any invertible matrix (as ccmm_gibbs_shadowrates' Psi; every caller's B = invA)
 * The other arguments as ccmm_gibbs_shadowrates (no YHAT0).  The reference's only caller
 * (mcmcVARshadowrateBlockHybridAelb.m:451-452, 469-470) passes 13 arguments to this 12-parameter
 * function and cannot run as shipped; this entry serves the function itself. */
int ccmm_gibbs_shadowrates_b3(ccmm_ctx* ctx, int B, int Ny, int elbT, int Ns, int p, const uint8_t* ndxS,
                              const uint8_t* sNaN, const double* Y, const double* STATE0, const double* A,
                              const double* Bmat, int B3d, const double* SVol, double elbBound, int Ndraws,
                              int burnin, const double* u, double* out, uint8_t* flags);

/* One draw from N(mu, sig^2) truncated to (-inf, elb] by inverse CDF
 * (drawTruncNormal.m:31-86) with a pre-drawn uniform u (the numeric-stream
 * form of drawTruncNormal.m:47-48).  flags (may be NULL): bit0 = |sig| > 1e-10
 * branch taken, bit1 = PHIbar > eps branch taken.  Host-side scalar; the
 * device form runs inside the block-hybrid sweep (k_elb_gibbs). */
double ccmm_draw_trunc_normal(double mu, double sig, double elb, double u, uint8_t* flags);

/* Batched device evaluation of drawTruncNormal over n independent cells. */
int ccmm_draw_trunc_normal_batch(ccmm_ctx* ctx, int n, const double* mu, const double* sig,
                                 double elb, const double* u, double* out, uint8_t* flags);

/* --------------------------------------------------- sweep-level (device-resident) */

typedef struct {
  int model;              /* CCMM_MODEL_* */
  int N, p, K;            /* K = N*p + 1 */
  int T;                  /* max T over data slots */
  int B;                  /* number of chains */
  int ndata;              /* number of data slots (vintages) */
  int dPHI;               /* N + 3 (mcmcVAR.m:164) */
  int rng_crn;            /* 1: sweeps read CRN arrays from the host; 0: Philox */
  int store_capacity;     /* kept draws stored per chain (0: no storage) */
  double logy2offset;     /* getKSC7values offset (ext; this build declares 1e-3) */
  uint64_t seed;          /* Philox key */
  /* CCMM_MODEL_BLOCKHYBRID only (ignored otherwise) */
  int Ns;                 /* number of shadow-rate variables, 1..5 (Nshadowrates; 5 with the Krippner / Wu-Xia data at ELB > 0.25) */
  int elbTmax;            /* max over data slots of elbT = T - elbT0 */
  int elb_gibbsburn;      /* Gibbs burn-in passes per sweep (gibbsdrawShadowrates call, :436: 100) */
  double elb;             /* ELBbound */
} ccmm_chain_config;

ccmm_chains* ccmm_chains_create(ccmm_ctx* ctx, const ccmm_chain_config* cfg);
void ccmm_chains_destroy(ccmm_chains* ch);
/* Kernel options of one chain set (see ccmm_set_option; initialised from its context at create). */
int ccmm_chains_set_option(ccmm_chains* ch, const char* name, int value);
int ccmm_chains_get_option(ccmm_chains* ch, const char* name, int* value);

/* Data slot `slot`: one vintage's design (mcmcVAR.m:62-72, 186; 164-169).
 *   Y T x N, X T x K, iVdiag K x N, iVb K x N, sPHI N x N, h0mean N, h0vcvsqrt N x N */
int ccmm_chains_set_data(ccmm_chains* ch, int slot, int T, const double* Y, const double* X,
                         const double* iVdiag, const double* iVb, const double* sPHI,
                         const double* h0mean, const double* h0vcvsqrt);
/* slot_of_chain B ints (default: all chains use slot 0). */
int ccmm_chains_set_slots(ccmm_chains* ch, const int* slot_of_chain);
/* Chain state PREVdraw (mcmcVAR.m:197-206, 386-392): PAI K x N x B, A N x N x B,
 * sqrtht T x N x B, h (Vol_states) T x N x B, sqrtPHI N x N x B.  Resets the sweep counter. */
int ccmm_chains_set_state(ccmm_chains* ch, const double* PAI, const double* A,
                          const double* sqrtht, const double* h, const double* sqrtPHI);
/* Philox stream id of every chain (counter word 1; B values; NULL restores the default,
 * the chain index).  A batch driver keys chains by their global (vintage, chain) unit so
 * draws do not depend on how units are sharded over GPUs or packed into chain sets. */
int ccmm_chains_set_rng_ids(ccmm_chains* ch, const uint32_t* ids);
/* Opt-in MFMA phase lock (id > 0; 0 = none).  Chain sets on one device given the same id
 * serialise the MFMA Gram + Cholesky phase of their coefficient block (large-system path,
 * K > 512 or N > 32) through a cross-stream event.  Groups of chains driven on separate
 * contexts then fall out of step, and the per-chain sequential blocks of one group (CTA
 * solve, SV recursion, ELB Gibbs) overlap another group's MFMA phase.  Draws are unchanged. */
int ccmm_chains_set_mfma_lock(ccmm_chains* ch, int id);
/* KSC mixture indicators of the last SV block (T x N x B int8, 1..7; the draw of the
 * em-matlabbox sampler, mcmcVAR.m:261). */
int ccmm_chains_get_kai(ccmm_chains* ch, int8_t* kai);
/* Record the drawTruncNormal branch flags (as ccmm_draw_trunc_normal: bit0 |sig| > 1e-10,
 * bit1 PHIbar > eps) of every ELB step; get_elb_flags returns the last sweep's as
 * Ns x elbTmax x (gibbsburn + 1) x B uint8 (0 for uncensored cells). */
int ccmm_chains_record_elb_flags(ccmm_chains* ch, int enable);
int ccmm_chains_get_elb_flags(ccmm_chains* ch, uint8_t* flags);
/* Per-chain status word since set_state (B ints, OR of CCMM_STATUS_*: 2 CTA Cholesky, 4 A-step
 * Cholesky, 8 SV sampler, 16 PHI Cholesky found a non-positive pivot; the block
 * then continued with a unit pivot, so the chain's draws are invalid; 32: a device hand-off
 * between workgroups or waves reached its spin cap, never expected).  A CTA Cholesky
 * failure is repaired within the sweep by the host QR branch of CTA.m:80-92, which
 * replaces bit 2 by bit 1 ("QR fallback used", informational: the draws are valid); bit 64
 * (informational) marks a sweep whose PS precision failed and whose Gibbs draw served instead.
 * Returns 1 if any chain carries a bit outside CCMM_STATUS_INFO, 0 otherwise; the batch driver re-runs
 * flagged units (goVARshadowrateBlockHybrid.m:287-310). */
int ccmm_chains_get_status(ccmm_chains* ch, int* status);
/* Any output pointer may be NULL.  invA, PHI, RESID are those of the last sweep. */
int ccmm_chains_get_state(ccmm_chains* ch, double* PAI, double* A, double* invA, double* sqrtht,
                          double* h, double* sqrtPHI, double* PHI, double* RESID);
/* CRN doubles consumed per chain per sweep (blocks in CCMM_RNG_* order). */
int64_t ccmm_chains_crn_len(const ccmm_chains* ch);
/* Run nsweeps Gibbs sweeps (the body of `while m < MCMCreps`, mcmcVAR.m:195-398,
 * excluding the predictive block).  crn: B x nsweeps x crn_len (chain slowest) or
 * NULL in Philox mode.  store != 0 stores each sweep's draw (post-burn-in
 * semantics of mcmcVAR.m:278-292) into the on-device draw buffer.  Asynchronous
 * with respect to the host unless crn != NULL. */
int ccmm_chains_sweep(ccmm_chains* ch, int nsweeps, const double* crn, int store);
/* Number of stored draws per chain so far. */
int ccmm_chains_stored(const ccmm_chains* ch);
/* Copy stored draws out in the reference layout (mcmcVAR.m:178-181, 289-292;
 * mcmcVARshadowrateBlockHybrid.m:284-288, 536-543):
 *   PAI_all M x K x N x B, PHI_all M x N(N+1)/2 x B, invA_all M x N x N x B,
 *   sqrtht_all M x T x N x B, shadowrate_all M x Ns x elbTmax x B (block-hybrid;
 *   NaN beyond a vintage's elbT).  Any pointer may be NULL.  Resets the store. */
int ccmm_chains_get_draws(ccmm_chains* ch, double* PAI_all, double* PHI_all, double* invA_all,
                          double* sqrtht_all, double* shadowrate_all);
/* Running moments of the stored PAI draws on the device (the PAImean / PAIstdev accumulation of
 * goVARshadowrateBlockHybrid.m:376-377 without copying every draw to the host): adds the draws stored
 * so far (in store order, x then x * x, one rounding each) to per-chain running sums, reset first when
 * reset != 0; copies the sums out (K x N x B each) when the pointers are non-NULL.  Does not reset the
 * store (call before ccmm_chains_get_draws). */
int ccmm_chains_pai_moments(ccmm_chains* ch, int reset, double* sum, double* sumsq);

/* ---- predictive density inside the chain set (post-burn-in block of
 *      mcmcVAR.m:298-381 and mcmcVARshadowrateBlockHybrid.m:550-669) ----
 * Once configured, every stored sweep (ccmm_chains_sweep with store != 0) also
 * simulates Nd forecast paths of H horizons per chain from the chain's draw, without
 * leaving the device: Xjumpoff from the chain's resident data (block hybrid: shadow-rate
 * lags plus the vintage's actual-rate lags, :511-520), SV paths, the companion recursion
 * (linear: ltitr + censored simulation + zero-shock mean path; block hybrid: one
 * simulation on the K + Nyields p states with the actual rates max(shadow, ELB), :615-623)
 * and the one-step log scores (logscoreGaussian.m, logscoreGaussianCensored.m).
 * CRN mode appends randn(N, H*Nd) and randn(N, H, Nd) (block CCMM_RNG_FCST) to every
 * sweep's CRN record.  Linear and block-hybrid models, N <= 32.
 *   ndxYields N bytes (ndxYIELDS), keep_paths != 0 keeps every path for quantiles/CRPS.
 * Call after set_elb_model (block hybrid) and before sweeping. */
int ccmm_chains_set_fcst(ccmm_chains* ch, int H, int Nd, const uint8_t* ndxYields, int keep_paths);
/* yrealized(:,1) of data slot `slot` (N values; goVARshadowrateBlockHybrid.m:267-283,
 * shadow rates floored at the ELB by the caller). */
int ccmm_chains_set_fcst_slot(ccmm_chains* ch, int slot, const double* yrealized);
/* Linear predictive density: the variables floored at the ELB inside the censored
 * simulation (N bytes; NULL restores the default ndxYields, mcmcVAR.m:360-366).
 * mcmcVARshadowrate.m:539-546 floors ndxOTHERYIELDS only. */
int ccmm_chains_set_fcst_censor(ccmm_chains* ch, const uint8_t* floor_in_recursion);
/* Kept draws with a forecast record so far (-1: not configured). */
int ccmm_chains_fcst_stored(const ccmm_chains* ch);
/* Copy out and reset the forecast records of the M kept draws so far:
 *   scores   Nd x M x 4 x B: (:,:,k,c) reshaped to fcstNdraws x 1 is, for k = 0..3,
 *            fcstLogscoreDraws (uncensored Gaussian), fcstLogscoreELBdraws (censored; the
 *            block-hybrid fcstLogscoreDraws, :588-593), fcstLogscoreXdraws, fcstLogscoreIdraws
 *   fYsum    N x H x B  sum over the M x Nd paths (linear fcstYdraws; block hybrid the
 *            uncensored fcstShadowrateDraws)
 *   fYcsum   N x H x B  sum of the censored paths (linear fcstYcensorDraws; block hybrid
 *            fcstYdraws with the yields floored at the ELB, :697-700)
 *   yhatsum  N x H x B  sum of the zero-shock mean paths (linear yhatdraws; zero for bh)
 *   paths, paths_censored  N x H x Nd x M x B (only with keep_paths)
 * Any pointer may be NULL.  Censored scores with 4..12 series at the ELB use a deterministic
 * lattice estimate of mvncdf (MATLAB: randomised QMC, absolute tolerance 1e-4); returns
 * CCMM_WARN_MVNCDF when some censored score needed mvncdf in more than 12 dimensions (NaN). */
int ccmm_chains_get_fcst(ccmm_chains* ch, double* scores, double* fYsum, double* fYcsum,
                         double* yhatsum, double* paths, double* paths_censored);

/* ---- shadow-rate models: block-hybrid (mcmcVARshadowrateBlockHybrid.m) and
 *      hybrid (mcmcVARhybridGibbs.m) ----
 * Hybrid: every equation uses the chain's X = [1, lags of the shadow-rate data,
 * Xffrlags] (CTA, mcmcVARhybridGibbs.m:376); the trailing Ns*p columns of the
 * slot X are the actual-rate lags floored at the ELB (:77-84) and stay fixed;
 * the ELB step adds Yhatactual = Xffrlags * PAI(Kshadow+1:end,:) (:429-431) and
 * uses PAI(1:Kshadow,:) in the companion matrix (:435-437).  actual_block must be
 * NULL (or all zero) for the hybrid model.
 * Data slot X/Y (ccmm_chains_set_data) are the vintage's ACTUAL data (X0, Y0,
 * :310-316); every chain keeps its own shadow-rate copy, reset to the slot's
 * data by ccmm_chains_set_state.  Equations with actual_block[j] != 0 use the
 * slot's X (CTAsys design of the actual-rate block), the others the chain's.
 *
 * ndxS: Ns strictly increasing 0-based shadow-rate variable indices (ndxSHADOWRATE);
 * actual_block: N bytes, actualrateBlock (:80-84).  Call before set_state. */
int ccmm_chains_set_elb_model(ccmm_chains* ch, const int* ndxS, const uint8_t* actual_block);
/* Per vintage: elbT0 (first VAR row, 0-based, of the ELB window; :176-183) and
 * sNaN Ns x elbT (column-major, elbT = T_slot - elbT0): nonzero where the shadow
 * rate is censored (data <= ELB, :163-171).  Call after ccmm_chains_set_data. */
int ccmm_chains_set_elb_slot(ccmm_chains* ch, int slot, int elbT0, const uint8_t* sNaN);
/* Acceptance-sampling branch of the ELB step (mcmcVARshadowrateBlockHybrid.m:435-466):
 * from sweep m >= ps_from_m (1-based; the reference: m >= MCMCburnin/2, i.e.
 * ps_from_m = ceil(MCMCburnin/2)) every sweep first draws nproposals (elb.Nproposals =
 * 1e3, :188) unconstrained proposals of the censored cells from their joint Gaussian
 * given the VAR — the em-matlabbox sampler VARTVPSVprecisionsamplerNaN (:439-441), restated
 * as the precision sampler y_m = L' \ (L \ b + z_k), P = L L' — and accepts the first
 * whose censored cells all lie below the ELB (:446-452); otherwise the Gibbs draw of
 * gibbsdrawShadowrates serves the sweep (:462-463).  CRN mode appends randn(nmiss,
 * nproposals) (block CCMM_RNG_PS, nmiss x nproposals column-major, sized Ns elbTmax
 * nproposals) to every sweep's record.  nproposals = 0: Gibbs every sweep (default).
 * Requires Ns (p + 1) <= 80. */
int ccmm_chains_set_elb_ps(ccmm_chains* ch, int nproposals, int ps_from_m);
/* PS bookkeeping (:303-305, 453-460): countAccept / countAcceptBurnin B ints since set_state
 * (sweeps whose proposal was accepted after / during burn-in), stackAccept M x B ints
 * (ndxAccept of each stored draw, 0 = no proposal accepted or Gibbs sweep; M = stored draws;
 * call before ccmm_chains_get_draws, which resets the store).  Any pointer may be NULL. */
int ccmm_chains_get_ps(ccmm_chains* ch, int* countAccept, int* countAcceptBurnin, int* stackAccept);
/* missingrate_all (mcmcVARshadowrate.m:270, 435, 498; mcmcVARhybridGibbs.m:332, 486): with enable != 0
 * every stored sweep also keeps proposal 1 of its PS branch (shadowrateProposals(:,:,1): the censored cells
 * from the sampler, the others the window's data); a sweep that ran the Gibbs branch stores NaN (:406).
 * Call before the first stored sweep.  get_missingrate: M x Ns x elbTmax x B, NaN beyond a vintage's
 * window; call before ccmm_chains_get_draws (which resets the store).  The block-hybrid driver keeps
 * missingrate NaN (doELBsampleAlternate = false, mcmcVARshadowrateBlockHybrid.m:470-478). */
int ccmm_chains_keep_missingrate(ccmm_chains* ch, int enable);
int ccmm_chains_get_missingrate(ccmm_chains* ch, double* missingrate_all);
/* Parity diagnostic of the PS branch: the conditional mean P^-1 b of the censored cells that
 * the last PS sweep's proposals were drawn around (VARTVPSVprecisionsamplerNaN at z = 0,
 * mcmcVARshadowrateBlockHybrid.m:439-441), Ns x elbTmax x B, NaN outside the censored cells
 * (the device's banded factor, back-substituted on the host). */
int ccmm_chains_get_ps_mean(ccmm_chains* ch, double* mean);
/* Parity diagnostic: the device's weighted Gram of every CTA system at the chain set's current
 * state (A, sqrtht, X), K x K x N x B: [c b'; b M] with c = sum_t w_t, b = X~' w, M = X~' diag(w) X~
 * (CTA.m:73 without the prior), exactly as the lag-structured coefficient kernel forms it before
 * the factorisation.  Only when that path is active (linear / block-hybrid models, N <= 32). */
int ccmm_chains_get_cta_gram(ccmm_chains* ch, double* G);
/* Parity diagnostic: the factor record of every CTA system at the current state as the lag-structured
 * kernel writes it, (NT (NT + 1) / 2 * 256 + 256) doubles per system (NT = ceil((K - 1) / 16)), systems
 * ordered (equation, chain): the 16 x 16 factor tiles in slot order (slot g = column-major enumeration of
 * the lower tile pairs (ti, tj); element (row (lane >> 4) + 4 r, column lane & 15) at g 256 + 64 r + lane;
 * off-diagonal slots the unit block factor's blocks, diagonal slots the inverses of the diagonal
 * factor tiles, transposed), then [1 / L00, L(1 + a, 0) for a = 0..16 NT - 1].  Same path as
 * ccmm_chains_get_cta_gram. */
int ccmm_chains_get_cta_factor(ccmm_chains* ch, double* F);
/* Current shadow rates, Ns x elbTmax x B (the last sweep's draw). */
int ccmm_chains_get_shadowrate(ccmm_chains* ch, double* shadowrate);
/* Current per-chain data: X T x K x B, Y T x N x B (block-hybrid: the chain's
 * shadow-rate X/Y, PREVdraw.X/Y; linear: the slot's data).  Either may be NULL. */
int ccmm_chains_get_xy(ccmm_chains* ch, double* X, double* Y);
/* Per-kernel device time (HIP events on the chain set's stream) accumulated
 * while profiling is on.  names: ';'-separated list written into buf. */
int ccmm_chains_profile(ccmm_chains* ch, int enable);
int ccmm_chains_kernel_times(ccmm_chains* ch, int max, double* ms, int64_t* launches,
                             char* names, int names_len);

/* ------------------------------------------------------------ post-processing
 * Per-vintage summaries of kept draws (goVARshadowrateBlockHybrid.m:349-480), on the
 * device: for each series the mean, median, quantiles at pct[0..nq-1] (MATLAB prctile:
 * the i-th sorted draw sits at percentile 100 (i - 0.5)/n, linear in between), std(., 1)
 * and, when realized is given, crpsDraws (the CRPS of the draws' empirical distribution,
 * mean|x - y| - sum_ij |x_i - x_j| / (2 n^2); em-matlabbox source absent).  Outputs
 * mean/median/stdev/crps S, quantiles S x nq (series fastest); any may be NULL. */
/* Host draws n x S (each series' n draws contiguous), realized S or NULL. */
int ccmm_draw_summaries(ccmm_ctx* ctx, int S, int n, const double* draws, const double* realized, int nq,
                        const double* pct, double* mean, double* median, double* quantiles, double* stdev,
                        double* crps);
/* The kept draws of the chains bound to data slot `slot` (contiguous chain indices), pooled:
 *   source 0  forecast paths (keep_paths; linear fcstYdraws, block hybrid the uncensored
 *             shadow-rate paths), series = selected rows x H (row fastest), draws = chains x
 *             kept records x Nd
 *   source 1  censored forecast paths (linear fcstYcensorDraws, block hybrid fcstYdraws)
 *   source 2  PAI draws, series = K x N, draws = chains x stored draws
 * rows: N bytes selecting the variables (NULL: all); cumcode: N bytes, cumsum over the
 * horizons for those variables first (:353-355; NULL: none). */
int ccmm_chains_summaries(ccmm_chains* ch, int source, int slot, const uint8_t* rows, const uint8_t* cumcode,
                          const double* realized, int nq, const double* pct, double* mean, double* median,
                          double* quantiles, double* stdev, double* crps);
/* As ccmm_chains_summaries, with the forecast paths of the variables selected by floor_rows (N
 * bytes) floored at `floor` first, y(y < floor) = floor, before any cumsum: the shadow-rate
 * VAR's draws (mcmcVARshadowrate.m:642-645 fcstYdraws, yields floored on the uncensored paths;
 * :676-681 fcstYcensorDraws, shadow rates floored on the censored paths) summarised by
 * goVARshadowrate.m:356-478.  Sources 0 and 1 only. */
int ccmm_chains_summaries_floor(ccmm_chains* ch, int source, int slot, const uint8_t* rows, const uint8_t* cumcode,
                                const uint8_t* floor_rows, double floor, const double* realized, int nq,
                                const double* pct, double* mean, double* median, double* quantiles, double* stdev,
                                double* crps);

/* ------------------------------------------------------------ batch run (the vintage loop)
 * ccmm_run_batch replaces the parfor over vintages of goVARshadowrateBlockHybrid.m:258-517
 * (goVARhybrid.m:258 for the hybrid model, goVAR.m:242 for the linear one) for the vintages
 * handed to this process: ONE device-resident chain set holds every vintage as a data slot with
 * `nchains` chains; each chain runs `burnin` + MCMCdraws sweeps (mcmcVARshadowrateBlockHybrid.m:
 * 56-58, 306-689) and every kept sweep simulates fcstNdraws / MCMCdraws forecast paths on the
 * device (:550-625).  The ELB step is the Gibbs sampler for m < ceil(burnin / 2) and the
 * accept-first PS proposals after (:433-466; hybrid: PS at every sweep, mcmcVARhybridGibbs.m:458;
 * Nproposals = 0: Gibbs every sweep).  Philox streams: chain c of vintage v is keyed by
 * unit(v) * nchains + c (+ 1000003 per retry), so results do not depend on how vintages are
 * sharded over processes.  Failure recovery (goVARshadowrateBlockHybrid.m:287-310): a vintage
 * whose chains flagged a non-SPD pivot (ccmm_chains_get_status bits other than 1) is re-run from
 * its initial state on fresh streams, up to max_retries times; after that its outputs are NaN.
 * The setup of each vintage (data matrices, Minnesota prior, initial PREVdraw) is the caller's:
 * the MATLAB driver's own code computes it (mcmcVARshadowrateBlockHybrid.m:30-295, :308-317). */
typedef struct {
  int T;                        /* VAR rows (thisT - p) */
  const double* Y;              /* T x N (actual data, :62-72) */
  const double* X;              /* T x K */
  const double* iVdiag;         /* K x N (diagonal of iV, mcmcVAR.m:186) */
  const double* iVb;            /* K x N */
  const double* sPHI;           /* N x N */
  const double* h0mean;         /* N     Vol_0mean */
  const double* h0vcvsqrt;      /* N x N Vol_0vcvsqrt */
  const double* PAI0;           /* K x N  PREVdraw.PAI at m == 0 (X\Y, :308) */
  const double* sqrtht0;        /* T x N  PREVdraw.sqrtht at m == 0 (AR residuals, :313) */
  const double* h0init;         /* T x N  PREVdraw.Vol_states at m == 0 (2 log(sqrtht0), :314), or NULL:
                                   computed here */
  int elbT0;                    /* shadow-rate models: first VAR row (0-based) of the ELB window */
  const uint8_t* sNaN;          /* Ns x (T - elbT0) censored cells (may be NULL when T == elbT0) */
  const double* yrealized;      /* N x H (goVARshadowrateBlockHybrid.m:267-283, floored at the ELB) */
  uint32_t unit;                /* global vintage index (Philox stream key) */
} ccmm_vintage;

typedef struct {
  int model;                    /* CCMM_MODEL_LINEAR, _BLOCKHYBRID or _HYBRID */
  int N, p;                     /* K = N p + 1 (+ Ns p for the hybrid model) */
  int Ns;                       /* shadow-rate models: number of shadow rates */
  const int* ndxS;              /* Ns 0-based ndxSHADOWRATE */
  const uint8_t* actual_block;  /* N bytes, actualrateBlock (block hybrid; NULL otherwise) */
  const uint8_t* ndxYields;     /* N bytes, ndxYIELDS (forecast censoring) */
  int nchains;                  /* chains per vintage */
  int MCMCdraws;                /* kept sweeps per chain */
  int burnin;                   /* burn-in sweeps per chain (the reference: MCMCdraws) */
  int gibbsburn;                /* Gibbs passes per ELB step before the kept one (100) */
  int Nproposals;               /* elb.Nproposals (1000); 0: Gibbs ELB step every sweep */
  int fcstNdraws;               /* multiple of MCMCdraws (:123-126) */
  int H;                        /* fcstNhorizons */
  double elb;                   /* ELBbound */
  uint64_t seed;                /* rndStream seed */
  int chunk;                    /* sweeps per device call (host synchronisation points) */
  int max_retries;
  int postprocess;              /* keep every kept draw and path in HBM; device summaries */
  int nq;                       /* number of quantiles (postprocess) */
  const double* pct;            /* nq percentiles (setQuantiles) */
  const uint8_t* cumcode;       /* N bytes or NULL: cumsum over horizons (:353-355) */
} ccmm_batch_config;

typedef struct {                /* V = number of vintages; any pointer may be NULL */
  double* logscore;             /* 4 x V log mean exp over the fcstNdraws * nchains one-step score
                                   draws (k as ccmm_chains_get_fcst: 1 = fcstYmvlogscore, 2 = X,
                                   3 = I; :437-447) */
  double* fcstYhat;             /* N x H x V mean censored path (:450) */
  double* fcstShadowYhat;       /* N x H x V mean uncensored (shadow-rate) path */
  double* PAImean;              /* K x N x V (:376) */
  double* PAIstdev;             /* K x N x V std(., 1) (:377) */
  double* shadowrate_all;       /* MCMCdraws x Ns x elbTmax x nchains x V kept shadow rates */
  int* countELBaccept;          /* V (countAccept + countAcceptBurnin over the vintage's chains) */
  int* attempts;                /* V: runs used (> max_retries + 1: failed, outputs NaN) */
  /* postprocess != 0 (goVARshadowrateBlockHybrid.m:349-480) */
  double* fcstYmedian;          /* N x H x V */
  double* fcstYcrps;            /* N x H x V */
  double* fcstYquantiles;       /* N x H x nq x V */
  double* fcstYcummedian;       /* N x H x V (cumcode applied to paths and yrealized) */
  double* fcstYcumcrps;         /* N x H x V */
  double* fcstYcumquantiles;    /* N x H x nq x V */
  double* fcstShadowYmedian;    /* Ny x H x V (rows ndxYields) */
  double* fcstShadowYquantiles; /* Ny x H x nq x V */
  double* PAImedian;            /* K x N x V */
  double* PAIquantiles;         /* K x N x nq x V */
  double* scoreDraws;           /* (fcstNdraws * nchains) x 4 x V, order (Nd, kept draw, chain) */
  double* shadowratePSRF;       /* Ns x V (shadow-rate models): ccmm_shadowrate_psrf of the vintage's kept
                                   shadow rates (goVARshadowrateBlockHybrid.m:322-325; the reference's
                                   one-chain statistic, averaged over the vintage's chains) */
  double* shadowratePSRFchains; /* Ns x V: ccmm_shadowrate_psrf_chains (psrf across the vintage's chains;
                                   NaN for one chain) -- not in the reference's output */
} ccmm_batch_out;

int ccmm_run_batch(ccmm_ctx* ctx, const ccmm_batch_config* cfg, int V, const ccmm_vintage* vintages,
                   ccmm_batch_out* out);

/* ------------------------------------------------------------ GIRF
 * Generalized impulse responses by antithetic simulation, batched over M MCMC draws
 * (generateGIRF2linear.m / generateGIRF2blockhybrid.m:199-259 with antitheticSim and
 * simVAR / simVARshadowrateBlockHybrid): per draw, nsim shock paths (SV paths
 * exp(cumsum(sqrtPHI randn)/2)) x 4 antithetic sets (+-z .* SV^{+-1} .* SV0) x 3 scenarios
 * (shock11 = 0, +shock11, -shock11 added to variable 1 at horizon 1), mapped by invA and
 * simulated over H horizons (bh != 0: actual-rate states max(shadow, ELB), yields floored at
 * the ELB in the output), cumcode variables cumsum / np, averaged over the 4 nsim paths.
 *   PAI K x N x M, invA N x N x M, sqrtPHI N x N x M (chol(PHI, 'lower')), SV0 N x M (jump-off
 *   sqrtht), Xjumpoff (K + Ny p) x M (linear: K), actual / ndxYields N bytes (bh), cumcode N
 *   bytes or NULL; z, svz N x H x nsim x M (randn(N, H, nsim), randn(N, H*nsim)) or both NULL
 *   (Philox keyed by (seed, draw)).
 *   yhat out N x H x 3 x M: fcstYHATdraws, fcstYHATdraws1plus, fcstYHATdraws1minus.
 * N <= 32. */
int ccmm_girf(ccmm_ctx* ctx, int M, int N, int p, int H, int nsim, const double* PAI, const double* invA,
              const double* sqrtPHI, const double* SV0, const double* Xjumpoff, int bh, const uint8_t* actual,
              const uint8_t* ndxYields, double elb, const uint8_t* cumcode, double np_, double shock11,
              const double* z, const double* svz, uint64_t seed, double* yhat);

/* generateGIRF2hybrid.m:176-259 (simVARhybrid, :361-386): the hybrid model's GIRFs.  The state
 * holds [1, p lags of y, p lags of the Ns actual (shadow-rate) variables]; the companion rows are
 * the full hybrid PAI (:226-227: fcstA(ndxfcstY,:) = PAIdraws), the actual-rate states are
 * max(shadow, ELB) (:373-375) and the output floors ndxYields (:378-381).
 *   PAI (K + Ns p) x N x M (K = N p + 1), Xjumpoff (K + Ns p) x M, ndxShadow / ndxYields N bytes;
 *   the rest as ccmm_girf. */
int ccmm_girf_hybrid(ccmm_ctx* ctx, int M, int N, int p, int H, int nsim, const double* PAI, const double* invA,
                     const double* sqrtPHI, const double* SV0, const double* Xjumpoff, const uint8_t* ndxShadow,
                     const uint8_t* ndxYields, double elb, const uint8_t* cumcode, double np_, double shock11,
                     const double* z, const double* svz, uint64_t seed, double* yhat);

/* ------------------------------------------------------------ diagnostics */

/* psrf(X) of DiagnosticsShadowrate.m:34-128 (== Diagnostics.m:28; Brooks & Gelman 1998, square-root
 * form): X n x D x M, M sequences of n draws of D variables; M == 1 splits the one chain into its
 * first and last floor(n/3) draws (:82-91).  R out: D.  Host computation.  CCMM_ERR_ARG "Too few
 * samples" as :103-105 when a sequence would be empty. */
int ccmm_psrf(int n, int D, int M, const double* X, double* R);

/* shadowratePSRF(:, vintage) of goVARshadowrateBlockHybrid.m:322-325 (goVARhybrid.m:322-323,
 * goVARshadowrate.m:332-333): for each shadow rate s, DiagnosticsShadowrate(shadowrate_all(:, s,
 * ELBdummy(startELB:thisT, s))) = the mean of psrf over the rate's censored months (NaN when there
 * are none).  draws M x Ns x ldT x C (the kept shadow rates of C chains; the first elbT months are
 * the vintage's window), mask Ns x elbT (ELBdummy(startELB:thisT, :)', = elb.sNaN).  The reference's
 * one-chain statistic (first / last thirds, :82-91) for every chain, averaged over the C chains, so the
 * value keeps the reference's meaning for any C.  out: Ns (NaN where psrf would stop with 'Too few
 * samples': M < 3).  The
 * reference's DiagnosticsShadowrate also evaluates ineff() (momentg), which errors below 100 draws
 * (Diagnostics.m momentg 'needs a larger number of ndraws'); its result is not an output and the
 * check is not reproduced. */
int ccmm_shadowrate_psrf(int M, int Ns, int elbT, int ldT, int C, const double* draws, const uint8_t* mask,
                         double* out);
/* The multi-chain form (no reference counterpart; parity unpinned beyond the psrf formula): per cell,
 * psrf over the C chains as its M-draw sequences (Brooks-Gelman across chains), averaged over the rate's
 * months at the ELB as ccmm_shadowrate_psrf.  out: Ns, NaN when C < 2 or M < 2. */
int ccmm_shadowrate_psrf_chains(int M, int Ns, int elbT, int ldT, int C, const double* draws, const uint8_t* mask,
                                double* out);

/* Predictive density of one kept draw per chain, batched over B chains.
 * Replaces the doPredictiveDensity block mcmcVAR.m:298-381 (same simulation in
 * mcmcVARshadowrateBlockHybrid.m:550-669), including logscoreGaussian.m:15-20 and
 * logscoreGaussianCensored.m:13-88.  Companion form with K = N*p + 1
 * (mcmcVAR.m:108-115).
 *   PAI K x N x B, invA N x N x B, logSV0 N x B (= Vol_states(end,:)', log
 *   variances), sqrtPHI N x N x B, Xjumpoff K x B, yrealized N (first column),
 *   ndxYields N (1 = yield, censored at elb), svz N x (H*Nd) x B (mcmcVAR.m:302)
 *   and z N x H x Nd x B (:306) or both NULL (Philox, block CCMM_RNG_FCST,
 *   counter sweep = `sweep`).
 * Outputs: fcstY, fcstYcensor N x H x Nd x B (fcstYdraws / fcstYcensorDraws),
 *   yhat N x H x B (yhatdraws), scores 4 x Nd x B = (fcstLogscoreDraws,
 *   fcstLogscoreELBdraws, fcstLogscoreXdraws, fcstLogscoreIdraws).
 * Returns CCMM_WARN_MVNCDF when some censored score needed mvncdf in more than 12
 * dimensions (that score is NaN; status[c] bit 1 marks the chain). */
int ccmm_fcst(ccmm_ctx* ctx, int B, int N, int p, int H, int Nd, const double* PAI,
              const double* invA, const double* logSV0, const double* sqrtPHI,
              const double* Xjumpoff, const double* yrealized, const uint8_t* ndxYields,
              double elb, const double* svz, const double* z, uint64_t seed, int sweep,
              double* fcstY, double* fcstYcensor, double* yhat, double* scores, int* status);

/* D16x16 = A16x4 * B4x16 computed by one v_mfma_f64_16x16x4_f64 with the operand
 * and accumulator lane maps the CTA SYRK kernel relies on (all column-major). */
int ccmm_selftest_mfma_f64(ccmm_ctx* ctx, const double* A16x4, const double* B4x16, double* D16x16);
/* nprobe independent D = C + A B (one v_mfma_f64_16x16x4_f64 each, caller-given accumulator),
 * probe q at A16x4 + 64 q, B4x16 + 64 q, C16x16 / D16x16 + 256 q: measures the instruction's
 * internal summation order and rounding points (tools/probe_mfma_order.py). */
int ccmm_selftest_mfma_f64_acc(ccmm_ctx* ctx, int nprobe, const double* A16x4, const double* B4x16,
                               const double* C16x16, double* D16x16);

#ifdef __cplusplus
}
#endif
#endif /* CCMM_H */
