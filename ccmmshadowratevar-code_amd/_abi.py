"""ctypes binding of libccmm (include/ccmm.h).

The product path: every numerical call goes through ``libccmm.so`` (HIP,
gfx950).  There is no CPU fallback: if the library cannot be loaded, or no GPU
is visible when a compute entry point is called, a ``RuntimeError`` is raised.

All array arguments follow the reference's MATLAB shapes; they are passed to
the C ABI column-major (``order='F'``), chain index slowest.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("CCMM_LIB", _HERE / "csrc" / "libccmm.so"))

ABI_VERSION = 4  # include/ccmm.h CCMM_ABI_VERSION this binding's structures follow
CCMM_OK = 0
CCMM_ERR_NOTSPD = -4
STATUS_INFO = 1 | 64  # informational status bits: QR fallback used, PS precision fell back to Gibbs
MODEL_LINEAR = 0
MODEL_BLOCKHYBRID = 1
MODEL_HYBRID = 2  # mcmcVARhybridGibbs.m: K = N*p + 1 + Ns*p
MODEL_SHADOWRATE = 3  # mcmcVARshadowrate.m: shadow-rate design for all equations, linear forecasts

RNG_PAI, RNG_A, RNG_SVU, RNG_SVZ, RNG_PHI, RNG_ELB, RNG_FCST, RNG_PS = 1, 2, 3, 4, 5, 6, 7, 8
CCMM_WARN_MVNCDF = 3

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_i8p = C.POINTER(C.c_int8)
_u8p = C.POINTER(C.c_uint8)
_i64p = C.POINTER(C.c_int64)


class ChainConfig(C.Structure):
    _fields_ = [("model", C.c_int), ("N", C.c_int), ("p", C.c_int), ("K", C.c_int),
                ("T", C.c_int), ("B", C.c_int), ("ndata", C.c_int), ("dPHI", C.c_int),
                ("rng_crn", C.c_int), ("store_capacity", C.c_int),
                ("logy2offset", C.c_double), ("seed", C.c_uint64),
                ("Ns", C.c_int), ("elbTmax", C.c_int), ("elb_gibbsburn", C.c_int),
                ("elb", C.c_double)]


class Vintage(C.Structure):
    """ccmm_vintage (include/ccmm.h)."""
    _fields_ = [("T", C.c_int), ("Y", _dp), ("X", _dp), ("iVdiag", _dp), ("iVb", _dp), ("sPHI", _dp),
                ("h0mean", _dp), ("h0vcvsqrt", _dp), ("PAI0", _dp), ("sqrtht0", _dp), ("h0init", _dp), ("elbT0", C.c_int),
                ("sNaN", _u8p), ("yrealized", _dp), ("unit", C.c_uint32)]


class BatchConfig(C.Structure):
    """ccmm_batch_config (include/ccmm.h)."""
    _fields_ = [("model", C.c_int), ("N", C.c_int), ("p", C.c_int), ("Ns", C.c_int), ("ndxS", _ip),
                ("actual_block", _u8p), ("ndxYields", _u8p), ("nchains", C.c_int), ("MCMCdraws", C.c_int),
                ("burnin", C.c_int), ("gibbsburn", C.c_int), ("Nproposals", C.c_int), ("fcstNdraws", C.c_int),
                ("H", C.c_int), ("elb", C.c_double), ("seed", C.c_uint64), ("chunk", C.c_int),
                ("max_retries", C.c_int), ("postprocess", C.c_int), ("nq", C.c_int), ("pct", _dp),
                ("cumcode", _u8p)]


BATCH_OUT_FIELDS = ("logscore", "fcstYhat", "fcstShadowYhat", "PAImean", "PAIstdev", "shadowrate_all",
                    "countELBaccept", "attempts", "fcstYmedian", "fcstYcrps", "fcstYquantiles", "fcstYcummedian",
                    "fcstYcumcrps", "fcstYcumquantiles", "fcstShadowYmedian", "fcstShadowYquantiles", "PAImedian",
                    "PAIquantiles", "scoreDraws", "shadowratePSRF", "shadowratePSRFchains")


class BatchOut(C.Structure):
    """ccmm_batch_out (include/ccmm.h)."""
    _fields_ = [(nm, _ip if nm in ("countELBaccept", "attempts") else _dp) for nm in BATCH_OUT_FIELDS]


_SIGS = {
    "ccmm_abi_version": (C.c_int, []),
    "ccmm_last_error": (C.c_char_p, []),
    "ccmm_ablation_build": (C.c_int, []),
    "ccmm_env_ignored": (C.c_int, [C.c_char_p, C.c_int]),
    "ccmm_option_count": (C.c_int, []),
    "ccmm_option_name": (C.c_char_p, [C.c_int]),
    "ccmm_option_default": (C.c_int, [C.c_char_p, _ip]),
    "ccmm_set_option": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    "ccmm_get_option": (C.c_int, [C.c_void_p, C.c_char_p, _ip]),
    "ccmm_chains_set_option": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    "ccmm_chains_get_option": (C.c_int, [C.c_void_p, C.c_char_p, _ip]),
    "ccmm_device_count": (C.c_int, []),
    "ccmm_create": (C.c_void_p, [C.c_int]),
    "ccmm_destroy": (None, [C.c_void_p]),
    "ccmm_synchronize": (C.c_int, [C.c_void_p]),
    "ccmm_cta": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp, C.c_int, _dp,
                           C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _ip]),
    "ccmm_cta_aswitching": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp, C.c_int, _dp,
                                      C.c_int, C.c_int, _dp, _dp, _u8p, _dp, _dp, _dp, _dp, _dp, _ip]),
    "ccmm_astep": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp]),
    "ccmm_sv_ksc": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp, _dp,
                              _dp, _dp, _dp, _dp, _i8p]),
    "ccmm_phi_iw": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, _dp, _dp, C.c_int, _dp, _dp,
                              _dp]),
    "ccmm_draw_trunc_normal": (C.c_double, [C.c_double, C.c_double, C.c_double, C.c_double, _u8p]),
    "ccmm_draw_trunc_normal_batch": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp, C.c_double, _dp,
                                               _dp, _u8p]),
    "ccmm_chains_create": (C.c_void_p, [C.c_void_p, C.POINTER(ChainConfig)]),
    "ccmm_chains_destroy": (None, [C.c_void_p]),
    "ccmm_chains_set_data": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp, _dp,
                                       _dp]),
    "ccmm_chains_set_slots": (C.c_int, [C.c_void_p, _ip]),
    "ccmm_chains_set_state": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp]),
    "ccmm_chains_get_state": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
    "ccmm_chains_crn_len": (C.c_int64, [C.c_void_p]),
    "ccmm_chains_sweep": (C.c_int, [C.c_void_p, C.c_int, _dp, C.c_int]),
    "ccmm_chains_stored": (C.c_int, [C.c_void_p]),
    "ccmm_chains_get_draws": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp]),
    "ccmm_chains_set_rng_ids": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "ccmm_chains_set_mfma_lock": (C.c_int, [C.c_void_p, C.c_int]),
    "ccmm_chains_get_kai": (C.c_int, [C.c_void_p, _i8p]),
    "ccmm_chains_record_elb_flags": (C.c_int, [C.c_void_p, C.c_int]),
    "ccmm_chains_get_elb_flags": (C.c_int, [C.c_void_p, _u8p]),
    "ccmm_gibbs_shadowrates": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_uint8), C.POINTER(C.c_uint8), _dp, _dp, _dp,
                                         _dp, _dp, _dp, C.c_double, C.c_int, C.c_int, _dp, _dp,
                                         C.POINTER(C.c_uint8)]),
    "ccmm_gibbs_shadowrates_b3": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.POINTER(C.c_uint8), C.POINTER(C.c_uint8), _dp, _dp, _dp, _dp,
                                            C.c_int, _dp, C.c_double, C.c_int, C.c_int, _dp, _dp,
                                            C.POINTER(C.c_uint8)]),
    "ccmm_chains_get_status": (C.c_int, [C.c_void_p, _ip]),
    "ccmm_chains_set_fcst": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _u8p, C.c_int]),
    "ccmm_chains_set_fcst_slot": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "ccmm_chains_fcst_stored": (C.c_int, [C.c_void_p]),
    "ccmm_chains_set_fcst_censor": (C.c_int, [C.c_void_p, _u8p]),
    "ccmm_chains_get_fcst": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp, _dp]),
    "ccmm_chains_set_elb_model": (C.c_int, [C.c_void_p, _ip, _u8p]),
    "ccmm_chains_set_elb_slot": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _u8p]),
    "ccmm_chains_get_shadowrate": (C.c_int, [C.c_void_p, _dp]),
    "ccmm_chains_get_cta_gram": (C.c_int, [C.c_void_p, _dp]),
    "ccmm_chains_get_cta_factor": (C.c_int, [C.c_void_p, _dp]),
    "ccmm_chains_set_elb_ps": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "ccmm_draw_summaries": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dp, _dp, C.c_int, _dp, _dp, _dp,
                                      _dp, _dp, _dp]),
    "ccmm_girf_hybrid": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp,
                                   _dp, _u8p, _u8p, C.c_double, _u8p, C.c_double, C.c_double, _dp, _dp,
                                   C.c_uint64, _dp]),
    "ccmm_girf": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp,
                            _dp, C.c_int, _u8p, _u8p, C.c_double, _u8p, C.c_double, C.c_double, _dp,
                            _dp, C.c_uint64, _dp]),
    "ccmm_chains_summaries": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _u8p, _u8p, _dp, C.c_int, _dp,
                                        _dp, _dp, _dp, _dp, _dp]),
    "ccmm_chains_summaries_floor": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _u8p, _u8p, _u8p, C.c_double, _dp,
                                              C.c_int, _dp, _dp, _dp, _dp, _dp, _dp]),
    "ccmm_chains_get_ps": (C.c_int, [C.c_void_p, _ip, _ip, _ip]),
    "ccmm_chains_get_ps_mean": (C.c_int, [C.c_void_p, _dp]),
    "ccmm_chains_keep_missingrate": (C.c_int, [C.c_void_p, C.c_int]),
    "ccmm_chains_get_missingrate": (C.c_int, [C.c_void_p, _dp]),
    "ccmm_chains_get_xy": (C.c_int, [C.c_void_p, _dp, _dp]),
    "ccmm_chains_profile": (C.c_int, [C.c_void_p, C.c_int]),
    "ccmm_chains_pai_moments": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp]),
    "ccmm_chains_kernel_times": (C.c_int, [C.c_void_p, C.c_int, _dp, _i64p, C.c_char_p, C.c_int]),
    "ccmm_fcst": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp,
                            _dp, _dp, _dp, _dp, _u8p, C.c_double, _dp, _dp, C.c_uint64,
                            C.c_int, _dp, _dp, _dp, _dp, _ip]),
    "ccmm_run_batch": (C.c_int, [C.c_void_p, C.POINTER(BatchConfig), C.c_int, C.POINTER(Vintage),
                                 C.POINTER(BatchOut)]),
    "ccmm_psrf": (C.c_int, [C.c_int, C.c_int, C.c_int, _dp, _dp]),
    "ccmm_shadowrate_psrf": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _u8p, _dp]),
    "ccmm_shadowrate_psrf_chains": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _u8p, _dp]),
    "ccmm_selftest_mfma_f64": (C.c_int, [C.c_void_p, _dp, _dp, _dp]),
    "ccmm_selftest_mfma_f64_acc": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp, _dp, _dp]),
}

_lib = None


def load_library(path: str | os.PathLike | None = None):
    """Load libccmm.so and bind every exported symbol; raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise RuntimeError(f"libccmm.so not found at {p}: build it with "
                           f"`python -c 'import __graft_entry__ as g; g.build()'` "
                           f"(there is no CPU fallback)")
    lib = C.CDLL(str(p))
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.ccmm_abi_version()
    if v != ABI_VERSION:  # the ctypes structures (ChainConfig, BatchConfig, BatchOut) follow one header
        raise RuntimeError(f"{p}: ABI version {v}, this binding expects {ABI_VERSION}; rebuild the library")
    if path is None:
        _lib = lib
    return lib


def exported_symbols():
    return list(_SIGS)


def last_error() -> str:
    return load_library().ccmm_last_error().decode(errors="replace")


def env_ignored() -> tuple[int, list[str]]:
    """Timing-only ablation variables set in the environment that this build ignores
    (ccmm_env_ignored; host only, no GPU needed)."""
    buf = C.create_string_buffer(1024)
    n = load_library().ccmm_env_ignored(buf, len(buf))
    names = buf.value.decode()
    return n, (names.split(",") if names else [])


def ablation_build() -> bool:
    return bool(load_library().ccmm_ablation_build())


def option_names() -> list[str]:
    """Names of the kernel options (ccmm_set_option; host only, no GPU needed)."""
    lib = load_library()
    return [lib.ccmm_option_name(i).decode() for i in range(lib.ccmm_option_count())]


def option_default(name: str) -> int:
    """ccmm_option_default: the value a new context starts from (host only)."""
    v = C.c_int(0)
    _check(load_library().ccmm_option_default(name.encode(), C.byref(v)), f"ccmm_option_default({name})")
    return int(v.value)


def _check(rc, what):
    if rc < 0:
        raise RuntimeError(f"{what} failed (rc={rc}): {last_error()}")
    return rc


def _f(a, dtype=np.float64):
    """Column-major contiguous copy (MATLAB layout)."""
    return np.asfortranarray(np.asarray(a, dtype=dtype))


def _ptr(a, ct=_dp):
    if a is None:
        return None
    return a.ctypes.data_as(ct)


def psrf(X):
    """ccmm_psrf: psrf(X) of DiagnosticsShadowrate.m:34-128; X n x D (one chain, split into thirds)
    or n x D x M.  Returns R (D,).  Host computation inside libccmm (no GPU needed)."""
    X = _f(X)
    if X.ndim == 1:
        X = X[:, None]
    n, D = X.shape[:2]
    M = X.shape[2] if X.ndim == 3 else 1
    R = np.zeros(D)
    _check(load_library().ccmm_psrf(n, D, M, _ptr(X), _ptr(R)), "ccmm_psrf")
    return R


def shadowrate_psrf(draws, mask, elbT=None, chains=False):
    """ccmm_shadowrate_psrf: shadowratePSRF(:, vintage) of goVARshadowrateBlockHybrid.m:322-325 (the
    reference's one-chain statistic, averaged over C chains); chains=True: ccmm_shadowrate_psrf_chains
    (psrf across the C chains).  draws M x Ns x ldT [x C] kept shadow rates, mask Ns x elbT
    (ELBdummy(startELB:thisT, :)').  Returns Ns values."""
    d = _f(draws)
    M, Ns, ldT = d.shape[:3]
    Cc = d.shape[3] if d.ndim == 4 else 1
    mk = np.asfortranarray(np.asarray(mask, bool).reshape(Ns, -1), dtype=np.uint8)
    eT = mk.shape[1] if elbT is None else int(elbT)
    out = np.zeros(Ns)
    lib = load_library()
    fn = lib.ccmm_shadowrate_psrf_chains if chains else lib.ccmm_shadowrate_psrf
    _check(fn(M, Ns, eT, ldT, Cc, _ptr(d), _ptr(mk, _u8p), _ptr(out)), "ccmm_shadowrate_psrf")
    return out


class Context:
    """A libccmm context bound to one HIP device (ccmm_create)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        n = self.lib.ccmm_device_count()
        if n <= 0:
            raise RuntimeError("no HIP device visible: libccmm requires an MI355X (gfx950) GPU")
        h = self.lib.ccmm_create(device)
        if not h:
            raise RuntimeError(f"ccmm_create({device}) failed: {last_error()}")
        self.handle = h
        self.device = device

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ccmm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        _check(self.lib.ccmm_synchronize(self.handle), "ccmm_synchronize")

    def set_option(self, name: str, value: int):
        """ccmm_set_option: a kernel form / schedule for the block-level calls and the chain sets
        created on this context afterwards."""
        _check(self.lib.ccmm_set_option(self.handle, name.encode(), int(value)), f"ccmm_set_option({name})")

    def get_option(self, name: str) -> int:
        v = C.c_int(0)
        _check(self.lib.ccmm_get_option(self.handle, name.encode(), C.byref(v)), f"ccmm_get_option({name})")
        return int(v.value)

    def options(self, **opts):
        """Context manager: set options for the block, restore the previous values after."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_option(k) for k in opts}
            try:
                for k, v in opts.items():
                    self.set_option(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_option(k, v)
        return cm()

    # ------------------------------------------------------------ block-level
    def cta(self, Y, X, A, sqrtht, iVdiag, iVb, PAI, z=None, y_per_chain=False, x_per_chain=False):
        """Batched CTA/CTAsys draw.  Shapes (MATLAB): Y T x N [x B], X T x K [x nx] [x B],
        A N x N x B, sqrtht T x N x B, iVdiag/iVb K x N, PAI K x N x B, z K x N x B."""
        A = _f(A)
        N = A.shape[0]
        B = A.shape[2] if A.ndim == 3 else 1
        PAI = _f(PAI).copy(order="F")
        K = PAI.shape[0]
        T = np.asarray(Y).shape[0]
        Xf = _f(X)
        if x_per_chain:
            nx = Xf.shape[2] if Xf.ndim == 4 else 1
        else:
            nx = Xf.shape[2] if Xf.ndim == 3 else 1
        status = np.zeros(B, dtype=np.int32)
        rc = self.lib.ccmm_cta(self.handle, B, T, N, K, _ptr(_f(Y)), int(y_per_chain), _ptr(Xf), nx,
                               int(x_per_chain), _ptr(A), _ptr(_f(sqrtht)), _ptr(_f(iVdiag)),
                               _ptr(_f(iVb)), _ptr(PAI), _ptr(_f(z)) if z is not None else None,
                               status.ctypes.data_as(_ip))
        _check(rc, "ccmm_cta")
        return PAI, status

    def cta_aswitching(self, Y, X, A, Aelb, atELB, sqrtht, iVdiag, iVb, PAI, z=None, y_per_chain=False,
                       x_per_chain=False):
        """Batched CTAsysAswitching draw: as ``cta`` plus Aelb N x N x B and atELB (T bools,
        shared by the chains): the months at the ELB use Aelb (CTAsysAswitching.m:61-80)."""
        A = _f(A)
        N = A.shape[0]
        B = A.shape[2] if A.ndim == 3 else 1
        PAI = _f(PAI).copy(order="F")
        K = PAI.shape[0]
        T = np.asarray(Y).shape[0]
        Xf = _f(X)
        if x_per_chain:
            nx = Xf.shape[2] if Xf.ndim == 4 else 1
        else:
            nx = Xf.shape[2] if Xf.ndim == 3 else 1
        at = np.ascontiguousarray(np.asarray(atELB, bool).ravel(), dtype=np.uint8)
        assert at.size == T, "atELB must hold T entries"
        status = np.zeros(B, dtype=np.int32)
        rc = self.lib.ccmm_cta_aswitching(self.handle, B, T, N, K, _ptr(_f(Y)), int(y_per_chain), _ptr(Xf), nx,
                                          int(x_per_chain), _ptr(A), _ptr(_f(Aelb)), at.ctypes.data_as(_u8p),
                                          _ptr(_f(sqrtht)), _ptr(_f(iVdiag)), _ptr(_f(iVb)), _ptr(PAI),
                                          _ptr(_f(z)) if z is not None else None, status.ctypes.data_as(_ip))
        _check(rc, "ccmm_cta_aswitching")
        return PAI, status

    def astep(self, RESID, sqrtht, z=None):
        RESID = _f(RESID)
        T, N = RESID.shape[:2]
        B = RESID.shape[2] if RESID.ndim == 3 else 1
        A = np.zeros((N, N, B), order="F")
        invA = np.zeros((N, N, B), order="F")
        rc = self.lib.ccmm_astep(self.handle, B, T, N, _ptr(RESID), _ptr(_f(sqrtht)),
                                 _ptr(_f(z)) if z is not None else None, _ptr(A), _ptr(invA))
        _check(rc, "ccmm_astep")
        return A, invA

    def sv_ksc(self, logy2T, hprevT, sqrtPHI, h0mean, h0vcvsqrt, u=None, z=None):
        logy2T = _f(logy2T)
        N, T = logy2T.shape[:2]
        B = logy2T.shape[2] if logy2T.ndim == 3 else 1
        hT = np.zeros((N, T, B), order="F")
        sh = np.zeros((N, T, B), order="F")
        h0 = np.zeros((N, B), order="F")
        kai = np.zeros((N, T, B), dtype=np.int8, order="F")
        rc = self.lib.ccmm_sv_ksc(self.handle, B, T, N, _ptr(logy2T), _ptr(_f(hprevT)),
                                  _ptr(_f(sqrtPHI)), _ptr(_f(h0mean)), _ptr(_f(h0vcvsqrt)),
                                  _ptr(_f(u)) if u is not None else None,
                                  _ptr(_f(z)) if z is not None else None,
                                  _ptr(hT), _ptr(h0), _ptr(sh), kai.ctypes.data_as(_i8p))
        _check(rc, "ccmm_sv_ksc")
        return hT, h0, sh, kai

    def gibbs_shadowrates(self, Y, STATE0, YHAT0, ndxS, sNaN, p, C, Psi, SVol, elbBound,
                          burnin=100, u=None, Ndraws=1, flags=False):
        """gibbsdrawShadowrates (ccmm_gibbs_shadowrates), batched over a trailing chain axis.

        Y Ny x elbT [x B], STATE0 K [x B], YHAT0 Ny x elbT [x B] or None, ndxS bool Ny,
        sNaN bool Ns x elbT, C K x K [x B], Psi K x Ny [x B], SVol Ny x elbT [x B],
        u Ns x elbT x (burnin + Ndraws) [x B] or None.  Returns draws Ns x elbT x Ndraws x B
        (and the drawTruncNormal branch flags Ns x elbT x passes x B when flags=True)."""
        Y = _f(Y)
        Ny, T = Y.shape[:2]
        B = Y.shape[2] if Y.ndim == 3 else 1
        nd = np.ascontiguousarray(np.asarray(ndxS, dtype=bool), dtype=np.uint8)
        sN = np.asfortranarray(np.asarray(sNaN, dtype=bool).astype(np.uint8))
        Ns = int(sN.shape[0])
        passes = burnin + Ndraws
        out = np.zeros((Ns, T, Ndraws, B), order="F")
        fl = np.zeros((Ns, T, passes, B), dtype=np.uint8, order="F") if flags else None
        rc = self.lib.ccmm_gibbs_shadowrates(
            self.handle, B, Ny, T, Ns, int(p), _ptr(nd, _u8p), _ptr(sN, _u8p), _ptr(Y),
            _ptr(_f(STATE0)), _ptr(_f(YHAT0)) if YHAT0 is not None else None, _ptr(_f(C)),
            _ptr(_f(Psi)), _ptr(_f(SVol)), float(elbBound), int(Ndraws), int(burnin),
            _ptr(_f(u)) if u is not None else None, _ptr(out), _ptr(fl, _u8p) if flags else None)
        _check(rc, "ccmm_gibbs_shadowrates")
        return (out, fl) if flags else out

    def gibbs_shadowrates_b3(self, Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, elbBound, burnin=100, u=None,
                             Ndraws=1, flags=False, month_varying=None):
        """gibbsdrawShadowratesB3 (ccmm_gibbs_shadowrates_b3), batched over a trailing chain axis.

        Y Ny x elbT [x B], STATE0 K [x B], ndxS bool Ny, sNaN bool Ns x elbT, A K x K [x B],
        Bm K x Ny [x B] or, with month_varying (default: Bm.ndim == 4, or 3 with B == 1 and the
        last axis elbT), K x Ny x elbT [x B]; SVol Ny x elbT [x B]; u Ns x elbT x passes [x B] or None."""
        Y = _f(Y)
        Ny, T = Y.shape[:2]
        B = Y.shape[2] if Y.ndim == 3 else 1
        Bm = np.asarray(Bm, float)
        if month_varying is None:
            month_varying = Bm.ndim == 4 or (Bm.ndim == 3 and B == 1 and Bm.shape[2] == T)
        nd = np.ascontiguousarray(np.asarray(ndxS, dtype=bool), dtype=np.uint8)
        sN = np.asfortranarray(np.asarray(sNaN, dtype=bool).astype(np.uint8))
        Ns = int(sN.shape[0])
        passes = burnin + Ndraws
        out = np.zeros((Ns, T, Ndraws, B), order="F")
        fl = np.zeros((Ns, T, passes, B), dtype=np.uint8, order="F") if flags else None
        rc = self.lib.ccmm_gibbs_shadowrates_b3(
            self.handle, B, Ny, T, Ns, int(p), _ptr(nd, _u8p), _ptr(sN, _u8p), _ptr(Y), _ptr(_f(STATE0)),
            _ptr(_f(A)), _ptr(_f(Bm)), int(bool(month_varying)), _ptr(_f(SVol)), float(elbBound), int(Ndraws),
            int(burnin), _ptr(_f(u)) if u is not None else None, _ptr(out), _ptr(fl, _u8p) if flags else None)
        _check(rc, "ccmm_gibbs_shadowrates_b3")
        return (out, fl) if flags else out

    def phi_iw(self, eta, sPHI, dPHI, Zdraw=None):
        eta = _f(eta)
        T, N = eta.shape[:2]
        B = eta.shape[2] if eta.ndim == 3 else 1
        sq = np.zeros((N, N, B), order="F")
        PHI = np.zeros((N, N, B), order="F")
        rc = self.lib.ccmm_phi_iw(self.handle, B, T, N, _ptr(eta), _ptr(_f(sPHI)), int(dPHI),
                                  _ptr(_f(Zdraw)) if Zdraw is not None else None, _ptr(sq),
                                  _ptr(PHI))
        _check(rc, "ccmm_phi_iw")
        return sq, PHI

    def fcst(self, PAI, invA, logSV0, sqrtPHI, Xjumpoff, yrealized, ndxYields, ELBbound,
             fcstNhorizons, Ndraws, svz=None, z=None, seed=0, sweep=0):
        """Predictive density of one kept draw per chain (mcmcVAR.m:298-381).

        PAI K x N [x B], invA N x N [x B], logSV0 N [x B], sqrtPHI N x N [x B],
        Xjumpoff K [x B], yrealized N, ndxYields bool N.  CRN: svz N x (H*Nd) [x B]
        (mcmcVAR.m:302), z N x H x Nd [x B] (:306); None = Philox.
        Returns fcstY, fcstYcensor (N x H x Nd x B), yhat (N x H x B),
        scores (4 x Nd x B: logscore, ELB logscore, X logscore, I logscore), status (B).
        """
        PAI = _f(PAI)
        K, N = PAI.shape[:2]
        B = PAI.shape[2] if PAI.ndim == 3 else 1
        p = (K - 1) // N
        if K != N * p + 1:
            raise ValueError("ccmm_fcst: K must equal N*p + 1 (mcmcVAR.m:108-115)")
        H, Nd = int(fcstNhorizons), int(Ndraws)
        fY = np.zeros((N, H, Nd, B), order="F")
        fYc = np.zeros((N, H, Nd, B), order="F")
        yhat = np.zeros((N, H, B), order="F")
        sc = np.zeros((4, Nd, B), order="F")
        st = np.zeros(B, dtype=np.int32)
        mask = np.ascontiguousarray(np.asarray(ndxYields, bool).astype(np.uint8))
        crn = svz is not None
        rc = self.lib.ccmm_fcst(self.handle, B, N, p, H, Nd, _ptr(PAI), _ptr(_f(invA)),
                                _ptr(_f(logSV0)), _ptr(_f(sqrtPHI)), _ptr(_f(Xjumpoff)),
                                _ptr(_f(yrealized)), _ptr(mask, _u8p), float(ELBbound),
                                _ptr(_f(svz)) if crn else None, _ptr(_f(z)) if crn else None,
                                int(seed), int(sweep), _ptr(fY), _ptr(fYc), _ptr(yhat),
                                _ptr(sc), _ptr(st, _ip))
        if rc != CCMM_WARN_MVNCDF:
            _check(rc, "ccmm_fcst")
        return fY, fYc, yhat, sc, st

    def draw_trunc_normal_batch(self, mu, sig, elb, u):
        mu = _f(mu).ravel(order="F")
        n = mu.size
        out = np.zeros(n)
        fl = np.zeros(n, dtype=np.uint8)
        rc = self.lib.ccmm_draw_trunc_normal_batch(self.handle, n, _ptr(mu),
                                                   _ptr(_f(sig).ravel(order="F")), float(elb),
                                                   _ptr(_f(u).ravel(order="F")), _ptr(out),
                                                   fl.ctypes.data_as(_u8p))
        _check(rc, "ccmm_draw_trunc_normal_batch")
        return out, fl

    def draw_summaries(self, draws, realized=None, pct=()):
        """Per-series summaries of draws (n x S, each column one series): dict of mean,
        median, quantiles (S x nq), stdev (std(., 1)), crps (when realized, S, is given)."""
        X = _f(draws)
        n, S = X.shape
        pct = _f(np.asarray(pct, float).ravel())
        out = dict(mean=np.zeros(S), median=np.zeros(S), quantiles=np.zeros((S, pct.size), order="F"),
                   stdev=np.zeros(S))
        rz = None
        if realized is not None:
            rz = _f(np.asarray(realized, float).ravel())
            out["crps"] = np.zeros(S)
        _check(self.lib.ccmm_draw_summaries(self.handle, S, n, _ptr(X), _ptr(rz), pct.size,
                                            _ptr(pct) if pct.size else None, _ptr(out["mean"]),
                                            _ptr(out["median"]), _ptr(out["quantiles"]) if pct.size else None,
                                            _ptr(out["stdev"]), _ptr(out.get("crps"))),
               "ccmm_draw_summaries")
        return out

    def girf(self, PAI, invA, sqrtPHI, SV0, Xjumpoff, H, nsim, shock11, *, bh=False, actual=None,
             ndxYields=None, elb=0.25, cumcode=None, np_=12, z=None, svz=None, seed=1012023,
             hybrid=False, ndxShadow=None, p=None):
        """Generalized impulse responses (ccmm_girf): PAI K x N x M, invA / sqrtPHI N x N x M,
        SV0 N x M, Xjumpoff (K [+ Ny p]) x M; z, svz N x H x nsim x M or None (Philox).
        hybrid=True (ccmm_girf_hybrid, generateGIRF2hybrid): PAI (K + Ns p) x N x M with the
        lag order ``p``, ring = ndxShadow, output floored for ndxYields.
        Returns N x H x 3 x M (baseline, +shock, -shock mean paths)."""
        PAI = _f(PAI)
        Kx, N, M = PAI.shape
        u8 = lambda m: None if m is None else np.ascontiguousarray(np.asarray(m, bool), dtype=np.uint8)
        act, yl, cc = u8(actual), u8(ndxYields), u8(cumcode)
        out = np.zeros((N, int(H), 3, M), order="F")
        zz = None if z is None else _f(z)
        sz = None if svz is None else _f(svz)
        if hybrid:
            sh = u8(ndxShadow)
            p = int(p) if p is not None else (Kx - 1) // (N + int(sh.sum()))
            _check(self.lib.ccmm_girf_hybrid(self.handle, M, N, p, int(H), int(nsim), _ptr(PAI), _ptr(_f(invA)),
                                             _ptr(_f(sqrtPHI)), _ptr(_f(SV0)), _ptr(_f(Xjumpoff)),
                                             sh.ctypes.data_as(_u8p), yl.ctypes.data_as(_u8p), float(elb),
                                             None if cc is None else cc.ctypes.data_as(_u8p), float(np_),
                                             float(shock11), _ptr(zz), _ptr(sz), int(seed), _ptr(out)),
                   "ccmm_girf_hybrid")
            return out
        p = (Kx - 1) // N
        _check(self.lib.ccmm_girf(self.handle, M, N, p, int(H), int(nsim), _ptr(PAI), _ptr(_f(invA)),
                                  _ptr(_f(sqrtPHI)), _ptr(_f(SV0)), _ptr(_f(Xjumpoff)), int(bool(bh)),
                                  None if act is None else act.ctypes.data_as(_u8p),
                                  None if yl is None else yl.ctypes.data_as(_u8p), float(elb),
                                  None if cc is None else cc.ctypes.data_as(_u8p), float(np_), float(shock11),
                                  _ptr(zz), _ptr(sz), int(seed), _ptr(out)), "ccmm_girf")
        return out

    def run_batch(self, *, model, N, p, Ns, ndxS, actual_block, ndxYields, nchains, MCMCdraws, burnin,
                  gibbsburn, Nproposals, fcstNdraws, H, elb, seed, chunk, max_retries, postprocess, pct,
                  cumcode, vintages, want=None):
        """ccmm_run_batch: the vintage loop as one device-resident chain set.  ``vintages``: list of
        dicts with T, Y, X, iVdiag, iVb, sPHI, h0mean, h0vcvsqrt, PAI0, sqrtht0, h0init (optional),
        elbT0, sNaN, yrealized (N x H), unit.  Returns the ccmm_batch_out arrays (MATLAB shapes, vintage last);
        ``want``: names to fetch (default all that apply)."""
        V = len(vintages)
        shadow = model in (MODEL_BLOCKHYBRID, MODEL_HYBRID)
        K = N * p + 1 + (Ns * p if model == MODEL_HYBRID else 0)
        Ns_ = Ns if shadow else 0
        pct = _f(np.asarray(pct, float).ravel())
        nq = pct.size
        C_ = int(nchains)
        keep = []                                                  # host buffers alive across the call
        def arr(a, dt=np.float64):
            a = np.asfortranarray(np.asarray(a, dtype=dt))
            keep.append(a)
            return a
        vs = (Vintage * max(V, 1))()
        elbTall = 0
        for i, u in enumerate(vintages):
            T = int(u["T"])
            e0 = int(u.get("elbT0", T))
            if shadow:
                elbTall = max(elbTall, T - e0)
            sn = None
            if shadow and T > e0:
                sn = arr(np.asarray(u["sNaN"], bool), np.uint8).ctypes.data_as(_u8p)
            vs[i] = Vintage(T, _ptr(arr(u["Y"])), _ptr(arr(u["X"])), _ptr(arr(u["iVdiag"])), _ptr(arr(u["iVb"])),
                            _ptr(arr(u["sPHI"])), _ptr(arr(u["h0mean"])), _ptr(arr(u["h0vcvsqrt"])),
                            _ptr(arr(u["PAI0"])), _ptr(arr(u["sqrtht0"])),
                            _ptr(arr(u["h0init"])) if u.get("h0init") is not None else None, e0, sn,
                            _ptr(arr(u["yrealized"])),
                            int(u["unit"]))
        u8 = lambda a: None if a is None else arr(np.asarray(a, bool), np.uint8).ctypes.data_as(_u8p)
        nd = arr(np.asarray(ndxS if shadow else [0], np.int32), np.int32)
        cfg = BatchConfig(model, N, p, Ns_, nd.ctypes.data_as(_ip), u8(actual_block), u8(ndxYields), C_,
                          MCMCdraws, burnin, gibbsburn, Nproposals, fcstNdraws, H, elb, seed, chunk,
                          max_retries, int(bool(postprocess)), nq, _ptr(pct) if nq else None, u8(cumcode))
        Ny = int(np.count_nonzero(ndxYields))
        shapes = dict(logscore=(4, V), fcstYhat=(N, H, V), fcstShadowYhat=(N, H, V), PAImean=(K, N, V),
                      PAIstdev=(K, N, V), countELBaccept=(V,), attempts=(V,))
        if shadow:
            shapes["shadowrate_all"] = (MCMCdraws, Ns_, elbTall, C_, V)
            shapes["shadowratePSRF"] = (Ns_, V)
            shapes["shadowratePSRFchains"] = (Ns_, V)
        if postprocess:
            shapes.update(fcstYmedian=(N, H, V), fcstYcrps=(N, H, V), fcstYquantiles=(N, H, nq, V),
                          fcstYcummedian=(N, H, V), fcstYcumcrps=(N, H, V), fcstYcumquantiles=(N, H, nq, V),
                          fcstShadowYmedian=(Ny, H, V), fcstShadowYquantiles=(Ny, H, nq, V),
                          PAImedian=(K, N, V), PAIquantiles=(K, N, nq, V), scoreDraws=(fcstNdraws * C_, 4, V))
        out = {}
        for nm, shp in shapes.items():
            if want is not None and nm not in want and nm != "attempts":
                continue
            if nm in ("countELBaccept", "attempts"):
                out[nm] = np.zeros(shp, np.int32)
            else:
                out[nm] = np.zeros(shp, order="F")
        bo = BatchOut(*[None if nm not in out else
                        (out[nm].ctypes.data_as(_ip) if out[nm].dtype == np.int32 else _ptr(out[nm]))
                        for nm in BATCH_OUT_FIELDS])
        rc = self.lib.ccmm_run_batch(self.handle, C.byref(cfg), V, vs, C.byref(bo))
        if rc != CCMM_WARN_MVNCDF:
            _check(rc, "ccmm_run_batch")
        return out

    def selftest_mfma_f64(self, A16x4, B4x16):
        D = np.zeros((16, 16), order="F")
        _check(self.lib.ccmm_selftest_mfma_f64(self.handle, _ptr(_f(A16x4)), _ptr(_f(B4x16)),
                                               _ptr(D)), "ccmm_selftest_mfma_f64")
        return D

    def selftest_mfma_f64_acc(self, A, B, Cacc):
        """D = C + A B per probe: A 16 x 4 x P, B 4 x 16 x P, C 16 x 16 x P (one MFMA each)."""
        A, B, Cacc = _f(A), _f(B), _f(Cacc)
        P = A.shape[2]
        assert A.shape == (16, 4, P) and B.shape == (4, 16, P) and Cacc.shape == (16, 16, P)
        D = np.zeros((16, 16, P), order="F")
        _check(self.lib.ccmm_selftest_mfma_f64_acc(self.handle, P, _ptr(A), _ptr(B), _ptr(Cacc), _ptr(D)),
               "ccmm_selftest_mfma_f64_acc")
        return D


def draw_trunc_normal(mu, sig, elb, u):
    """Host scalar drawTruncNormal (drawTruncNormal.m:31-86); returns (draw, flags)."""
    fl = C.c_uint8(0)
    v = load_library().ccmm_draw_trunc_normal(float(mu), float(sig), float(elb), float(u),
                                              C.byref(fl))
    return v, int(fl.value)


class Chains:
    """Device-resident chain set (ccmm_chains_*): B chains of one model."""

    KERNELS = ("k_resid", "k_cta_weights", "k_cta_solve", "k_astep",
               "k_sv_mix", "k_sv_part", "k_phi_gen", "k_phi", "k_store", "k_gram_chol",
               "k_elb_prep", "k_elb_cond", "k_elb_gibbs", "k_elb_rebuild", "k_gram_chol_lag",
               "k_cta_solve_lag", "k_fcst", "k_gram_big", "k_chol_big", "k_cta_solve_big",
               "k_astep_big", "k_sv_big", "k_phi_big", "k_ps_chol", "k_ps_prop")

    def __init__(self, ctx: Context, *, N, p, T, B, ndata=1, model=MODEL_LINEAR, crn=False,
                 store_capacity=0, logy2offset=1e-3, seed=1012023, dPHI=None, Ns=0, elbTmax=0,
                 elb_gibbsburn=100, elb=0.25, options=None):
        self.ctx = ctx
        self.lib = ctx.lib
        K = N * p + 1 + (Ns * p if model == MODEL_HYBRID else 0)
        self.cfg = ChainConfig(model, N, p, K, T, B, ndata, N + 3 if dPHI is None else dPHI,
                               int(crn), store_capacity, logy2offset, seed, Ns, elbTmax,
                               elb_gibbsburn, elb)
        self.model, self.Ns, self.elbTmax, self.elb_gibbsburn = model, Ns, elbTmax, elb_gibbsburn
        h = self.lib.ccmm_chains_create(ctx.handle, C.byref(self.cfg))
        if not h:
            raise RuntimeError(f"ccmm_chains_create failed: {last_error()}")
        self.handle = h
        self.N, self.p, self.K, self.T, self.B = N, p, K, T, B
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def set_option(self, name: str, value: int):
        """ccmm_chains_set_option: a kernel form / schedule of this chain set (include/ccmm.h)."""
        _check(self.lib.ccmm_chains_set_option(self.handle, name.encode(), int(value)),
               f"ccmm_chains_set_option({name})")

    def get_option(self, name: str) -> int:
        v = C.c_int(0)
        _check(self.lib.ccmm_chains_get_option(self.handle, name.encode(), C.byref(v)),
               f"ccmm_chains_get_option({name})")
        return int(v.value)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ccmm_chains_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def crn_len(self):
        return int(self.lib.ccmm_chains_crn_len(self.handle))

    def crn_layout(self):
        """Per-sweep CRN record of one chain (ccmm_chains_sweep): name -> (offset, length,
        kind) in CCMM_RNG_* order, sizes from the set's maximum T / elbT (include/ccmm.h)."""
        cf = self.cfg
        N, T = self.N, self.T
        blocks = [("PAI", self.K * N, "n"), ("A", N * (N - 1) // 2, "n"), ("SVU", N * T, "u"),
                  ("SVZ", N * (T + 1), "n"), ("PHI", N * (T + cf.dPHI), "n")]
        if self.model in (MODEL_BLOCKHYBRID, MODEL_HYBRID, MODEL_SHADOWRATE):
            blocks.append(("ELB", self.Ns * self.elbTmax * (cf.elb_gibbsburn + 1), "u"))
        if getattr(self, "fH", 0):
            blocks.append(("FCST", 2 * N * self.fH * self.fNd, "n"))
        if getattr(self, "ps_np", 0):
            blocks.append(("PS", self.Ns * self.elbTmax * self.ps_np, "n"))
        out, o = {}, 0
        for name, n, kind in blocks:
            out[name] = (o, n, kind)
            o += n
        assert o == self.crn_len, (o, self.crn_len)
        return out

    def draw_crn(self, rng, nsweeps=1):
        """A random CRN array (crn_len, nsweeps, B): normals / uniforms per block."""
        lay = self.crn_layout()
        out = np.empty((self.crn_len, nsweeps, self.B), order="F")
        for o, n, kind in lay.values():
            shape = (n, nsweeps, self.B)
            out[o:o + n] = rng.random(shape) if kind == "u" else rng.standard_normal(shape)
        return out

    def set_data(self, slot, Y, X, iVdiag, iVb, sPHI, h0mean, h0vcvsqrt):
        Y = _f(Y)
        rc = self.lib.ccmm_chains_set_data(self.handle, slot, Y.shape[0], _ptr(Y), _ptr(_f(X)),
                                           _ptr(_f(iVdiag)), _ptr(_f(iVb)), _ptr(_f(sPHI)),
                                           _ptr(_f(h0mean)), _ptr(_f(h0vcvsqrt)))
        _check(rc, "ccmm_chains_set_data")

    def set_slots(self, slots):
        s = np.ascontiguousarray(slots, dtype=np.int32)
        _check(self.lib.ccmm_chains_set_slots(self.handle, s.ctypes.data_as(_ip)),
               "ccmm_chains_set_slots")

    def get_kai(self):
        """KSC indicators of the last SV block, T x N x B int8."""
        k = np.zeros((self.T, self.N, self.B), dtype=np.int8, order="F")
        _check(self.lib.ccmm_chains_get_kai(self.handle, k.ctypes.data_as(_i8p)), "ccmm_chains_get_kai")
        return k

    def get_cta_gram(self):
        """The device's weighted Gram of every CTA system at the current state, K x K x N x B
        ([c b'; b M], no prior; lag-structured path only)."""
        G = np.zeros((self.K, self.K, self.N, self.B), order="F")
        _check(self.lib.ccmm_chains_get_cta_gram(self.handle, _ptr(G)), "ccmm_chains_get_cta_gram")
        return G

    def get_cta_factor(self):
        """The device's CTA factor record of every system at the current state (ccmm_chains_get_cta_factor),
        decoded: S (NT*NT*256 per system, slot (ti, tj) at ti + tj NT as 16 x 16 row-major, the layout of
        oracle/cta_mirror.factor), l (16 NT), 1 / L00; arrays over (equation, chain)."""
        NT = (self.K - 1 + 15) // 16
        ntile = NT * (NT + 1) // 2
        n = ntile * 256 + 256
        raw = np.zeros((n, self.N, self.B), order="F")
        _check(self.lib.ccmm_chains_get_cta_factor(self.handle, _ptr(raw)), "ccmm_chains_get_cta_factor")
        S = np.zeros((NT * NT * 256, self.N, self.B))
        lane = np.arange(64)
        gi = 0
        for tj in range(NT):
            for ti in range(tj, NT):
                for r in range(4):
                    rows = (lane >> 4) + 4 * r
                    cols = lane & 15
                    base = (ti + tj * NT) * 256
                    S[base + rows * 16 + cols] = raw[gi * 256 + 64 * r + lane]
                gi += 1
        return S, raw[ntile * 256 + 1:ntile * 256 + 1 + 16 * NT], raw[ntile * 256]

    def record_elb_flags(self, enable=True):
        _check(self.lib.ccmm_chains_record_elb_flags(self.handle, int(bool(enable))),
               "ccmm_chains_record_elb_flags")

    def get_elb_flags(self):
        """drawTruncNormal branch flags of the last sweep's ELB step,
        Ns x elbTmax x (gibbsburn + 1) x B uint8."""
        f = np.zeros((self.Ns, self.elbTmax, self.elb_gibbsburn + 1, self.B), dtype=np.uint8, order="F")
        _check(self.lib.ccmm_chains_get_elb_flags(self.handle, f.ctypes.data_as(_u8p)),
               "ccmm_chains_get_elb_flags")
        return f

    def set_mfma_lock(self, lock_id):
        """Serialise the MFMA Gram + Cholesky phase with other chain sets of the same id
        (ccmm_chains_set_mfma_lock); 0 turns it off."""
        _check(self.lib.ccmm_chains_set_mfma_lock(self.handle, int(lock_id)), "ccmm_chains_set_mfma_lock")

    def set_rng_ids(self, ids):
        """Philox stream id per chain (None: the chain index)."""
        if ids is None:
            _check(self.lib.ccmm_chains_set_rng_ids(self.handle, None), "ccmm_chains_set_rng_ids")
            return
        a = np.ascontiguousarray(ids, dtype=np.uint32)
        assert a.size == self.B
        _check(self.lib.ccmm_chains_set_rng_ids(self.handle, a.ctypes.data_as(C.POINTER(C.c_uint32))),
               "ccmm_chains_set_rng_ids")

    def get_status(self):
        st = np.zeros(self.B, dtype=np.int32)
        _check(self.lib.ccmm_chains_get_status(self.handle, st.ctypes.data_as(_ip)),
               "ccmm_chains_get_status")
        return st

    def set_state(self, PAI, A, sqrtht, h, sqrtPHI):
        """Arrays K x N x B, N x N x B, T x N x B, T x N x B, N x N x B."""
        rc = self.lib.ccmm_chains_set_state(self.handle, _ptr(_f(PAI)), _ptr(_f(A)),
                                            _ptr(_f(sqrtht)), _ptr(_f(h)), _ptr(_f(sqrtPHI)))
        _check(rc, "ccmm_chains_set_state")

    def get_state(self):
        N, K, T, B = self.N, self.K, self.T, self.B
        out = dict(PAI=np.zeros((K, N, B), order="F"), A=np.zeros((N, N, B), order="F"),
                   invA=np.zeros((N, N, B), order="F"), sqrtht=np.zeros((T, N, B), order="F"),
                   h=np.zeros((T, N, B), order="F"), sqrtPHI=np.zeros((N, N, B), order="F"),
                   PHI=np.zeros((N, N, B), order="F"), RESID=np.zeros((T, N, B), order="F"))
        rc = self.lib.ccmm_chains_get_state(self.handle, *[_ptr(out[k]) for k in
                                                           ("PAI", "A", "invA", "sqrtht", "h",
                                                            "sqrtPHI", "PHI", "RESID")])
        _check(rc, "ccmm_chains_get_state")
        return out

    def sweep(self, nsweeps=1, crn=None, store=False):
        """crn: array of shape (crn_len, nsweeps, B) column-major (chain slowest) or None."""
        cp = None
        if crn is not None:
            crn = _f(crn)
            assert crn.size == self.crn_len * nsweeps * self.B
            cp = _ptr(crn)
        rc = self.lib.ccmm_chains_sweep(self.handle, int(nsweeps), cp, int(bool(store)))
        _check(rc, "ccmm_chains_sweep")
        return rc

    def stored(self):
        return int(self.lib.ccmm_chains_stored(self.handle))

    def get_draws(self, which=None):
        """Stored draws (then reset); ``which``: names to fetch (default all)."""
        M = self.stored()
        N, K, T, B = self.N, self.K, self.T, self.B
        shapes = dict(PAI_all=(M, K, N, B), PHI_all=(M, N * (N + 1) // 2, B), invA_all=(M, N, N, B),
                      sqrtht_all=(M, T, N, B))
        if self.model in (MODEL_BLOCKHYBRID, MODEL_HYBRID, MODEL_SHADOWRATE):
            shapes["shadowrate_all"] = (M, self.Ns, self.elbTmax, B)
        out = {k: np.zeros(v, order="F") for k, v in shapes.items() if which is None or k in which}
        rc = self.lib.ccmm_chains_get_draws(self.handle, *[_ptr(out.get(k)) for k in
                                                           ("PAI_all", "PHI_all", "invA_all",
                                                            "sqrtht_all", "shadowrate_all")])
        _check(rc, "ccmm_chains_get_draws")
        return out

    # ------------------------------------------------ predictive density (on device)
    def set_fcst(self, H, Nd, ndxYields, keep_paths=False):
        """Forecast every stored sweep (ccmm_chains_set_fcst): H horizons, Nd draws per kept
        draw; ndxYields bool N (ndxYIELDS)."""
        m = np.ascontiguousarray(np.asarray(ndxYields, bool), dtype=np.uint8)
        _check(self.lib.ccmm_chains_set_fcst(self.handle, int(H), int(Nd), m.ctypes.data_as(_u8p),
                                             int(bool(keep_paths))), "ccmm_chains_set_fcst")
        self.fH, self.fNd, self.fKeep = int(H), int(Nd), bool(keep_paths)

    def set_fcst_slot(self, slot, yrealized):
        """yrealized(:,1) of data slot ``slot`` (N values, shadow rates floored at the ELB)."""
        y = _f(np.asarray(yrealized, float).reshape(self.N, -1, order="F")[:, 0])
        _check(self.lib.ccmm_chains_set_fcst_slot(self.handle, int(slot), _ptr(y)),
               "ccmm_chains_set_fcst_slot")

    def set_fcst_censor(self, floor_in_recursion=None):
        """Variables floored inside the censored simulation (None: ndxYields)."""
        m = None if floor_in_recursion is None else \
            np.ascontiguousarray(np.asarray(floor_in_recursion, bool), dtype=np.uint8)
        _check(self.lib.ccmm_chains_set_fcst_censor(self.handle, None if m is None else m.ctypes.data_as(_u8p)),
               "ccmm_chains_set_fcst_censor")

    def fcst_stored(self):
        return int(self.lib.ccmm_chains_fcst_stored(self.handle))

    def get_fcst(self, paths=False):
        """Forecast records of the kept draws so far (then reset): scores Nd x M x 4 x B,
        fYsum / fYcsum / yhatsum N x H x B, and with ``paths`` the paths N x H x Nd x M x B."""
        M = self.fcst_stored()
        N, H, Nd, B = self.N, self.fH, self.fNd, self.B
        out = dict(M=M, scores=np.zeros((Nd, M, 4, B), order="F"),
                   fYsum=np.zeros((N, H, B), order="F"), fYcsum=np.zeros((N, H, B), order="F"),
                   yhatsum=np.zeros((N, H, B), order="F"))
        if paths:
            out["paths"] = np.zeros((N, H, Nd, M, B), order="F")
            out["paths_censored"] = np.zeros((N, H, Nd, M, B), order="F")
        rc = self.lib.ccmm_chains_get_fcst(self.handle, _ptr(out["scores"]), _ptr(out["fYsum"]),
                                           _ptr(out["fYcsum"]), _ptr(out["yhatsum"]),
                                           _ptr(out.get("paths")), _ptr(out.get("paths_censored")))
        if rc != CCMM_WARN_MVNCDF:
            _check(rc, "ccmm_chains_get_fcst")
        out["warn_mvncdf"] = rc == CCMM_WARN_MVNCDF
        return out

    # ------------------------------------------------ block-hybrid shadow-rate model
    def set_elb_model(self, ndxS, actual_block=None):
        """ndxS: 0-based shadow-rate variable indices; actual_block: bool N (actualrateBlock;
        None for the hybrid model)."""
        nd = np.ascontiguousarray(ndxS, dtype=np.int32)
        abp = None
        if actual_block is not None:
            ab = np.ascontiguousarray(np.asarray(actual_block, bool), dtype=np.uint8)
            abp = ab.ctypes.data_as(_u8p)
        _check(self.lib.ccmm_chains_set_elb_model(self.handle, nd.ctypes.data_as(_ip), abp),
               "ccmm_chains_set_elb_model")

    def set_elb_slot(self, slot, elbT0, sNaN):
        """sNaN: bool Ns x elbT (elbT = T_slot - elbT0)."""
        m = np.asfortranarray(np.asarray(sNaN, bool), dtype=np.uint8)
        _check(self.lib.ccmm_chains_set_elb_slot(self.handle, int(slot), int(elbT0),
                                                 m.ctypes.data_as(_u8p) if m.size else None),
               "ccmm_chains_set_elb_slot")

    def set_elb_ps(self, nproposals=1000, ps_from_m=1):
        """Acceptance-sampling branch (mcmcVARshadowrateBlockHybrid.m:435-466) from sweep
        m >= ps_from_m (1-based; the reference: ceil(MCMCburnin / 2)); 0 proposals disables."""
        _check(self.lib.ccmm_chains_set_elb_ps(self.handle, int(nproposals), int(ps_from_m)),
               "ccmm_chains_set_elb_ps")
        self.ps_np = int(nproposals)

    def get_ps(self):
        """countAccept, countAcceptBurnin (B) and stackAccept (M x B, 0 = none) of the
        stored draws (call before get_draws)."""
        M, B = self.stored(), self.B
        ca = np.zeros(B, np.int32)
        cb = np.zeros(B, np.int32)
        st = np.zeros((max(M, 1), B), np.int32, order="F")
        _check(self.lib.ccmm_chains_get_ps(self.handle, ca.ctypes.data_as(_ip), cb.ctypes.data_as(_ip),
                                           st.ctypes.data_as(_ip)), "ccmm_chains_get_ps")
        return dict(countAccept=ca, countAcceptBurnin=cb, stackAccept=st[:M])

    def keep_missingrate(self, enable=True):
        """Keep proposal 1 of every stored PS sweep (missingrate_all, ccmm_chains_keep_missingrate)."""
        _check(self.lib.ccmm_chains_keep_missingrate(self.handle, int(bool(enable))), "ccmm_chains_keep_missingrate")

    def get_missingrate(self):
        """missingrate_all of the stored draws, M x Ns x elbTmax x B (call before get_draws)."""
        out = np.zeros((self.stored(), self.Ns, self.elbTmax, self.B), order="F")
        if out.size:
            _check(self.lib.ccmm_chains_get_missingrate(self.handle, _ptr(out)), "ccmm_chains_get_missingrate")
        return out

    def get_ps_mean(self):
        """The last PS sweep's conditional mean of the censored cells (P^-1 b), Ns x elbTmax x B,
        NaN elsewhere (ccmm_chains_get_ps_mean)."""
        out = np.zeros((self.Ns, self.elbTmax, self.B), order="F")
        _check(self.lib.ccmm_chains_get_ps_mean(self.handle, _ptr(out)), "ccmm_chains_get_ps_mean")
        return out

    def summaries(self, source, slot, rows=None, cumcode=None, realized=None, pct=(), floor_rows=None, floor=0.0):
        """Device summaries of the kept draws of data slot ``slot`` (ccmm_chains_summaries):
        source 0 paths / 1 censored paths (series = rows x H) / 2 PAI (K x N).  floor_rows (N
        bools): those variables' paths floored at ``floor`` first (ccmm_chains_summaries_floor)."""
        N = self.N
        if source in (0, 1):
            nr = N if rows is None else int(np.count_nonzero(rows))
            S = nr * self.fH
        else:
            S = self.K * N
        pct = _f(np.asarray(pct, float).ravel())
        out = dict(mean=np.zeros(S), median=np.zeros(S), quantiles=np.zeros((S, pct.size), order="F"),
                   stdev=np.zeros(S))
        rz = None
        if realized is not None:
            rz = _f(np.asarray(realized, float).ravel(order="F"))
            assert rz.size == S
            out["crps"] = np.zeros(S)
        rw = None if rows is None else np.ascontiguousarray(np.asarray(rows, bool), dtype=np.uint8)
        cc = None if cumcode is None else np.ascontiguousarray(np.asarray(cumcode, bool), dtype=np.uint8)
        if floor_rows is not None:
            fr = np.ascontiguousarray(np.asarray(floor_rows, bool), dtype=np.uint8)
            assert fr.size == N
            _check(self.lib.ccmm_chains_summaries_floor(
                self.handle, int(source), int(slot), None if rw is None else rw.ctypes.data_as(_u8p),
                None if cc is None else cc.ctypes.data_as(_u8p), fr.ctypes.data_as(_u8p), float(floor), _ptr(rz),
                pct.size, _ptr(pct) if pct.size else None, _ptr(out["mean"]), _ptr(out["median"]),
                _ptr(out["quantiles"]) if pct.size else None, _ptr(out["stdev"]), _ptr(out.get("crps"))),
                "ccmm_chains_summaries_floor")
            return out
        _check(self.lib.ccmm_chains_summaries(
            self.handle, int(source), int(slot), None if rw is None else rw.ctypes.data_as(_u8p),
            None if cc is None else cc.ctypes.data_as(_u8p), _ptr(rz), pct.size,
            _ptr(pct) if pct.size else None, _ptr(out["mean"]), _ptr(out["median"]),
            _ptr(out["quantiles"]) if pct.size else None, _ptr(out["stdev"]), _ptr(out.get("crps"))),
            "ccmm_chains_summaries")
        return out

    def get_shadowrate(self):
        out = np.zeros((self.Ns, self.elbTmax, self.B), order="F")
        _check(self.lib.ccmm_chains_get_shadowrate(self.handle, _ptr(out)), "ccmm_chains_get_shadowrate")
        return out

    def get_xy(self):
        X = np.zeros((self.T, self.K, self.B), order="F")
        Y = np.zeros((self.T, self.N, self.B), order="F")
        _check(self.lib.ccmm_chains_get_xy(self.handle, _ptr(X), _ptr(Y)), "ccmm_chains_get_xy")
        return X, Y

    def profile(self, enable=True):
        _check(self.lib.ccmm_chains_profile(self.handle, int(enable)), "ccmm_chains_profile")

    def kernel_times(self):
        n = len(self.KERNELS)
        ms = np.zeros(n)
        cnt = np.zeros(n, dtype=np.int64)
        buf = C.create_string_buffer(1024)
        _check(self.lib.ccmm_chains_kernel_times(self.handle, n, _ptr(ms), cnt.ctypes.data_as(_i64p),
                                                 buf, 1024), "ccmm_chains_kernel_times")
        names = buf.value.decode().split(";")
        return {nm: (float(ms[i]), int(cnt[i])) for i, nm in enumerate(names[:n])}
