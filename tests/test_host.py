"""CPU tests of the host side: the C-ABI library loads and exports every symbol
include/ccmm.h declares; host-only entry points behave; the host model setup
(ccmm_amd.model, mirror of mcmcVAR.m:28-206) equals the oracle's restatement."""
import os
import re
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT, rel_err


def header_functions():
    src = (ROOT / "include" / "ccmm.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ccmm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol(pkg):
    lib = pkg.load_library()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(pkg._abi.exported_symbols())


def test_abi_version_and_host_entry_points(pkg):
    lib = pkg.load_library()
    assert lib.ccmm_abi_version() == 4 == pkg._abi.ABI_VERSION
    # the ChainConfig ctypes mirror has the header's fields in order
    src = (ROOT / "include" / "ccmm.h").read_text()
    start = src.index("typedef struct {", src.index("sweep-level")) + len("typedef struct {")
    body = re.sub(r"/\*.*?\*/", "", src[start:src.index("} ccmm_chain_config;")], flags=re.S)
    names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl:  # "int N, p, K" -> N, p, K
            names += [n.strip() for n in decl.split(None, 1)[1].split(",")]
    assert names == [f[0] for f in pkg._abi.ChainConfig._fields_]
    # host scalar drawTruncNormal (no GPU needed) matches the oracle's branches
    v, fl = pkg._abi.draw_trunc_normal(0.7, 1e-12, 0.25, 0.3)
    assert (v, fl) == (0.7, 0)
    v, fl = pkg._abi.draw_trunc_normal(60.0, 1.0, 0.25, 0.3)
    assert fl == 1 and abs(v - 0.25) < 1e-12


def test_host_trunc_normal_matches_oracle_golden(pkg):
    g = np.load(ROOT / "tests" / "golden" / "truncnorm_kat.npz")
    for i in range(g["mu"].size):
        v, fl = pkg._abi.draw_trunc_normal(g["mu"][i], g["sig"][i], float(g["elb"]), g["u"][i])
        assert fl == g["flags"][i]
        assert abs(v - g["draw"][i]) <= 1e-12 * max(1.0, abs(g["draw"][i]))


def test_no_gpu_fails_loudly(pkg):
    """Without a visible GPU the product path refuses to run (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    with pytest.raises(RuntimeError, match="no HIP device"):
        pkg.Context(0)


def test_host_setup_matches_oracle(pkg, oracle, fred):
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    np.testing.assert_array_equal(mpm, oracle.set_minnesota_mean(fred["ncode"]))
    for thisT in (len(fred["ydates"]), 599):
        m = pkg.model.build_var(thisT, 12, 12, fred["data"], fred["ydates"], mpm, True)
        su = oracle.var_setup(thisT, 12, 12, fred["data"], fred["ydates"], mpm, True)
        assert (m.T, m.K, m.N) == (su.T, su.K, su.N)
        np.testing.assert_array_equal(m.X, su.X)
        np.testing.assert_array_equal(m.Y, su.Y)
        assert rel_err(m.iVdiag, su.iVdiag) < 1e-13
        assert rel_err(m.iVb, su.iVb, 1e-12) < 1e-13
        assert rel_err(m.sPHI, su.sPHI, 1.0) < 1e-15
        np.testing.assert_array_equal(m.Xjumpoff, su.Xjumpoff)
    st = pkg.model.initial_state(m, 3)
    so = oracle.init_state(su)
    assert st["PAI"].shape == (su.K, su.N, 3)
    assert rel_err(st["sqrtht"][..., 2], so["sqrtht"]) < 1e-14


def test_shadow_yield_sets(pkg, oracle, fred):
    for elb in (0.125, 0.25, 0.5):
        a = pkg.model.setShadowYields(fred["ncode"], elb)
        b = oracle.set_shadow_yields(fred["ncode"], elb)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    s, o, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    assert [fred["ncode"][i] for i in s] == ["FEDFUNDS", "TB6MS", "GS1"]
    assert [fred["ncode"][i] for i in o] == ["GS5", "GS10", "BAA"]
    assert oracle.elb_t0(fred["data"], s, 0.25, 12) == 585


def test_realized_values_floor_shadow_rates(pkg, fred):
    """yrealized of a vintage (goVAR.m:252-267): data rows after the jump-off, NaN past
    the sample end, shadow-rate series floored at the ELB; other series untouched."""
    s, o, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    data = fred["data"]
    thisT = len(fred["ydates"]) - 30      # 2020-02: the funds rate goes to the ELB in 2020-04
    yr = pkg.samplers.realized_values(data, thisT, 48, s, 0.25)
    assert yr.shape == (data.shape[1], 48)
    assert np.all(np.isnan(yr[:, 30:])) and np.all(np.isfinite(yr[:, :30]))
    raw = data[thisT:thisT + 30].T
    floored = raw[s] < 0.25
    assert floored.any()
    np.testing.assert_array_equal(yr[s, :30][floored], 0.25)
    np.testing.assert_array_equal(yr[s, :30][~floored], raw[s][~floored])
    others = np.setdiff1d(np.arange(data.shape[1]), s)
    np.testing.assert_array_equal(yr[others, :30], raw[others])


def test_govar_batch_floors_yrealized_and_picks_rank_device(pkg, monkeypatch):
    """goVAR_batch hands run_vintage the floored yrealized, and a rank under a
    process group defaults to its LOCAL_RANK device."""
    data = np.full((60, 3), 1.0)
    data[:, 2] = 0.1                       # a shadow-rate series below the ELB
    seen = []

    def run_vintage(thisT, yreal, seed):
        seen.append(yreal.copy())
        ls = np.zeros((4, 1))
        return ls, ls, ls, ls, np.zeros((3, 2))

    pkg.samplers.goVAR_batch(data, np.arange(60.0), [40, 50], 2, 12, 4, 4, 2, np.ones(3), [2],
                             run_vintage=run_vintage, ndxSHADOWRATE=[2])
    assert len(seen) == 2
    for y in seen:
        np.testing.assert_array_equal(y[2], 0.25)
        np.testing.assert_array_equal(y[:2], 1.0)
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert pkg.samplers._rank_device(object(), None) == 3
    assert pkg.samplers._rank_device(object(), 1) == 1
    assert pkg.samplers._rank_device(None, None) == 0


def test_vintage_batch_argument_checks(pkg, fred):
    """The batch drivers refuse what they do not build before touching a device: an unknown
    model, the shadow-rate VAR on the native engine (its floored summaries run through the
    Python driver), max VAR roots for the hybrid model (goVARhybrid.m:383-430 commented out)."""
    S = pkg.samplers
    ndxS, ndxO, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    args = (fred["data"], fred["ydates"], ndxS, ndxO, mpm)
    with pytest.raises(ValueError, match="unknown model"):
        S.goVARshadowrateBlockHybrid_batch(*args, model="linear", Tjumpoffs=[700])
    with pytest.raises(ValueError, match="Python engine"):
        S.goVARshadowrate_batch(*args, engine="native", Tjumpoffs=[700])
    with pytest.raises(ValueError, match="max VAR roots"):
        S.goVARhybrid_batch(*args, maxlambda=True, Tjumpoffs=[700])
    with pytest.raises(ValueError, match="multiple of MCMCdraws"):
        S.goVARshadowrate_batch(*args, MCMCdraws=10, fcstNdraws=15, Tjumpoffs=[700])


def test_psrf_entry_points_match_oracle(pkg):
    """ccmm_psrf / ccmm_shadowrate_psrf (host computations inside libccmm) against the oracle's psrf
    restatement (DiagnosticsShadowrate.m:34-128): one chain (thirds), C chains, the ELB mask."""
    from oracle.ccmm_oracle_stats import psrf, diagnostics_shadowrate, diagnostics_shadowrate_chain_mean
    A = pkg._abi
    rng = np.random.default_rng(11)
    X = np.cumsum(rng.standard_normal((301, 6)), axis=0)
    assert np.max(np.abs(A.psrf(X) - psrf(X))) < 1e-12
    X3 = rng.standard_normal((40, 3, 5))
    assert np.max(np.abs(A.psrf(X3) - psrf(X3))) < 1e-12
    M, Ns, ldT, elbT = 120, 3, 9, 7
    for C in (1, 3):
        d = rng.standard_normal((M, Ns, ldT, C)) * rng.random((1, Ns, ldT, 1)) + rng.random((1, 1, ldT, C))
        mask = rng.random((Ns, elbT)) < 0.5
        mask[2] = False                                # rate with no month at the ELB: NaN
        got = A.shadowrate_psrf(d, mask)
        gotc = A.shadowrate_psrf(d, mask, chains=True)
        for s in range(Ns):
            cells = d[:, s, :elbT, :][:, mask[s], :]
            want = diagnostics_shadowrate_chain_mean(cells)     # the reference's statistic per chain
            wantc = diagnostics_shadowrate(cells) if C > 1 else np.nan   # psrf across the chains
            for g, w in ((got[s], want), (gotc[s], wantc)):
                if np.isnan(w):
                    assert np.isnan(g)
                else:
                    assert abs(g - w) < 1e-12 * max(1.0, abs(w)), (C, s, g, w)
    assert np.all(np.isnan(A.shadowrate_psrf(np.ones((2, 2, 3)), np.ones((2, 3), bool))))   # too few draws


ABLATION_VARS = ("CCMM_CHOL_SKIP", "CCMM_SOLVE_SKIP", "CCMM_SV_SKIP", "CCMM_GC_MODE", "CCMM_LAG_MODE",
                 "CCMM_BIG_MASK", "CCMM_ELB_MODE", "CCMM_SV_MODE", "CCMM_FCST_MODE", "CCMM_POISON")
# the kernel A/B switches of round 5 and every schedule selector: a default build
# reads none of them (kernel forms and schedules are explicit options, ccmm_set_option)
SELECTOR_VARS = {"CCMM_OLD_SOLVE": None, "CCMM_OLD_CHOL": None, "CCMM_GC18": None, "CCMM_NO_LAG": None,
                 "CCMM_NO_QR_FALLBACK": None, "CCMM_SOLVE_WAVES": None,
                 "CCMM_ASTEP_V1": ("astep_serial", 0), "CCMM_PS_CHOL_V1": ("ps_chol_lds", 0),
                 "CCMM_FORCE_BIG": ("large_path", 0), "CCMM_SV_MFMA": ("sv_mfma", 1),
                 "CCMM_SOLVE_SPLIT": ("solve_split", -1), "CCMM_SOLVE_ASYNC": ("solve_async", 1),
                 "CCMM_SV_NWG": ("sv_nwg", 0), "CCMM_ELB_WAVES": ("elb_waves", 8), "CCMM_ELB_OCT": ("elb_oct", 1),
                 "CCMM_ELB_ASYNC": ("elb_async", 1), "CCMM_ELB_PARTS": ("elb_parts", 0),
                 "CCMM_ELB_SPEC": ("elb_spec", 0),
                 "CCMM_FCST_REG": ("fcst_reg", 1), "CCMM_FCST_OVERLAP": ("fcst_overlap", 1), "CCMM_PHI_OVERLAP": ("phi_overlap", 1),
                 "CCMM_QR_FALLBACK": ("qr_fallback", 1), "CCMM_LAG": ("lag", 1), "CCMM_FORCE_QR": ("force_qr", 0),
                 "CCMM_GIRF_GENERIC": ("girf_generic", 0), "CCMM_BIG_LAGX": ("big_lagx", 1)}


def test_default_build_ignores_every_selector(pkg, monkeypatch):
    """No CCMM_* variable changes what the default library runs: with every A/B switch and schedule
    selector set (to a non-default value), each option still starts from its built-in default, and
    ccmm_env_ignored names every variable."""
    lib = pkg.load_library()
    assert lib.ccmm_ablation_build() == 0
    for v in list(SELECTOR_VARS) + list(ABLATION_VARS):
        monkeypatch.delenv(v, raising=False)
    assert pkg._abi.env_ignored() == (0, [])
    for v, o in SELECTOR_VARS.items():
        monkeypatch.setenv(v, "0" if o is not None and o[1] == 1 else "1")
    n, names = pkg._abi.env_ignored()
    assert n == len(SELECTOR_VARS) and sorted(names) == sorted(SELECTOR_VARS), names
    opts = set(pkg._abi.option_names())
    for v, o in SELECTOR_VARS.items():
        if o is not None:
            assert o[0] in opts
            assert pkg._abi.option_default(o[0]) == o[1], (v, o)
    assert opts == {o[0] for o in SELECTOR_VARS.values() if o is not None}


def test_default_build_ignores_timing_ablations(pkg, monkeypatch):
    """The timing-only ablation switches (results invalid) are read only by a -DCCMM_ABLATION build
    (libccmm_ablation.so); the default library ignores them and names them (include/ccmm.h)."""
    lib = pkg.load_library()
    assert lib.ccmm_ablation_build() == 0
    for v in ABLATION_VARS:
        monkeypatch.delenv(v, raising=False)
    assert pkg._abi.env_ignored() == (0, [])
    for v in ABLATION_VARS:
        monkeypatch.setenv(v, "1")
    n, names = pkg._abi.env_ignored()
    assert n == len(ABLATION_VARS) and sorted(names) == sorted(ABLATION_VARS)
    # CCMM_SV_MODE bit 128 (full-row SV block factors) is read by the ablation build only, like the rest
    monkeypatch.setenv("CCMM_SV_MODE", "128")
    n, names = pkg._abi.env_ignored()
    assert "CCMM_SV_MODE" in names and n == len(ABLATION_VARS)


def test_ablation_build_honours_switches():
    """libccmm_ablation.so (make ablation), when built, reports ablation mode, ignores nothing and takes
    an option's default from its CCMM_* variable (checked in a child process: the timing build is never
    loaded beside the product library)."""
    import subprocess
    import sys
    p = ROOT / "ccmmshadowratevar-code_amd" / "csrc" / "libccmm_ablation.so"
    if not p.exists():
        pytest.skip("libccmm_ablation.so not built")
    code = ("import ctypes, sys; lib = ctypes.CDLL(sys.argv[1]); v = ctypes.c_int(0); "
            "lib.ccmm_option_default(b'elb_waves', ctypes.byref(v)); "
            "print(lib.ccmm_ablation_build(), lib.ccmm_env_ignored(None, 0), v.value)")
    env = dict(os.environ, CCMM_CHOL_SKIP="1", CCMM_ELB_WAVES="4")
    out = subprocess.run([sys.executable, "-c", code, str(p)], env=env, capture_output=True, text=True,
                         check=True, timeout=120).stdout.split()
    assert out == ["1", "0", "4"], out
