"""Driver of the compiled CPU restatement (oracle/cpu_sweep.cpp) -- TEST / BASELINE INFRASTRUCTURE ONLY:
bench.py's cpu_baseline leg and tests/test_cpu_baseline.py call it; the product never does.

The linear sweep of mcmcVAR.m:211-274 as written (kron-materialised CTA, explicit inverse) and the
block-hybrid sweep of mcmcVARshadowrateBlockHybrid.m:332-520 as written (kron CTAsys, the QR form of
gibbsdrawShadowrates), one single-threaded process per chain (the parfor worker of goVAR*.m), BLAS /
LAPACK from the OpenBLAS that numpy and scipy use (opened by the binary with dlopen)."""
from __future__ import annotations

import json
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
BIN = _HERE / "cpu_sweep"


def blas_path():
    """The OpenBLAS shared library scipy's LAPACK wrappers use (LP64 scipy_d*_ entry points)."""
    import scipy
    libs = Path(scipy.__file__).resolve().parent.parent / "scipy.libs"
    cands = sorted(libs.glob("libscipy_openblas*.so*")) if libs.is_dir() else []
    if not cands:
        raise RuntimeError(f"no libscipy_openblas in {libs}")
    return str(cands[0])


def ensure_built():
    if not BIN.exists() or BIN.stat().st_mtime < (_HERE / "cpu_sweep.cpp").stat().st_mtime:
        subprocess.run(["make", "-C", str(_HERE), "cpu_sweep"], check=True, capture_output=True)
    return BIN


def write_state(path, su, st, bs=None):
    """state.bin of cpu_sweep.cpp: the setup (oracle.var_setup) and a chain state; with bs (an
    oracle.ccmm_oracle_bh.BHSetup) the block-hybrid block, Y / X then being the chain's shadow-rate data
    (st["Y"], st["X"])."""
    F = lambda a: np.asfortranarray(np.asarray(a, np.float64)).ravel(order="F")
    Y, X = (st["Y"], st["X"]) if bs is not None else (su.Y, su.X)
    with open(path, "wb") as fh:
        np.array([su.N, su.K, su.T, su.dPHI], np.int32).tofile(fh)
        for a in (Y, X, su.iVdiag, su.iVb, su.sPHI, su.Vol_0mean, su.Vol_0vcvsqrt,
                  np.array([su.logy2offset]), st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"]):
            F(a).tofile(fh)
        if bs is not None:
            np.array([0x31304842, su.p, len(bs.ndxS), bs.elbT0, bs.elbT, bs.gibbsburn, bs.Ydata.shape[0]],
                     np.int32).tofile(fh)
            for a in (np.array([bs.ELB]), bs.Xactual, bs.actualrateBlock.astype(float),
                      np.asarray(bs.ndxS, float), bs.sNaN.astype(float), bs.Ydata):
                F(a).tofile(fh)


def _env():
    env = dict(os.environ)
    env["CCMM_CPU_BLAS"] = blas_path()
    env["OPENBLAS_NUM_THREADS"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    return env


def crn_sweep(su, st, crn, workdir, bs=None, form="kron"):
    """One sweep on the injected common random numbers (oracle.crn_sizes order; block hybrid: + uELB);
    returns the new PAI, A, sqrtht, h, sqrtPHI, the KSC indicators and (bs) the shadow rates."""
    ensure_built()
    workdir = Path(workdir)
    sp, cp, op = workdir / "state.bin", workdir / "crn.bin", workdir / "out.bin"
    write_state(sp, su, st, bs)
    with open(cp, "wb") as fh:
        for k in ("zPAI", "zA", "uSV", "zSV", "zPHI") + (("uELB",) if bs is not None else ()):
            np.asfortranarray(crn[k], dtype=np.float64).ravel(order="F").tofile(fh)
    mode = "crn" if form == "kron" else "crn-syrk"
    subprocess.run([str(BIN), mode, str(sp), str(cp), str(op)], check=True, env=_env(), capture_output=True)
    v = np.fromfile(op, np.float64)
    N, K, T = su.N, su.K, su.T
    out, o = {}, 0
    shapes = [("PAI", (K, N)), ("A", (N, N)), ("sqrtht", (T, N)), ("h", (T, N)), ("sqrtPHI", (N, N)),
              ("kai", (N, T))]
    if bs is not None:
        shapes.append(("shadowrate", (len(bs.ndxS), bs.elbT)))
    for k, shp in shapes:
        n = int(np.prod(shp))
        out[k] = v[o:o + n].reshape(shp, order="F")
        o += n
    out["kai"] = out["kai"].astype(np.int8)
    return out


def bench_process(state_path, seconds, seed, form="kron"):
    """Start one single-threaded worker process (the caller runs several at once); returns the Popen.
    form: "kron" (CTA / CTAsys as written) or "syrk" (the algorithmic weighted-SYRK form)."""
    ensure_built()
    mode = "bench" if form == "kron" else "bench-syrk"
    return subprocess.Popen([str(BIN), mode, str(state_path), f"{seconds:.3f}", str(int(seed))],
                            env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def bench_result(proc, timeout):
    out, err = proc.communicate(timeout=timeout)
    if proc.returncode != 0:
        raise RuntimeError(f"cpu_sweep failed ({proc.returncode}): {err.strip()}")
    r = json.loads(out.strip().splitlines()[-1])
    return int(r["sweeps"]), float(r["seconds"])
