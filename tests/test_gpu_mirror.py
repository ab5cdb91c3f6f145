"""Parity on the real data at the north star's 1e-9: the device's arithmetic
order is measured and restated, so that the remaining difference is the factorisation only.

  * v_mfma_f64_16x16x4_f64: D = C + sum_k A(i,k) B(k,j) is four fused multiply-adds in k order
    (probes with cancellation and non-representable products; tools/probe_mfma_order.py).
  * The lag-structured coefficient kernel's weighted Gram [c b'; b M] (ccmm_chains_get_cta_gram)
    equals the C restatement in that order (oracle/cta_lag_mirror.c) BIT FOR BIT, on the real
    data (fredblockMD20-2022-09, N = 20, p = 12, T = 750, K = 241).
  * The factor record the kernel writes (intercept peel, 16 x 16 diagonal-tile factors and
    inverses with IEEE sqrt / division pivots, MFMA panel products and trailing updates; the
    unit block factor's blocks) equals the C restatement BIT FOR BIT (ccmm_chains_get_cta_factor
    vs oracle/cta_mirror.factor).
  * One CRN sweep on the real data against the oracle with CTA in that order end to end
    (oracle.linear_sweep(cta_form="mirror"): the mirrored factorisation and block substitutions):
    PAI, A, sqrtht and sqrtPHI within 1e-9 (|Δ| / max(|x|, sd_post)); KSC indicators bit-exact."""
import numpy as np
import pytest

from conftest import ROOT, rel_err
from helpers import crn_flat, random_state

pytestmark = pytest.mark.gpu


def test_mfma_f64_sequential_fma_order(ctx):
    import importlib.util
    spec = importlib.util.spec_from_file_location("pmo", ROOT / "tools" / "probe_mfma_order.py")
    pmo = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pmo)
    A, B, Cm = pmo.make_probes(24, seed=3)
    D = ctx.selftest_mfma_f64_acc(A, B, Cm)
    hits, total = pmo.evaluate(A, B, Cm, D, names={"fma_seq_0123", "exact_single_round", "rprod_seq_0123"})
    print(hits, total)
    assert hits["fma_seq_0123"] == total
    assert hits["exact_single_round"] < total and hits["rprod_seq_0123"] < total   # the probes discriminate


def _real(pkg, oracle, fred):
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    su = oracle.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    return su, m


def test_cta_gram_bit_exact_real_data(pkg, ctx, oracle, fred):
    from oracle import cta_mirror
    su, m = _real(pkg, oracle, fred)
    B = 2
    sts = [random_state(oracle, su, seed=300 + c) for c in range(B)]
    ch = pkg.Chains(ctx, N=su.N, p=su.p, T=su.T, B=B, crn=True)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    G = ch.get_cta_gram()
    ch.close()
    for c in range(B):
        for j in (0, 7, su.N - 1):
            sw = cta_mirror.weights(sts[c]["A"], sts[c]["sqrtht"], j)
            want = cta_mirror.gram(su.X, sw)
            got = G[:, :, j, c]
            nd = int(np.count_nonzero(got != want))
            print("chain", c, "eq", j, "entries differing", nd, "max rel", float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1e-300))))
            np.testing.assert_array_equal(got, want)


def test_cta_factor_bit_exact_real_data(pkg, ctx, oracle, fred):
    from oracle import cta_mirror
    su, m = _real(pkg, oracle, fred)
    B = 2
    sts = [random_state(oracle, su, seed=400 + c) for c in range(B)]
    ch = pkg.Chains(ctx, N=su.N, p=su.p, T=su.T, B=B, crn=True)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    S, lv, r = ch.get_cta_factor()
    ch.close()
    for c in range(B):
        for j in (0, 7, su.N - 1):
            sw = cta_mirror.weights(sts[c]["A"], sts[c]["sqrtht"], j)
            (Sw, lw, rw), bad = cta_mirror.factor(cta_mirror.gram(su.X, sw), su.iVdiag[:, j])
            assert not bad
            nd = int(np.count_nonzero(S[:, j, c] != Sw))
            rel = float(np.max(np.abs(S[:, j, c] - Sw) / np.maximum(np.abs(Sw), 1e-300)))
            print("chain", c, "eq", j, "factor entries differing", nd, "of", Sw.size, "max rel", rel,
                  "| l", int(np.count_nonzero(lv[:, j, c] != lw)), "| 1/L00", r[j, c] == rw)
            np.testing.assert_array_equal(lv[:, j, c], lw)
            assert r[j, c] == rw
            np.testing.assert_array_equal(S[:, j, c], Sw)


def test_linear_sweep_real_data_1e9(pkg, ctx, oracle, fred):
    su, m = _real(pkg, oracle, fred)
    B = 4
    sts = [random_state(oracle, su, seed=100 + c) for c in range(B)]
    rng = np.random.default_rng(21)
    crns = [oracle.draw_crn(rng, su.N, su.K, su.T, su.dPHI) for _ in range(B)]
    ch = pkg.Chains(ctx, N=su.N, p=su.p, T=su.T, B=B, crn=True)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    flat = np.stack([crn_flat(oracle, crns[c], su)[:, None] for c in range(B)], -1)
    ch.sweep(1, crn=flat)
    got = ch.get_state()
    kai = ch.get_kai()
    ch.close()
    worst = 0.0
    for c in range(B):
        st = oracle.linear_sweep(sts[c], su, crns[c], cta_form="mirror")
        _, _, sd = oracle.cta(su.Y, su.X, su.N, su.K, sts[c]["A"], sts[c]["sqrtht"], su.iVdiag, su.iVb,
                              sts[c]["PAI"], np.zeros((su.K, su.N)), return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "A": rel_err(got["A"][..., c], st["A"], oracle.a_step_sd(st["RESID"], sts[c]["sqrtht"])),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3)}
        print("chain", c, {k: f"{v:.2e}" for k, v in e.items()},
              "PAI entries differing", int(np.count_nonzero(got["PAI"][..., c] != st["PAI"])))
        np.testing.assert_array_equal(kai[..., c], st["kai"])
        worst = max(worst, max(e.values()))
    assert worst < 1e-9, worst
