"""GPU parity: every libccmm block, called through the C ABI, against the CPU
oracle on the same inputs and common random numbers (CRN).

Tolerances (fp64):
  * CTA draws: |delta| / max(|x|, sd_post) <= 1e-9 on well-conditioned
    systems; on the reference initialisation of the real data (cond(iV_post)
    up to ~1e13) the bound is 1e-6: there a mere reordering of
    the SYRK summation moves draws by ~5e-7 sd (measured).
  * A, SV, PHI blocks: 1e-9 relative.
  * KSC mixture indicators and truncated-normal branch flags: bit-exact.
"""
import numpy as np
import pytest

from conftest import rel_err
from helpers import crn_flat, random_state, toy_setup

pytestmark = pytest.mark.gpu


def test_mfma_f64_layout(ctx):
    rng = np.random.default_rng(0)
    A = rng.integers(-8, 8, (16, 4)).astype(float)
    B = rng.integers(-8, 8, (4, 16)).astype(float)
    D = ctx.selftest_mfma_f64(A, B)
    np.testing.assert_array_equal(D, A @ B)


def _cta_case(oracle, su, st, rng):
    z = rng.standard_normal((su.K, su.N))
    PAI0 = st["PAI"] + 0.01 * rng.standard_normal(st["PAI"].shape)
    want, status, sd = oracle.cta(su.Y, su.X, su.N, su.K, st["A"], st["sqrtht"], su.iVdiag,
                                  su.iVb, PAI0, z, return_sd=True)
    return PAI0, z, want, sd


def test_cta_toy(ctx, oracle):
    su = toy_setup(oracle, N=4, p=2, Tobs=62)
    rng = np.random.default_rng(3)
    B = 3
    cases = [_cta_case(oracle, su, random_state(oracle, su, seed=10 + c), rng) for c in range(B)]
    sts = [random_state(oracle, su, seed=10 + c) for c in range(B)]
    got, status = ctx.cta(su.Y, su.X, np.stack([s["A"] for s in sts], -1),
                          np.stack([s["sqrtht"] for s in sts], -1), su.iVdiag, su.iVb,
                          np.stack([c[0] for c in cases], -1), np.stack([c[1] for c in cases], -1))
    assert not status.any()
    for c in range(B):
        assert rel_err(got[..., c], cases[c][2], cases[c][3]) < 1e-9


def test_cta_real_smooth(ctx, oracle, fred):
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    su = oracle.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    st = random_state(oracle, su, seed=5)
    rng = np.random.default_rng(4)
    PAI0, z, want, sd = _cta_case(oracle, su, st, rng)
    got, status = ctx.cta(su.Y, su.X, st["A"][..., None], st["sqrtht"][..., None], su.iVdiag,
                          su.iVb, PAI0[..., None], z[..., None])
    assert not status.any()
    err = rel_err(got[..., 0], want, sd)
    print("cta real smooth rel err (sd units)", err)
    assert err < 1e-8


def test_cta_real_reference_init(ctx, oracle, fred):
    """At the reference initialisation (A = I, sqrtht from AR residuals,
    mcmcVAR.m:197-206) cond(iV_post) reaches ~1e13: every fp64 evaluation
    (the oracle as written included) sits ~5e-5 sd from an 80-bit evaluation
    (tests/golden/cta_refinit.npz).  Bar: the GPU is as accurate as the
    oracle against that extended-precision answer, and within 2e-4 sd of it."""
    g = np.load(__import__("conftest").ROOT / "tests/golden/cta_refinit.npz")
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    su = oracle.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    st = oracle.init_state(su)
    got, status = ctx.cta(su.Y, su.X, st["A"][..., None], st["sqrtht"][..., None], su.iVdiag,
                          su.iVb, st["PAI"][..., None], g["z"][..., None])
    sd, ld = g["sd"], g["PAI_longdouble"]
    e_gpu = rel_err(got[..., 0], ld, sd)
    e_orc = rel_err(g["PAI_oracle"], ld, sd)
    print(f"cta reference-init: gpu vs 80-bit {e_gpu:.2e}, oracle vs 80-bit {e_orc:.2e}")
    assert e_gpu < max(2.0 * e_orc, 1e-9)
    assert rel_err(got[..., 0], g["PAI_oracle"], sd) < 2e-4


def test_ctasys_per_equation_designs(ctx, oracle):
    su = toy_setup(oracle, N=4, p=2, Tobs=62, seed=2)
    st = random_state(oracle, su, seed=8)
    rng = np.random.default_rng(9)
    XX = np.repeat(su.X[:, :, None], su.N, axis=2)
    XX[:, 1:, 2:] += 0.1 * rng.standard_normal((su.T, su.K - 1, su.N - 2))  # two distinct slabs
    XX[:, :, 3] = XX[:, :, 2]
    z = rng.standard_normal((su.K, su.N))
    want, _, sd = oracle.cta_sys(su.Y, XX, su.N, su.K, su.T, st["A"], st["sqrtht"], su.iVdiag,
                                 su.iVb, st["PAI"], z, return_sd=True)
    got, status = ctx.cta(su.Y, XX, st["A"][..., None], st["sqrtht"][..., None], su.iVdiag,
                          su.iVb, st["PAI"][..., None], z[..., None])
    assert rel_err(got[..., 0], want, sd) < 1e-9


@pytest.mark.parametrize("Tobs", [90, 1100])  # 1100: a sample longer than 1024 months
def test_astep(ctx, oracle, Tobs):
    su = toy_setup(oracle, N=6, p=2, Tobs=Tobs, seed=4)
    st = random_state(oracle, su, seed=2)
    rng = np.random.default_rng(1)
    RESID = su.Y - su.X @ st["PAI"]
    z = rng.standard_normal(su.N * (su.N - 1) // 2)
    A, invA = oracle.a_step(RESID, st["sqrtht"], z)
    gA, ginvA = ctx.astep(RESID[..., None], st["sqrtht"][..., None], z[:, None])
    assert rel_err(gA[..., 0], A, 1e-3) < 1e-10
    assert rel_err(ginvA[..., 0], invA, 1e-3) < 1e-10


@pytest.mark.parametrize("N", [5, 20, 30])  # k_sv_part buckets 8, 20 and 32 (two waves, LDS)
def test_sv_ksc(ctx, oracle, N):
    su = toy_setup(oracle, N=N, p=2, Tobs=120, seed=6)
    st = random_state(oracle, su, seed=3)
    rng = np.random.default_rng(2)
    RESID = su.Y - su.X @ st["PAI"]
    logy2 = np.log((RESID @ st["A"].T) ** 2 + su.logy2offset)
    u = rng.random((su.N, su.T))
    z = rng.standard_normal((su.N, su.T + 1))
    h, h0, sh, kai = oracle.sv_ksc_corrsqrt(logy2.T, st["h"].T, st["sqrtPHI"], su.Vol_0mean,
                                           su.Vol_0vcvsqrt, u, z)
    gh, gh0, gsh, gkai = ctx.sv_ksc(logy2.T[..., None], st["h"].T[..., None],
                                    st["sqrtPHI"][..., None], su.Vol_0mean, su.Vol_0vcvsqrt,
                                    u[..., None], z[..., None])
    np.testing.assert_array_equal(gkai[..., 0], kai)
    assert rel_err(gh[..., 0], h, 1.0) < 1e-9
    assert rel_err(gsh[..., 0], sh, 1e-2) < 1e-9
    assert rel_err(gh0[:, 0], h0, 1.0) < 1e-9


def test_phi_iw(ctx, oracle):
    su = toy_setup(oracle, N=5, p=2, Tobs=120, seed=6)
    rng = np.random.default_rng(11)
    eta = 0.1 * rng.standard_normal((su.T, su.N))
    Z = rng.standard_normal((su.N, su.T + su.dPHI))
    sq, PHI = oracle.phi_iw(eta, su.sPHI, Z)
    gsq, gPHI = ctx.phi_iw(eta[..., None], su.sPHI, su.dPHI, Z[..., None])
    assert rel_err(gPHI[..., 0], PHI, np.abs(PHI).max()) < 1e-12
    assert rel_err(gsq[..., 0], sq, np.abs(sq).max()) < 1e-12


def test_truncnorm_batch(ctx, oracle):
    rng = np.random.default_rng(12)
    n = 4000
    mu = rng.normal(0.5, 2.0, n)
    sig = np.abs(rng.normal(0.0, 1.0, n))
    sig[:50] = 1e-12            # sigma <= tol branch
    mu[50:100] = 40.0           # PHIbar <= eps branch
    sig[50:100] = 1.0
    u = rng.random(n)
    want = np.array([oracle.draw_trunc_normal(mu[i], sig[i], 0.25, u[i]) for i in range(n)])
    got, fl = ctx.draw_trunc_normal_batch(mu, sig, 0.25, u)
    np.testing.assert_array_equal(fl, want[:, 1].astype(np.uint8))
    assert rel_err(got, want[:, 0], 1e-3) < 1e-12
    assert np.all(got[100:] <= 0.25 + 1e-12)


@pytest.mark.parametrize("B,nsweeps,tol,form", [(4, 1, 5e-8, "kron"), (4, 3, 1e-6, "kron"), (4, 1, 1e-9, "mirror"),
                                                (4, 3, 1e-9, "mirror")])
def test_linear_sweep_crn(pkg, ctx, oracle, fred, B, nsweeps, tol, form):
    """Full linear BVAR-SV sweeps (CTA -> A -> SV -> PHI) on real data, CRN per chain, in units of
    max(|x|, posterior sd).  form="kron": the oracle's CTA as written (CTA.m); the summation
    orders differ, so one sweep sits at 5e-8 and three chained sweeps compound to 1e-6.
    form="mirror": the oracle's CTA in the device's operation order (oracle/cta_mirror.py): 1e-9
    for one sweep and for three chained sweeps."""
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    su = oracle.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    sts = [random_state(oracle, su, seed=100 + c) for c in range(B)]
    rng = np.random.default_rng(21)
    crns = [[oracle.draw_crn(rng, su.N, su.K, su.T, su.dPHI) for _ in range(nsweeps)]
            for _ in range(B)]
    ch = pkg.Chains(ctx, N=su.N, p=su.p, T=su.T, B=B, crn=True)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h",
                                                               "sqrtPHI")])
    flat = np.stack([np.stack([crn_flat(oracle, crns[c][m_], su) for m_ in range(nsweeps)], -1)
                     for c in range(B)], -1)
    ch.sweep(nsweeps, crn=flat)
    got = ch.get_state()
    kai = ch.get_kai()
    prev = {}
    prev_sqrtht = prev.get
    for c in range(B):
        st = sts[c]
        for m_ in range(nsweeps):
            prev[c] = st["sqrtht"]
            st = oracle.linear_sweep(st, su, crns[c][m_], cta_form=form)
        _, _, sd = oracle.cta(su.Y, su.X, su.N, su.K, st["A"], st["sqrtht"], su.iVdiag, su.iVb,
                              st["PAI"], np.zeros((su.K, su.N)), return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "A": rel_err(got["A"][..., c], st["A"], oracle.a_step_sd(st["RESID"], prev_sqrtht(c))),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3)}
        print("chain", c, nsweeps, form, e, "| PAI entries differing",
              int(np.count_nonzero(got["PAI"][..., c] != st["PAI"])))
        assert max(e.values()) < tol, e
        np.testing.assert_array_equal(kai[..., c], st["kai"])  # KSC indicators: bit-exact


def test_linear_sweep_philox_batch(pkg, ctx, oracle, fred):
    """Production mode: 64 chains, Philox draws, stored draws finite and distinct."""
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    B = 64
    ch = pkg.Chains(ctx, N=m.N, p=m.p, T=m.T, B=B, crn=False, store_capacity=4, seed=1012023)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(6, store=False)
    ch.sweep(4, store=True)
    d = ch.get_draws()
    assert d["PAI_all"].shape == (4, m.K, m.N, B)
    for v in d.values():
        assert np.all(np.isfinite(v))
    assert np.std(d["PAI_all"][-1, 1, 0, :]) > 0  # chains differ
