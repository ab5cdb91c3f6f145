"""Monte Carlo parity on the reference's own data (fredblockMD20-2022-09, 2022-08 jump-off,
N = 20, p = 12, T = 750, K = 241): posterior means from 128 Philox device chains against long
oracle chains committed as tests/golden/mcse_real_{linear,bh}.npz (tools/
make_mcse_real_fixture.py: 1000 burn-in + 2000 kept sweeps per chain, Geweke NSE with the 15 %
taper of Diagnostics.m:134-300; each fixture pools seven independent chains, whose between-chain
spread bounds the oracle's standard error from below: one linear chain's spectral NSE understates
the spread of the seven chain means by up to 2.3x), the device chains averaging the same window of
sweeps.

  linear  configs[1] / SURVEY §8d C2: mcmcVAR.m sweeps from the reference initialisation.
  bh      configs[2] / C3: mcmcVARshadowrateBlockHybrid.m at ELB 0.25 with the reference's ELB
          schedule (Gibbs for m < MCMCburnin / 2 = 500, then 1000 PS proposals, accept-first,
          Gibbs fallback; ~3 % of proposals sets accepted on this window), so the Gibbs-fallback
          regime of the real run has a posterior-level check.

Quantities: intercepts, own and FEDFUNDS first-lag coefficients of every equation, the
subdiagonal of A, diag(PHI), sqrtht at three months (+ 24 censored shadow-rate cells for bh).
Each must agree within 4.5 combined standard errors: the device chains are independent, so
their estimate's standard error is the spread of the 128 chain means / sqrt(128).  A different
generator stream makes this the test that the device samples the same posterior."""
import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _fixture(kind):
    path = ROOT / "tests" / "golden" / f"mcse_real_{kind}.npz"
    if not path.exists():
        pytest.fail(f"{path.name} missing: run tools/make_mcse_real_fixture.py {kind}")
    return np.load(path)


def _oracle_accept(g):
    if "accept_rate" in g:
        return float(g["accept_rate"])
    return float(g["accept"]) / (int(g["burn"]) + int(g["keep"]) - int(g["burn"]) // 2)


def _vech_diag_index(N):
    """Positions of PHI's diagonal in PHI_all = PHI_((tril(PHI_))~=0) (column-major vech)."""
    off, out = 0, []
    for j in range(N):
        out.append(off)
        off += N - j
    return np.array(out)


def _run(pkg, ctx, oracle, fred, g, kind, B=128, burn=1000, keep=2000, chunk=50, perturb=None):
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    thisT = len(fred["ydates"])
    rows, cols, tsel = g["sel_rows"], g["sel_cols"], list(g["tsel"])
    if kind == "linear":
        m = pkg.model.build_var(thisT, 12, 12, fred["data"], fred["ydates"], mpm, True)
        if perturb is not None:
            m = perturb(m)
        ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=B, crn=False, store_capacity=chunk, seed=31337)
    else:
        ndxS, ndxO, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
        e0 = pkg.model.elbT0_of(fred["data"], ndxS, 0.25, 12)
        bm = pkg.model.build_bh(thisT, 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0, True)
        m = bm.var
        ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=B, crn=False, store_capacity=chunk, seed=31337,
                        model=pkg.MODEL_BLOCKHYBRID, Ns=len(bm.ndxS), elbTmax=bm.elbT, elb_gibbsburn=100,
                        elb=0.25)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    if kind == "bh":
        ch.set_elb_model(bm.ndxS, bm.actual_block)
        ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
        ch.set_elb_ps(1000, -(-burn // 2))                  # m >= MCMCburnin / 2 (:435)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(burn)
    N = m.N
    dix = _vech_diag_index(N)
    sums = None
    for done in range(0, keep, chunk):
        ch.sweep(chunk, store=True)
        d = ch.get_draws()
        P = d["PAI_all"][:, rows, cols, :]                                  # M x nsel x B
        A = np.linalg.inv(np.moveaxis(d["invA_all"], 3, 1))                 # M x B x N x N
        asub = np.moveaxis(A[:, :, np.arange(1, N), np.arange(N - 1)], 1, 2)
        phi = d["PHI_all"][:, dix, :]
        sq = d["sqrtht_all"][:, tsel, :, :].reshape(chunk, len(tsel) * N, B, order="F")
        parts = [P, asub, phi, sq]
        if kind == "bh":
            sr = d["shadowrate_all"].reshape(chunk, -1, B, order="F")[:, g["cells"], :]
            parts.append(sr)
        Q = np.concatenate(parts, axis=1)                                   # M x nq x B
        s = Q.sum(axis=0)
        sums = s if sums is None else sums + s
    status = ch.get_status()
    acc = None
    if kind == "bh":
        ps = ch.get_ps()
        acc = float((ps["countAccept"].sum() + ps["countAcceptBurnin"].sum()) / (B * (burn + keep - burn // 2)))
    ch.close()
    assert not np.any(status & ~65), status
    return sums / keep, acc                                                # nq x B chain means


def _zscores(g, means):
    B = means.shape[1]
    m_gpu = means.mean(axis=1)
    nse_gpu = means.std(axis=1, ddof=1) / np.sqrt(B)
    se_o = np.maximum(g["nse3"], g["se_between"]) if "se_between" in g else g["nse3"]
    return (m_gpu - g["pmean"]) / np.sqrt(se_o ** 2 + nse_gpu ** 2), m_gpu, nse_gpu, se_o


@pytest.mark.parametrize("name", ["minnesota_precision_x1.5", "phi_prior_scale_x2"])
def test_mcse_detects_a_perturbed_sampler(pkg, ctx, oracle, fred, name):
    """Power of the posterior-level check: the same device run with ONE sampler detail changed
    (the Minnesota prior precision iV scaled by 1.5, i.e. theta by 1/sqrt(1.5), mcmcVAR.m:129-150;
    or the inverse-Wishart scale s_PHI doubled, mcmcVAR.m:165) must fail the 4.5-sigma bar that
    the unperturbed sampler passes (test_real_data_posterior_means_within_mcse)."""
    import dataclasses
    g = _fixture("linear")

    def perturb(m):
        if name.startswith("minnesota"):
            return dataclasses.replace(m, iVdiag=m.iVdiag * 1.5, iVb=m.iVb * 1.5)
        return dataclasses.replace(m, sPHI=m.sPHI * 2.0)

    means, _ = _run(pkg, ctx, oracle, fred, g, "linear", burn=int(g["burn"]), keep=int(g["keep"]), perturb=perturb)
    z = _zscores(g, means)[0]
    print(f"{name}: max |z| {np.abs(z).max():.1f}, {int(np.sum(np.abs(z) > 4.5))} of {z.size} quantities beyond 4.5")
    assert np.abs(z).max() > 4.5


@pytest.mark.parametrize("kind", ["linear", "bh"])
def test_real_data_posterior_means_within_mcse(pkg, ctx, oracle, fred, kind):
    g = _fixture(kind)
    # the oracle's kept window (sweeps burn .. burn + keep): slow directions (the intercepts of
    # the bh model) still drift after 1000 sweeps, so both sides average the same window
    means, acc = _run(pkg, ctx, oracle, fred, g, kind, burn=int(g["burn"]), keep=int(g["keep"]))
    B = means.shape[1]
    m_gpu = means.mean(axis=1)
    nse_gpu = means.std(axis=1, ddof=1) / np.sqrt(B)
    # pooled fixtures (several independent oracle chains): the oracle side's standard error is the
    # larger of the pooled spectral NSE and the spread of the chain means
    se_o = np.maximum(g["nse3"], g["se_between"]) if "se_between" in g else g["nse3"]
    z = (m_gpu - g["pmean"]) / np.sqrt(se_o ** 2 + nse_gpu ** 2)
    print(f"{kind}: {z.size} quantities, max |z| {np.abs(z).max():.2f}, median |z| {np.median(np.abs(z)):.2f}"
          + ("" if acc is None else f", device PS accept rate {acc:.3f}, oracle {_oracle_accept(g):.3f}"))
    for q in np.argsort(-np.abs(z))[:5]:
        print(f"  q{q}: gpu {m_gpu[q]:.5f} +- {nse_gpu[q]:.5f}  oracle {g['pmean'][q]:.5f} +- {se_o[q]:.5f}"
              f"  z {z[q]:.2f}")
    assert np.abs(z).max() < 4.5, np.round(z, 2)
