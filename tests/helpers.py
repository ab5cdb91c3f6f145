"""Shared test inputs: synthetic VAR data (toy sizes) and chain states."""
import numpy as np


def synth_var_data(N=4, p=2, Tobs=62, seed=0):
    """A stable VAR(p) sample with stochastic volatility (Nobs x N)."""
    rng = np.random.default_rng(seed)
    Pi = [0.5 * np.eye(N) + rng.uniform(-0.05, 0.05, (N, N))]
    Pi += [(0.2 / l ** 2) * np.eye(N) for l in range(2, p + 1)]
    y = np.zeros((Tobs, N))
    y[:p] = rng.standard_normal((p, N))
    lh = np.zeros(N)
    for t in range(p, Tobs):
        lh = lh + 0.1 * rng.standard_normal(N)
        y[t] = 0.3 + sum(Pi[l] @ y[t - 1 - l] for l in range(p)) + np.exp(lh / 2) * rng.standard_normal(N)
    return y


def toy_setup(oracle, N=4, p=2, Tobs=62, seed=0):
    data = synth_var_data(N, p, Tobs, seed)
    ydates = np.arange(Tobs, dtype=float)
    mpm = np.ones(N)
    return oracle.var_setup(Tobs, p, 12, data, ydates, mpm, True)


def random_state(oracle, su, seed=1):
    """A chain state away from the reference initialisation: smooth volatility,
    non-trivial A (well conditioned posterior precision)."""
    rng = np.random.default_rng(seed)
    N, T = su.N, su.T
    st = oracle.init_state(su)
    A = np.eye(N) + np.tril(rng.uniform(-0.3, 0.3, (N, N)), -1)
    h = np.cumsum(0.05 * rng.standard_normal((T, N)), axis=0) + np.log(np.var(su.Y, axis=0))
    st["A"] = A
    st["h"] = h
    st["sqrtht"] = np.exp(h / 2)
    L = np.tril(rng.uniform(-0.02, 0.02, (N, N)), -1) + np.diag(rng.uniform(0.05, 0.15, N))
    st["sqrtPHI"] = L
    return st


def crn_flat(oracle, crn, su):
    return np.concatenate([crn[k].ravel(order="F") for k, _ in oracle.crn_sizes(su.N, su.K, su.T,
                                                                                 su.dPHI)])


def synth_bh_data(N=5, p=2, Tobs=150, elb_window=(80, 120), ndxS=(2, 3), seed=3, elb=0.25):
    """Toy block-hybrid data: a VAR sample whose shadow-rate variables sit at or
    below the ELB (mixed censoring across the Ns rates) inside ``elb_window``."""
    y = synth_var_data(N, p, Tobs, seed)
    rng = np.random.default_rng(seed + 1)
    a, b = elb_window
    for k, s in enumerate(ndxS):
        y[:a, s] = 2.0 + np.abs(y[:a, s])               # above the ELB before the window
        y[a:b, s] = elb - rng.uniform(0.01, 0.2, b - a)  # censored
        if k % 2 == 1:                                   # second rate: a few uncensored months
            y[a + 5:b:7, s] = elb + rng.uniform(0.05, 0.3, len(range(a + 5, b, 7)))
        y[b:, s] = elb + 0.5 + np.abs(y[b:, s])
    return y


def toy_bh_setup(bh, N=5, p=2, Tobs=150, ndxS=(2, 3), ndxO=(4,), seed=3, elb=0.25):
    data = synth_bh_data(N, p, Tobs, ndxS=ndxS, seed=seed, elb=elb)
    ydates = np.arange(Tobs, dtype=float)
    hit = np.any(data[:, list(ndxS)] <= elb, axis=1)
    elbT0 = int(np.argmax(hit)) - p
    return bh.bh_setup(Tobs, p, 12, data, ydates, np.asarray(ndxS), np.asarray(ndxO), np.ones(N),
                       elb, elbT0)


def bh_crn_flat(bh, crn, bs):
    return np.concatenate([crn[k].ravel(order="F") for k, _ in bh.bh_crn_sizes(bs)])


def toy_hybrid_setup(hy, N=5, p=2, Tobs=150, ndxS=(2, 3), seed=3, elb=0.25):
    """Toy hybrid model (mcmcVARhybridGibbs.m) on the block-hybrid toy data."""
    data = synth_bh_data(N, p, Tobs, ndxS=ndxS, seed=seed, elb=elb)
    ydates = np.arange(Tobs, dtype=float)
    hit = np.any(data[:, list(ndxS)] <= elb, axis=1)
    elbT0 = int(np.argmax(hit)) - p
    return hy.hybrid_setup(Tobs, p, 12, data, ydates, np.asarray(ndxS), np.ones(N), elb, elbT0)


def hybrid_crn_flat(hy, crn, hs):
    return np.concatenate([crn[k].ravel(order="F") for k, _ in hy.hybrid_crn_sizes(hs)])
