#!/usr/bin/env python
"""Measure the internal association and rounding of v_mfma_f64_16x16x4_f64.

D(i,j) = C(i,j) + sum_k A(i,k) B(k,j) is evaluated on the device for probes built to
separate the candidate evaluation orders (cancellation patterns such as 1, 2^-53, -1,
2^-53 along k, products that are not representable, accumulators that cancel the
leading part of the products), then compared entry by entry against every candidate
model evaluated exactly on the host (fractions, one correctly rounded step per
model operation).  The model that matches every entry is the one the oracle's mirrored
Gram (oracle/gram_mirror.c) must follow.

Usage: python tools/probe_mfma_order.py [--out gpurun_out/mfma_probe.npz]
"""
from __future__ import annotations

import argparse
import itertools
import sys
from fractions import Fraction
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def r(x: Fraction) -> Fraction:
    """Round an exact rational to the nearest double (ties to even)."""
    return Fraction(float(x))


def models():
    """name -> f(c, p[4] exact products, q[4] rounded products) -> Fraction."""
    out = {}
    for perm in itertools.permutations(range(4)):
        tag = "".join(map(str, perm))

        def seq(c, p, q, perm=perm):          # d = c; d = fma(a_k, b_k, d) in order perm
            d = c
            for k in perm:
                d = r(d + p[k])
            return d

        def seq_clast(c, p, q, perm=perm):    # s = sum in order perm (each step fused), then + c
            s = p[perm[0]]
            s = r(s)
            for k in perm[1:]:
                s = r(s + p[k])
            return r(s + c)

        def seq_rp(c, p, q, perm=perm):       # products rounded, then added in order perm
            d = c
            for k in perm:
                d = r(d + q[k])
            return d
        out[f"fma_seq_{tag}"] = seq
        out[f"sum_then_c_{tag}"] = seq_clast
        out[f"rprod_seq_{tag}"] = seq_rp
    out["exact_single_round"] = lambda c, p, q: r(c + sum(p))
    out["exact_prods_round_then_c"] = lambda c, p, q: r(r(sum(p)) + c)
    out["tree_exact_pairs"] = lambda c, p, q: r(r(r(p[0] + p[1]) + r(p[2] + p[3])) + c)
    out["tree_pairs_c_inner"] = lambda c, p, q: r(r(p[0] + p[1] + c) + r(p[2] + p[3]))
    out["tree_rprod"] = lambda c, p, q: r(r(r(q[0] + q[1]) + r(q[2] + q[3])) + c)
    out["rprod_exact_sum"] = lambda c, p, q: r(c + sum(q))
    out["pairs_fused_seq"] = lambda c, p, q: r(r(c + p[0] + p[1]) + p[2] + p[3])
    out["pairs_fused_seq_rev"] = lambda c, p, q: r(r(c + p[2] + p[3]) + p[0] + p[1])
    return out


def make_probes(P: int, seed: int = 0):
    """P probes (16 x 4, 4 x 16, 16 x 16 each), column-major like the device selftest."""
    rng = np.random.default_rng(seed)
    A = np.zeros((16, 4, P))
    B = np.zeros((4, 16, P))
    C = np.zeros((16, 16, P))
    u = 2.0 ** -53
    for q in range(P):
        kind = q % 6
        if kind == 0:   # one-hot products against an accumulator that cancels the leading part
            a = 1.0 + rng.integers(1, 2 ** 20, (16, 4)) * 2.0 ** -40
            b = 1.0 + rng.integers(1, 2 ** 20, (4, 16)) * 2.0 ** -40
            mask = np.zeros((16, 4))
            mask[np.arange(16), rng.integers(0, 4, 16)] = 1.0
            A[..., q] = a * mask
            B[..., q] = b
            C[..., q] = -(A[..., q] @ B[..., q])
        elif kind == 1:  # 1, u, -1, u along k in random positions (association probe)
            for i in range(16):
                perm = rng.permutation(4)
                A[i, :, q] = np.array([1.0, u, -1.0, u])[perm] * rng.choice([1.0, -1.0])
            B[..., q] = rng.choice([1.0, 1.0 + 2.0 ** -52, 1.0 - 2.0 ** -53, 0.5, 3.0], (4, 16))
            C[..., q] = rng.choice([0.0, u, -u, 1.0, -1.0, 0.25 * u], (16, 16))
        elif kind == 2:  # big/small mixtures of the magnitudes of the products
            A[..., q] = rng.choice([1.0, 2.0 ** 30, 2.0 ** -30, 1.0 + 2.0 ** -50], (16, 4)) * \
                rng.choice([1.0, -1.0], (16, 4))
            B[..., q] = rng.choice([1.0, 2.0 ** 29, 2.0 ** -31, 1.0 - 2.0 ** -51], (4, 16)) * \
                rng.choice([1.0, -1.0], (4, 16))
            C[..., q] = rng.choice([0.0, 1.0, -1.0, 2.0 ** 59, -2.0 ** 59], (16, 16))
        elif kind == 3:  # random with a cancelling accumulator
            A[..., q] = rng.standard_normal((16, 4))
            B[..., q] = rng.standard_normal((4, 16))
            C[..., q] = -(A[..., q] @ B[..., q]) * (1.0 + rng.standard_normal((16, 16)) * 1e-12)
        elif kind == 4:  # random, wide exponent range
            A[..., q] = rng.standard_normal((16, 4)) * 2.0 ** rng.integers(-20, 20, (16, 4))
            B[..., q] = rng.standard_normal((4, 16)) * 2.0 ** rng.integers(-20, 20, (4, 16))
            C[..., q] = rng.standard_normal((16, 16)) * 2.0 ** rng.integers(-20, 20, (16, 16))
        else:            # Gram-like: positive weights times data of mixed sign
            A[..., q] = rng.standard_normal((16, 4)) * 3.0
            B[..., q] = rng.standard_normal((4, 16)) * 3.0
            C[..., q] = rng.standard_normal((16, 16)) * 50.0
    return A, B, C


def evaluate(A, B, C, D, names=None):
    """Per model: number of probe entries it reproduces bit for bit."""
    ms = models()
    if names is not None:
        ms = {k: v for k, v in ms.items() if k in names}
    P = A.shape[2]
    hits = {k: 0 for k in ms}
    total = 0
    for q in range(P):
        for i in range(16):
            for j in range(16):
                a = [Fraction(float(A[i, k, q])) for k in range(4)]
                b = [Fraction(float(B[k, j, q])) for k in range(4)]
                p = [a[k] * b[k] for k in range(4)]
                qq = [r(x) for x in p]
                c = Fraction(float(C[i, j, q]))
                d = D[i, j, q]
                total += 1
                for k, f in ms.items():
                    if float(f(c, p, qq)) == d or (np.isnan(d) and False):
                        hits[k] += 1
    return hits, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--probes", type=int, default=60)
    ap.add_argument("--out", default="gpurun_out/mfma_probe.npz")
    args = ap.parse_args()
    import __graft_entry__ as ge
    pkg = ge.load_package()
    ctx = pkg.Context(0)
    A, B, C = make_probes(args.probes)
    D = ctx.selftest_mfma_f64_acc(A, B, C)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez(args.out, A=A, B=B, C=C, D=D)
    hits, total = evaluate(A, B, C, D)
    best = sorted(hits.items(), key=lambda kv: -kv[1])
    print(f"{total} probe entries")
    for k, v in best[:12]:
        print(f"  {k:28s} {v:6d} {'ALL' if v == total else ''}")


if __name__ == "__main__":
    main()
