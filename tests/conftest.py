import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import __graft_entry__  # noqa: E402

CSV = ROOT / "tests" / "golden" / "data" / "fredblockMD20-2022-09.csv"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libccmm kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def pkg():
    return __graft_entry__.load_package()


@pytest.fixture(scope="session")
def oracle():
    from oracle import ccmm_oracle
    return ccmm_oracle


@pytest.fixture(scope="session")
def fred(oracle):
    return oracle.load_fred_csv(CSV)


@pytest.fixture(scope="session")
def ctx(pkg):
    return pkg.Context(0)


def rel_err(got, want, scale=None):
    """max |got - want| / max(|want|, scale) — the parity metric of SURVEY.md §7/§8c."""
    got = np.asarray(got, float)
    want = np.asarray(want, float)
    den = np.abs(want)
    if scale is not None:
        den = np.maximum(den, np.broadcast_to(scale, den.shape))
    den = np.where(den == 0, 1.0, den)
    return float(np.max(np.abs(got - want) / den))
