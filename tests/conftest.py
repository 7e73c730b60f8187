import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIX = os.path.join(ROOT, "tests", "fixtures")
GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def sup():
    import superman_amd
    superman_amd._lib.load()
    return superman_amd


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.load()
    return oracle


def fixture_path(name: str) -> str:
    return os.path.join(FIX, name)


def rel(a: float, b: float) -> float:
    if a == b:
        return 0.0
    return abs(a - b) / max(abs(a), abs(b), 1e-300)


def seg_skip_fraction(sup, a, kernel="sparse"):
    """Fraction of wave-chunks whose rows untouched by the walk bits (the
    segmented walk's outer-tree tail) hold an exact zero in every lane, i.e. the
    chunks the generated kernel skips; restated from the plan's column map in
    numpy (x0 = a[:, n-1] - rowsum / 2, chunk-start Gray state of the lane and
    chunk bits)."""
    return float(seg_skipped_chunks(sup, a, kernel).mean())


def seg_skipped_chunks(sup, a, kernel="sparse"):
    """Per wave-chunk (index order): True when the segmented kernel skips it."""
    n = a.shape[0]
    info = sup.plan_info(a, kernel, jit=1)
    cm, L, m = [int(c) for c in info["colmap"]], info["L"], info["m"]
    x0 = a[:, n - 1] - a.sum(1) / 2
    rest = [j for j in range(n) if not a[j, cm[L:L + m]].any()]
    if not rest:
        return np.zeros(1 << (n - 1 - L - m), bool)
    cols = cm[:L] + cm[L + m:]
    h = len(cols) - L
    # x = x0 + sum_k bit_k(gray(p)) a[:, cols[k]] with p = (chunk << L) | lane:
    # bits >= L are gray(chunk), bits < L depend on the lane and chunk & 1
    # (integer matrices: every sum is exact, so the split does not change a bit)
    ar = a[rest].astype(np.float64)
    ch = np.arange(1 << h, dtype=np.int64)
    gc = ch ^ (ch >> 1)
    xc = np.tile(x0[rest].astype(np.float64), (1 << h, 1))
    for k in range(h):
        xc += ((gc >> k) & 1)[:, None] * ar[:, cols[L + k]][None, :]
    allz = np.ones(1 << h, bool)
    for par in (0, 1):
        sel = (ch & 1) == par
        xp = xc[sel]
        az = np.ones(len(xp), bool)
        for lane in range(1 << L):
            pl = lane | (par << L)
            gl = pl ^ (pl >> 1)
            xl = sum(((gl >> k) & 1) * ar[:, cols[k]] for k in range(L)) if L else 0.0
            az &= ((xp + xl) == 0).any(1)
        allz[sel] = az
    return allz
