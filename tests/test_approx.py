"""Randomized estimators (reference -a / -i) on the host.

* oracle/approx.py restates the estimators (kernel_rasmussen /
  kernel_approximation, gpu_approximation_dense.cu:155-371) with Philox4x32-10,
  itself checked against the published known-answer vectors; the engine's
  64-sample block sums must match it bit for bit;
* the estimators are unbiased for the permanent of the 0/1 pattern: on
  matrices with an exactly known permanent the estimate lies within 5 standard
  errors (seeded, so the check is deterministic);
* grid graphs (util.h:403-520): the permanent equals the number of domino
  tilings, counted independently by a transfer matrix.
"""
import subprocess

import numpy as np
import pytest

from conftest import rel
from oracle import approx as A


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert A.philox4x32_10((0, 0, 0, 0), (0, 0)) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert A.philox4x32_10((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF)) == (0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                            0x6D5451FD)
    assert A.philox4x32_10((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)) == (
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)


def _mats():
    rng = np.random.default_rng(21)
    out = []
    for n, d in ((6, 0.6), (9, 0.45), (12, 0.35)):
        a = (rng.random((n, n)) < d).astype(np.int32)
        a[np.arange(n), rng.permutation(n)] = 1
        out.append(a)
    return out


@pytest.mark.parametrize("algo,method", [(1, "rasmussen"), (2, "scaling")])
def test_block_sums_match_restatement(sup, algo, method):
    for a in _mats():
        want = A.block_sums(a, method, seed=7, block=0)
        got, st = sup.approx(a, algo, samples=64, seed=7, cpu=True, threads=2, return_stats=True)
        assert st["samples"] == 64
        assert got == want[0] / 64.0
        assert st["zero_fraction"] == want[2] / 64.0


@pytest.mark.parametrize("algo", [1, 2])
def test_unbiased_on_known_permanents(sup, orc, algo):
    for a in _mats() + [np.ones((7, 7), np.int32), np.eye(10, dtype=np.int32)]:
        exact = float(orc.exact_perman((a != 0).astype(np.int64)))
        est, st = sup.approx(a, algo, samples=64 * 4000, seed=3, cpu=True, threads=8, return_stats=True)
        if st["std_error"] == 0.0:
            assert est == exact  # J_n / permutation matrices: every sample is exact
        else:
            assert abs(est - exact) < 5 * st["std_error"], (a.shape, est, exact, st["std_error"])
    # values are ignored: the estimators target the permanent of the pattern
    a = _mats()[1]
    b = a * np.random.default_rng(4).integers(1, 9, a.shape)
    assert sup.approx(a, algo, samples=640, seed=9, cpu=True) == sup.approx(b.astype(np.int32), algo, samples=640,
                                                                            seed=9, cpu=True)


def test_reproducible_across_threads_and_seeds(sup):
    g = sup.grid_graph(6, 6)
    r1 = sup.approx(g, 2, samples=5000, seed=11, cpu=True, threads=1)
    r8 = sup.approx(g, 2, samples=5000, seed=11, cpu=True, threads=8)
    assert r1 == r8
    assert sup.approx(g, 2, samples=5000, seed=12, cpu=True, threads=8) != r8
    assert sup.approx(g, 1, samples=5000, seed=11, cpu=True) == sup.approx(g, 3, samples=5000, seed=11, cpu=True)


def test_grid_graph_counts_tilings(sup):
    for m, n in ((2, 2), (2, 3), (3, 4), (4, 4), (4, 6), (6, 6), (5, 6), (8, 8), (6, 10)):
        g = sup.grid_graph(m, n)
        assert g.shape == (m * n // 2, m * n // 2)
        t = A.domino_tilings(m, n)
        if g.shape[0] <= 30:
            assert sup.perman_cpu(g, threads=8) == t, (m, n)
        est, st = sup.approx(g, 1, samples=64 * 3000, seed=5, cpu=True, threads=8, return_stats=True)
        assert abs(est - t) < 5 * st["std_error"] + 1e-9 * t, (m, n, est, t)
    with pytest.raises(sup.SupError):
        sup.grid_graph(3, 5)  # both odd: no perfect matching layout (util.h:404-407)


def test_large_sparse_grid(sup):
    # 36 x 36 is the reference's default -i board (nov = 648: 16-word bitsets)
    g = sup.grid_graph(12, 12)
    t = A.domino_tilings(12, 12)
    est, st = sup.approx(g, 1, samples=64 * 400, seed=2, cpu=True, threads=8, return_stats=True)
    assert abs(est - t) < 5 * st["std_error"]
    big = sup.grid_graph(36, 36)
    assert big.shape == (648, 648) and big.sum() == 2 * 36 * 35
    est, st = sup.approx(big, 1, samples=128, seed=1, cpu=True, threads=8, return_stats=True)
    assert st["samples"] == 128 and np.isfinite(est)


def test_cli_approx(sup):
    exe = sup._lib.PERMAN_BIN
    r = subprocess.run([exe, "-i", "-m", "4", "-n", "6", "-c", "-p1", "-x", "6400", "-t", "4"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0].startswith("Result: rasmussen_sparse ") and lines[1].startswith("Try: rasmussen_sparse ")
    val = float(lines[2].split()[1])
    g = sup.grid_graph(4, 6)
    assert val == sup.approx(g, 1, samples=6400, seed=1, cpu=True)
    assert rel(val, 281.0) < 0.05
