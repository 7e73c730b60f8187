"""Exact integer permanent (sup_perman_exact; superman_amd/csrc/exact.cpp,
walk_exact.hip) on host threads — no GPU needed.

The reference computes int and -b (binary) inputs in fp64 (rounded beyond
2^53); the exact path evaluates the same Ryser / Gray walk of 2A in residue
arithmetic and joins the residues by CRT.  Checked against:
* known answers (J_n = n!, permutation matrices, a zero row);
* exact rational Ryser (oracle.exact_perman, independent Python) for n <= 10;
* an independent plain-Ryser CRT oracle (oracle.c orc_exact_mod + Python
  CRT, other primes) for n up to 20, negative entries included;
* the reference's own __float128 results (goldens from the compiled
  reference): the exact integer rounded to fp64 equals the reference's quad
  result rounded to fp64, bit for bit, on every synthetic int matrix (n <= 22;
  the reference's own fp64 results already differ from n = 16 on).
"""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, fixture_path


def _rand(n, d, seed, lo=1, hi=6):
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < d
    mask[np.arange(n), rng.permutation(n)] = True
    return np.where(mask, rng.integers(lo, hi, (n, n)), 0).astype(np.int32)


def test_known_answers(sup):
    for n in range(1, 13):
        assert sup.perman_exact(np.ones((n, n), np.int32), cpu=True, threads=4) == math.factorial(n)
    p = np.eye(15, dtype=np.int32)[np.random.default_rng(0).permutation(15)]
    assert sup.perman_exact(p, cpu=True, threads=4) == 1
    z = _rand(12, 0.5, 1)
    z[4, :] = 0
    assert sup.perman_exact(z, cpu=True, threads=4) == 0
    # J_20: 20! > 2^53, exact
    assert sup.perman_exact(np.ones((20, 20), np.int32), cpu=True, threads=8) == math.factorial(20)


@pytest.mark.parametrize("n,seed", [(5, 1), (8, 2), (10, 3)])
def test_vs_rational_ryser(sup, orc, n, seed):
    a = _rand(n, 0.6, seed, -4, 5)  # negative entries too
    assert sup.perman_exact(a, cpu=True, threads=4) == orc.exact_perman(a)


@pytest.mark.parametrize("n,d,lo,hi,seed", [(14, 0.5, 1, 6, 4), (16, 0.3, -5, 6, 5), (18, 0.5, 0, 2, 6),
                                            (20, 0.5, 1, 6, 7)])
def test_vs_crt_oracle(sup, orc, n, d, lo, hi, seed):
    a = _rand(n, d, seed, lo, hi)
    got = sup.perman_exact(a, cpu=True, threads=8)
    assert got == orc.exact_perman_crt(a, 8)
    # same value whatever the storage type
    assert sup.perman_exact(a.astype(np.float64), cpu=True, threads=8) == got
    # and within fp64 rounding of the fp64 walk
    f = sup.perman_cpu(a.astype(np.float64), "dense", threads=8)
    assert abs(f - got) <= 1e-10 * max(abs(got), 1)


def test_vs_reference_quad_goldens(sup, golden):
    names = sorted({k.split("|")[0] for k in golden if k.startswith("synth/") and "_int" in k})
    checked = 0
    for nm in names:
        q = golden.get(f"{nm}|dense_q|r0|b0|t4")
        if q is None:
            continue
        a = sup.read_matrix(fixture_path(nm))[0]
        e = sup.perman_exact(a, cpu=True, threads=8)
        assert float(e) == q, (nm, e, q)  # the reference's quad result, rounded to fp64, bit for bit
        checked += 1
    assert checked >= 20  # n = 1 .. 22; the reference's fp64 results are inexact from n = 16


def test_rejects_non_integers(sup):
    a = np.ones((6, 6))
    a[2, 3] = 0.5
    with pytest.raises(sup.SupError):
        sup.perman_exact(a, cpu=True)
    b = np.ones((6, 6))
    b[0, 0] = 2.0 ** 40
    with pytest.raises(sup.SupError):
        sup.perman_exact(b, cpu=True)


def test_cli_exact(sup, tmp_path):
    a = _rand(14, 0.5, 9)
    path = tmp_path / "m14"
    nz = np.argwhere(a != 0)
    with open(path, "w") as f:
        f.write(f"14 {len(nz)} int\n")
        for i, j in nz:
            f.write(f"{i} {j} {a[i, j]}\n")
    exe = os.path.join(ROOT, "superman_amd", "bin", "perman")
    out = subprocess.run([exe, "-f", str(path), "-c", "-E", "-t", "4"], capture_output=True, text=True, check=True)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("Permanent:")][0]
    assert int(line.split()[1]) == sup.perman_exact(a, cpu=True, threads=4)
    # -b: every listed entry is 1 (util.h:343-358)
    out = subprocess.run([exe, "-f", str(path), "-c", "-E", "-b", "-t", "4"], capture_output=True, text=True,
                         check=True)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("Permanent:")][0]
    assert int(line.split()[1]) == sup.perman_exact((a != 0).astype(np.int32), cpu=True, threads=4)


def test_large_entries_vs_crt_oracle(sup, orc):
    """6-digit decimals scaled to integers (the corpus ground-truth use): row
    sums near 2^28, so the residue chain runs with small primes and must reduce
    before its first product."""
    rng = np.random.default_rng(11)
    for n in (9, 13):
        a = np.where(rng.random((n, n)) < 0.6, rng.integers(1, 5_000_000, (n, n)), 0).astype(np.int64)
        a[np.arange(n), rng.permutation(n)] = 4_999_999
        got = sup.perman_exact(a.astype(np.float64), cpu=True, threads=8)
        assert got == orc.exact_perman_crt(a, 8)


def test_tiny_and_degenerate(sup, orc):
    for a in (np.array([[5]]), np.array([[-7]]), np.array([[1, 2], [3, 4]]), np.zeros((2, 2)),
              np.array([[1, -1, 2], [0, 3, -4], [5, 6, -7]]), np.zeros((5, 5))):
        assert sup.perman_exact(a.astype(np.int32), cpu=True, threads=2) == orc.exact_perman(a)


def test_reduced_exact_vs_direct(sup, orc, tmp_path):
    """-o with exact leaves: the d1/d2/d34 tree folds its coefficients into the
    integer leaves, so the exact leaf permanents add up to the exact permanent."""
    rng = np.random.default_rng(3)
    n = 26
    a = np.where(rng.random((n, n)) < 0.12, rng.integers(1, 4, (n, n)), 0).astype(np.int32)
    a[np.arange(n), rng.permutation(n)] = 1
    r, st = sup.perman_reduced_exact(a, cpu=True, threads=8, min_n=12, return_stats=True)
    assert st["leaves"] > 10
    assert r == sup.perman_exact(a, cpu=True, threads=8) == orc.exact_perman_crt(a, 8)
    # CLI -o -E (singleton compression, then one leaf at this size)
    path = tmp_path / "m26"
    nz = np.argwhere(a != 0)
    with open(path, "w") as f:
        f.write(f"{n} {len(nz)} int\n")
        for i, j in nz:
            f.write(f"{i} {j} {a[i, j]}\n")
    exe = os.path.join(ROOT, "superman_amd", "bin", "perman")
    out = subprocess.run([exe, "-f", str(path), "-c", "-E", "-o", "-t", "8"], capture_output=True, text=True,
                         check=True)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("Permanent:")][0]
    assert int(line.split()[1]) == r
    with pytest.raises(sup.SupError):
        sup.perman_reduced_exact(a.astype(np.float64) + 0.5, cpu=True)


def test_exact_corpus_integers_consistent():
    """tests/golden/exact_corpus.json: every committed exact integer (the GPU
    residue walk's output, profiles/r3/probe_exact_truth.log) divided by its
    decimal scale rounds to the committed fp64 value the -m gpu tests pin the
    benchmarked walks against (tests/test_gpu_pinned.py)."""
    import json
    import os
    from fractions import Fraction

    from conftest import ROOT, fixture_path
    ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
    assert set(ex["_integers"]) >= {"double__32_0.50_0", "double__36_0.20_0", "double__40_0.90_0",
                                    "synth44_0.15_int"}
    for name, rec in ex["_integers"].items():
        with open(fixture_path(name)) as f:
            n = int(f.readline().split()[0])
        scale = 1 if rec["scale"] == "1" else 10 ** (6 * n)
        assert float(Fraction(int(rec["integer"]), scale)) == ex[name]


def test_exact_corpus_vs_reference_quad(golden):
    """The exact permanents the benchmarked walks are pinned to
    (tests/golden/exact_corpus.json, this engine's residue walk + CRT) against
    the reference's own -q mode (parallel_perman64<__float128,double>,
    rev/cpu_algos.hpp:761-873, compiled from its sources; tests/golden/
    make_golden.py) wherever the reference ran it: n = 30 and, since round 6,
    BASELINE config 2's n = 32 matrix (906 s on 8 cores).  The quad results
    are printed with 17 digits, so they agree with the exact value to within
    an ulp or two of fp64; the reference's own fp64 result is ~1e-10 away."""
    import json
    import os

    from conftest import ROOT
    ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
    checked = 0
    for name in ("double__30_0.50_0", "double__32_0.50_0"):
        q = golden[f"{name}|dense_q|r0|b0|t8"]
        e = ex[name]
        assert abs(q - e) <= 4.5e-16 * abs(e), (name, q, e)
        f64 = golden[f"{name}|dense|r0|b0|t8"]
        assert abs(f64 - e) > 1e-12 * abs(e)  # the reference's fp64 walk is the inaccurate side
        checked += 1
    assert checked == 2
