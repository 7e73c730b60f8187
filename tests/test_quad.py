"""Double-double permanent (sup_perman_quad) on host threads — the host twin
of walk_dd.hip, the MI355X form of the reference's quad-precision calculation
(v2 `-q`, revised_perman/main.cpp:141-142 -> parallel_perman64<__float128,S>).

Pinned against the reference itself: every `dense_q` golden (the reference's
__float128 Ryser, compiled from its sources, tests/golden/make_golden.py) up
to n = 22 equals hi bit for bit once rounded to fp64; on integer matrices
hi + lo is the exact integer (checked against the exact residue path)."""
from fractions import Fraction

import numpy as np
import pytest

from conftest import fixture_path

QUAD_MAX_N_CPU = 22


def _quad_goldens(golden, max_n):
    out = []
    for k, q in sorted(golden.items()):
        if "|dense_q|" not in k or k.endswith("seconds"):
            continue
        out.append((k.split("|")[0], q))
    return out


def test_quad_host_matches_reference_quad_goldens(sup, golden):
    checked = 0
    for nm, q in _quad_goldens(golden, QUAD_MAX_N_CPU):
        a = sup.read_matrix(fixture_path(nm))[0]
        if a.shape[0] > QUAD_MAX_N_CPU:
            continue
        hi, lo = sup.perman_quad(a, cpu=True, threads=8)
        assert hi == q, (nm, hi, q)  # the reference's __float128 result, rounded once to fp64
        assert abs(lo) <= abs(hi) * 2.0 ** -52, nm  # normalised pair
        checked += 1
    assert checked >= 40


@pytest.mark.parametrize("n,lo_v,hi_v,seed", [(9, -3, 4, 1), (14, 1, 6, 2), (18, 0, 2, 3), (21, -5, 6, 4)])
def test_quad_host_int_is_exact(sup, n, lo_v, hi_v, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(lo_v, hi_v, (n, n)).astype(np.int32)
    hi, lo = sup.perman_quad(a, cpu=True, threads=8)
    e = sup.perman_exact(a, cpu=True, threads=8)
    if abs(e) < 2 ** 100:
        assert Fraction(hi) + Fraction(lo) == e
    else:
        assert abs(Fraction(hi) + Fraction(lo) - e) <= abs(e) * Fraction(1, 2 ** 100)


def test_quad_host_thread_invariance(sup):
    a = sup.read_matrix(fixture_path("synth/20_0.50_double"))[0]
    r1 = sup.perman_quad(a, cpu=True, threads=1)
    assert r1 == sup.perman_quad(a, cpu=True, threads=7) == sup.perman_quad(a, cpu=True, threads=16)


def test_quad_tiny_and_degenerate(sup):
    assert sup.perman_quad(np.array([[2.5]]), cpu=True) == (2.5, 0.0)
    assert sup.perman_quad(np.array([[1.0, 2.0], [3.0, 4.0]]), cpu=True)[0] == 10.0
    z = np.ones((6, 6))
    z[3] = 0.0
    assert sup.perman_quad(z, cpu=True)[0] == 0.0
    # 0.1 is not representable: the double-double start vector keeps the digits the fp64 one rounds away
    a = np.full((12, 12), 0.1)
    hi, lo = sup.perman_quad(a, cpu=True)
    want = Fraction(479001600) * Fraction(0.1) ** 12
    assert abs(Fraction(hi) + Fraction(lo) - want) <= want * Fraction(1, 2 ** 95)


def test_reduced_quad_int_is_exact(sup):
    """-o with double-double leaves and combine: on an integer matrix the d1/d2/d34
    leaves are integer matrices, so hi + lo is the exact permanent."""
    rng = np.random.default_rng(3)
    n = 26
    a = np.where(rng.random((n, n)) < 0.12, rng.integers(1, 4, (n, n)), 0).astype(np.int32)
    a[np.arange(n), rng.permutation(n)] = 1
    (hi, lo), st = sup.perman_reduced_quad(a, cpu=True, threads=8, min_n=12, return_stats=True)
    assert st["leaves"] > 10
    assert Fraction(hi) + Fraction(lo) == sup.perman_reduced_exact(a, cpu=True, threads=8, min_n=12)


def test_reduced_quad_scaled_vs_direct(sup):
    """-o -u: leaves scaled (scalesk) in fp64, factors divided out in double-double."""
    a = sup.read_matrix(fixture_path("mtx/can_24_ps.mtx"))[0]
    hi, lo = sup.perman_quad(a, cpu=True, threads=8)
    for scale in (None, 4):
        (rh, rl), st = sup.perman_reduced_quad(a, scale=scale, cpu=True, threads=8, min_n=20, return_stats=True)
        assert st["leaves"] >= 1
        assert abs(rh - hi) <= 1e-13 * abs(hi), (scale, rh, hi)


def test_cli_quad_cpu(sup, tmp_path):
    """perman -c -q (and with -o): the double-double lines of the CLI."""
    import os
    import subprocess
    rng = np.random.default_rng(5)
    n = 16
    a = np.where(rng.random((n, n)) < 0.3, rng.integers(1, 4, (n, n)), 0).astype(np.int32)
    a[np.arange(n), rng.permutation(n)] = 1
    path = tmp_path / "m16"
    nz = np.argwhere(a != 0)
    with open(path, "w") as f:
        f.write(f"{n} {len(nz)} int\n")
        for i, j in nz:
            f.write(f"{i} {j} {a[i, j]}\n")
    exe = os.path.join(os.path.dirname(sup.__file__), "bin", "perman")
    e = sup.perman_exact(a, cpu=True)
    for extra in ([], ["-o"]):
        out = subprocess.run([exe, "-f", str(path), "-c", "-q", "-t", "4"] + extra, capture_output=True, text=True,
                             check=True).stdout
        assert "cpu_perman64_quad" in out
        hi, lo = [float(v) for v in [l for l in out.splitlines() if l.startswith("Permanent (double-double)")][0]
                  .split(":")[1].split()]
        assert Fraction(hi) + Fraction(lo) == e


def test_cli_v2_precision_flags(sup, tmp_path):
    """v2's -w (single-precision storage: the permanent of the float-rounded
    entries), -h (single-precision calculation: computed in fp64 with a note)
    and -e <grid multiplier> (accepted, no effect): revised_perman/main.cpp
    :1431-1460."""
    import os
    import subprocess
    rng = np.random.default_rng(11)
    n = 14
    a = np.where(rng.random((n, n)) < 0.5, rng.random((n, n)) + 0.1, 0.0)
    a[np.arange(n), rng.permutation(n)] = 0.3
    path = tmp_path / "m14"
    nz = np.argwhere(a != 0)
    with open(path, "w") as f:
        f.write(f"{n} {len(nz)} double\n")
        for i, j in nz:
            f.write(f"{i} {j} {float(a[i, j])!r}\n")
    exe = os.path.join(os.path.dirname(sup.__file__), "bin", "perman")

    def hi_of(extra):
        r = subprocess.run([exe, "-f", str(path), "-c", "-q", "-t", "2"] + extra, capture_output=True, text=True,
                           check=True)
        line = [l for l in r.stdout.splitlines() if l.startswith("Permanent (double-double)")][0]
        return float(line.split(":")[1].split()[0]), r.stderr

    full, _ = hi_of([])
    single, _ = hi_of(["-w"])
    hi_f, _ = sup.perman_quad(a.astype(np.float32).astype(np.float64), cpu=True, threads=2)
    hi_d, _ = sup.perman_quad(a, cpu=True, threads=2)
    assert full == hi_d
    assert single == hi_f and single != full
    same, err = hi_of(["-h", "-e", "4"])
    assert same == full and "-h" in err
