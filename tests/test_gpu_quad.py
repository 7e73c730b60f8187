"""Double-double walk on the GPU (walk_dd.hip through sup_perman_quad), the
MI355X form of the reference's quad-precision calculation (v2 `-q`,
revised_perman/main.cpp:141-142, parallel_perman64<__float128,S>).

Bit-identical to its host twin (quad.cpp; same dd.hpp operations in the same
order); rounded to fp64 it equals the reference's own __float128 results at
n = 30; against exact ground truth (the residue path on 10^6 A for the 6-digit
decimal corpus) it carries ~1e-25 where the fp64 walks carry ~1e-12."""
import subprocess
from fractions import Fraction

import numpy as np
import pytest

from conftest import fixture_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu(sup):
    if sup.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")


@pytest.mark.parametrize("n,seed", [(1, 1), (2, 2), (5, 3), (13, 4), (20, 5), (24, 6)])
def test_gpu_quad_bit_identical_to_host_twin(sup, n, seed):
    rng = np.random.default_rng(seed)
    a = np.where(rng.random((n, n)) < 0.6, rng.uniform(-2.0, 5.0, (n, n)), 0.0)
    (hi, lo), st = sup.perman_quad(a, return_stats=True)
    assert st["devices_used"] == 1 and st["kernel_ms"] > 0
    assert (hi, lo) == sup.perman_quad(a, cpu=True, threads=16)
    assert (hi, lo) == sup.perman_quad(a, gpu_num=sup.device_count())


@pytest.mark.parametrize("name", ["double__30_0.20_0", "double__30_0.50_0", "int__30_0.20_0", "int__30_0.50_0"])
def test_gpu_quad_reference_quad_goldens_n30(sup, golden, name):
    a = sup.read_matrix(fixture_path(name))[0]
    q = golden[f"{name}|dense_q|r0|b0|t8"]
    hi, lo = sup.perman_quad(a)
    assert hi == q  # the reference's __float128 Ryser, rounded once to fp64
    if a.dtype.kind == "i":
        e = sup.perman_exact(a)
        assert abs(Fraction(hi) + Fraction(lo) - e) <= abs(e) * Fraction(1, 10 ** 28)


def test_gpu_quad_decimal_ground_truth_n30(sup):
    """double/30_0.50_0 holds 6-digit decimals: perm(A) = perm(round(1e6 A)) / 1e6^n exactly."""
    a = sup.read_matrix(fixture_path("double__30_0.50_0"))[0]
    n = a.shape[0]
    ai = np.rint(a * 1e6).astype(np.int64)
    assert np.all(ai.astype(np.float64) / 1e6 == a)
    truth = Fraction(sup.perman_exact(ai.astype(np.int32)), 10 ** (6 * n))
    hi, lo = sup.perman_quad(a)
    # the fp64 inputs are the binary neighbours of the decimals (1e-17 relative
    # each), so the walk of those inputs sits within ~n * 1e-17 of the decimal truth
    err = abs((Fraction(hi) + Fraction(lo)) - truth) / truth
    assert err < 1e-15


def test_gpu_quad_bench_matrix(sup):
    """The bench matrix (n = 40, 2^39 Gray steps): the rounded exact permanent."""
    import json, os
    here = os.path.dirname(__file__)
    ex = json.load(open(os.path.join(here, "golden", "exact_corpus.json")))["double__40_0.50_0"]
    a = sup.read_matrix(fixture_path("double__40_0.50_0"))[0]
    (hi, lo), st = sup.perman_quad(a, return_stats=True)
    assert abs(hi - ex) <= abs(ex) * 2.0 ** -52
    assert st["kernel_ms"] > 0


def test_cli_quad_gpu(sup):
    import os
    exe = os.path.join(os.path.dirname(sup.__file__), "bin", "perman")
    out = subprocess.run([exe, "-f", fixture_path("synth/20_0.50_double"), "-g", "-p4", "-q"], capture_output=True,
                         text=True, check=True).stdout
    hi = float([l for l in out.splitlines() if l.startswith("Permanent:")][0].split()[1])
    assert hi == sup.perman_quad(sup.read_matrix(fixture_path("synth/20_0.50_double"))[0], cpu=True)[0]
    assert "gpu_perman64_quad" in out


def test_gpu_chesapeake_reduced_quad(sup):
    """chesapeake (n = 39 pattern matrix): its exact permanent is 13173481190272
    (two independent exact GPU computations, test_gpu_exact.py).  The fp64 -o
    reduction loses every digit to the fp64 walk's cancellation in its merged
    leaves (the reference's own -o gives -2.6e24, HISTORY.md §7); with
    double-double leaves and combine, and the integer merges exact, -o -q gives
    the exact value."""
    a = sup.read_matrix(fixture_path("mtx/chesapeake.mtx"))[0]
    (hi, lo), st = sup.perman_reduced_quad(a, min_n=30, return_stats=True)
    assert st["leaves"] > 100
    assert Fraction(hi) + Fraction(lo) == 13173481190272
    (dh, dl) = sup.perman_quad(a)
    assert Fraction(dh) + Fraction(dl) == 13173481190272
