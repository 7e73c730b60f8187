"""GPU exact integer permanent (walk_exact.hip through sup_perman_exact): the
residues and hence the exact integer equal the host threads' and the
independent plain-Ryser CRT oracle's; at the corpus sizes (n = 30, 36) the
exact value sits within fp64 rounding of the reference's goldens and of the
fp64 walks, and rounds to the reference's __float128 result."""
import numpy as np
import pytest

from conftest import fixture_path, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu(sup):
    if sup.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")


def _rand(n, d, seed, lo=1, hi=6):
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < d
    mask[np.arange(n), rng.permutation(n)] = True
    return np.where(mask, rng.integers(lo, hi, (n, n)), 0).astype(np.int32)


@pytest.mark.parametrize("n,d,lo,hi,seed", [(7, 1.0, 1, 2, 1), (12, 0.5, -3, 4, 2), (20, 0.5, 1, 6, 3),
                                            (22, 0.4, 0, 2, 4), (24, 0.5, -5, 6, 5)])
def test_gpu_exact_vs_cpu_and_oracle(sup, orc, n, d, lo, hi, seed):
    a = _rand(n, d, seed, lo, hi)
    got, st = sup.perman_exact(a, return_stats=True)
    assert st["devices_used"] == 1 and st["kernel_ms"] > 0
    assert got == sup.perman_exact(a, cpu=True, threads=16)
    assert got == orc.exact_perman_crt(a, 16)


@pytest.mark.parametrize("chunk_log2", [0, 1, 4])
def test_gpu_exact_queue_with_cpu_worker(sup, chunk_log2):
    """The chunk queue (gpu_exact_dense.cu:776-904 semantics) on every visible
    device plus the hybrid CPU worker: residue sums are exact, so the integer is
    the single device's whatever the item size and whoever took which item."""
    a = _rand(26, 0.5, 11, -2, 5)
    want = sup.perman_exact(a)
    got, st = sup.perman_exact(a, gpu_num=sup.device_count(), cpu_worker=True, threads=8,
                               chunk_log2=chunk_log2, return_stats=True)
    assert got == want
    assert st["devices_used"] == sup.device_count()
    assert 0 <= st["chunks_done_cpu"]
    if chunk_log2 == 1:  # 2^12 items of 2 wave-chunks: the host worker surely takes some
        assert st["chunks_done_cpu"] > 0


def test_gpu_exact_known(sup):
    import math
    for n in (10, 21, 26):
        assert sup.perman_exact(np.ones((n, n), np.int32)) == math.factorial(n)


def test_gpu_exact_synth_goldens(sup, golden):
    names = sorted({k.split("|")[0] for k in golden if k.startswith("synth/") and "_int" in k})
    for nm in names:
        q = golden.get(f"{nm}|dense_q|r0|b0|t4")
        if q is None:
            continue
        a = sup.read_matrix(fixture_path(nm))[0]
        assert float(sup.perman_exact(a)) == q, nm


@pytest.mark.parametrize("name", ["int__30_0.20_0", "int__30_0.50_0"])
def test_gpu_exact_corpus_n30(sup, golden, name):
    a, _, _ = sup.read_matrix(fixture_path(name))
    e = sup.perman_exact(a)
    q = golden.get(f"{name}|dense_q|r0|b0|t8")
    f = golden[f"{name}|dense|r0|b0|t8"]
    assert rel(float(e), q) < 1e-15  # the reference's __float128 result
    assert rel(float(e), f) < 1e-9   # the reference's fp64 result
    assert rel(float(e), sup.perman(a, algo=4, jit=1)) < 1e-9
    # -b (binary): every listed entry is 1 (util.h:343-358); reference fp64 golden
    b, _, _ = sup.read_matrix(fixture_path(name), binary=True)
    eb = sup.perman_exact(b)
    fb = golden.get(f"{name}|dense|r0|b1|t8")
    if fb is not None:
        assert rel(float(eb), fb) < 1e-9
    assert rel(float(eb), sup.perman(b, algo=4)) < 1e-9


def test_gpu_exact_n36(sup):
    a, _, _ = sup.read_matrix(fixture_path("int__36_0.20_0"))
    e, st = sup.perman_exact(a, return_stats=True)
    assert rel(float(e), sup.perman(a, algo=4, jit=1)) < 1e-9
    assert st["kernel_ms"] > 0


def test_gpu_exact_decimal_ground_truth_n30(sup, golden):
    """double/30_0.50_0 holds 6-digit decimals, so perm(A) = perm(round(1e6 A)) / 1e6^n
    exactly: the true permanent.  The reference's __float128 result agrees to the
    binary64 rounding of the entries; our fp64 walk is within 1e-11 and never
    further from the truth than the reference's own fp64 result."""
    from fractions import Fraction
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    ai = np.rint(a * 1e6)
    e = sup.perman_exact(ai)
    exact = Fraction(e, 10 ** (6 * a.shape[0]))
    q = golden["double__30_0.50_0|dense_q|r0|b0|t8"]
    f = golden["double__30_0.50_0|dense|r0|b0|t8"]
    assert rel(float(exact), q) < 1e-14
    ours = sup.perman(a, algo=4, jit=1)
    err = lambda v: float(abs(Fraction(v) - exact) / exact)  # noqa: E731
    assert err(ours) < 1e-11
    assert err(ours) <= err(f)


def test_cli_exact_gpu(sup):
    import subprocess
    exe = sup._lib.PERMAN_BIN
    f = fixture_path("int__30_0.20_0")
    r = subprocess.run([exe, "-f", f, "-g", "-p4", "-E"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("Result: gpu_perman64_exact_residue ")
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("Permanent:")][0]
    a, _, _ = sup.read_matrix(f)
    assert int(line.split()[1]) == sup.perman_exact(a) == 4472440649521736776293900


def test_gpu_exact_tiny(sup, orc):
    rng = np.random.default_rng(8)
    for n in range(1, 9):
        a = rng.integers(-3, 4, (n, n)).astype(np.int32)
        assert sup.perman_exact(a) == orc.exact_perman(a), n


def test_gpu_chesapeake_exact_two_ways(sup):
    """chesapeake (n = 39, the matrix whose fp64 -o reduction has no correct digit
    in the reference or here, HISTORY.md §7): the exact permanent from the -o tree
    (231 exact leaves, big-integer sum) equals the exact direct walk.  The matrix
    cancels badly: the fp64 direct walk is within the north star's 1e-6, closer
    than the best of the reference's five published runs
    (revised_perman/sparyser/RealResults/chesapeake.mtx.a*.out: 13173497329080 at
    best, 1.2e-6 off)."""
    a, _, _ = sup.read_mtx(fixture_path("mtx/chesapeake.mtx"))
    r, st = sup.perman_reduced_exact(a, return_stats=True)
    assert st["leaves"] == 231
    d = sup.perman_exact(a)
    assert r == d == 13173481190272
    published_best = 13173497329080
    err = rel(float(d), sup.perman(a, algo=4, jit=1))
    assert err < 1e-6 and err < rel(float(d), float(published_best))
