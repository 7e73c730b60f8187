"""MatrixMarket input and the -o / -u reductions on the host.

* the reader against the reference's own reader (mmio.c banner +
  read_matrix.hpp readDenseMatrix / readSymmetricDenseMatrix, run by
  oracle/_ref/ref_v2 'read'; goldens store sha256 of the fp64 matrix);
* the reduction tree against the reference's own d1compress / d2compress /
  d34compress / scalesk / scaleMatrix (util.h:1199-1593, driven as
  main.cpp:993-1259 by the harness 'leaves' mode): every leaf bit-identical;
* the expansion identities exactly: sum over leaves of exact leaf permanents
  == exact permanent (Fraction Ryser), on matrices small enough for that;
* the CPU engine on the leaves against the reference's 'reduce' results.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import FIX, fixture_path, rel

MTX = sorted(f for f in os.listdir(os.path.join(FIX, "mtx")) if f.endswith(".mtx"))


def _sha(m: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(m, dtype=np.float64).tobytes()).hexdigest()


@pytest.mark.parametrize("name", MTX)
def test_mtx_reader_matches_reference(sup, golden, name):
    for b in (0, 1):
        a, typ, nz = sup.read_matrix(fixture_path("mtx/" + name), binary=bool(b))
        assert a.shape[0] == golden[f"mtx/{name}|read|b{b}|n"]
        assert _sha(a) == golden[f"mtx/{name}|read|b{b}|sha256"], (name, b)
        assert typ == ("int" if b or "real" not in open(fixture_path("mtx/" + name)).readline() else "double")
        a2, _, _ = sup.read_mtx(fixture_path("mtx/" + name), binary=bool(b))
        assert np.array_equal(a, a2)


def test_mtx_reader_errors(sup, tmp_path):
    def w(text):
        p = tmp_path / "m.mtx"
        p.write_text(text)
        return str(p)

    bad = ["%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",
           "%%MatrixMarket matrix coordinate complex general\n2 2 1\n1 1 1 0\n",
           "%%MatrixMarket matrix coordinate real general\n2 3 1\n1 1 1\n",
           "%%MatrixMarket vector coordinate real general\n2 2 1\n1 1 1\n",
           "%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 1\n",  # truncated
           "%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1\n"]  # out of range
    for text in bad:
        with pytest.raises(sup.SupError) as e:
            sup.read_mtx(w(text))
        assert e.value.code == -6
    # comments, symmetric mirroring with the same value, later duplicates win
    a, t, nz = sup.read_mtx(w("%%MatrixMarket matrix coordinate integer symmetric\n% c\n% d\n3 3 3\n"
                              "2 1 5\n3 3 7\n2 1 6\n"))
    assert t == "int" and nz == 3
    assert a.tolist() == [[0, 6, 0], [6, 0, 0], [0, 0, 7]]
    a, t, _ = sup.read_mtx(w("%%MatrixMarket matrix coordinate real skew-symmetric\n2 2 1\n2 1 -2.5\n"))
    assert t == "double" and a.tolist() == [[0, -2.5], [-2.5, 0]]  # mirrored unnegated, as the reference
    a, t, _ = sup.read_mtx(w("%%MatrixMarket matrix coordinate pattern general\n2 2 2\n1 2\n2 1\n"))
    assert t == "int" and a.tolist() == [[0, 1], [1, 0]]
    # v1 and MatrixMarket through the same entry point (CLI -f)
    a1, _, _ = sup.read_matrix(w("%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 1.5\n2 2 2\n"))
    assert a1.tolist() == [[1.5, 0], [0, 2]]


REDUCE = [("Tina_DisCog_p.mtx", 30, -1), ("Trefethen_20_s.mtx", 30, -1), ("can_24_ps.mtx", 20, -1),
          ("can_24_ps.mtx", 20, 4), ("ibm32_p.mtx", 30, -1), ("ibm32_p.mtx", 20, -1), ("ibm32_p.mtx", 20, 4),
          ("mycielskian5_ps.mtx", 20, -1), ("mycielskian5_ps.mtx", 20, 4), ("chesapeake.mtx", 20, -1),
          ("chesapeake.mtx", 30, -1), ("will57.mtx", 30, -1)]


@pytest.mark.parametrize("name,min_n,thr", REDUCE)
def test_leaves_match_reference(sup, golden, name, min_n, thr):
    a, _, _ = sup.read_matrix(fixture_path("mtx/" + name))
    _, leaves = sup.decompose(a, lambda m: 0.0, compress=True, scale=thr if thr > 0 else None, min_n=min_n)
    want = golden[f"mtx/{name}|leaves|n{min_n}|u{thr}"]
    h = hashlib.sha256()
    for m in leaves:
        h.update(np.ascontiguousarray(m, dtype=np.float64).tobytes())
    assert len(leaves) == want["count"]
    assert max((m.shape[0] for m in leaves), default=0) == want["max_n"]
    assert h.hexdigest() == want["sha256"]


def test_expansion_identities_exact(sup, orc):
    # d1 / d2 / d34 expansions are exact identities: with exact leaf
    # permanents the tree sums to the exact permanent
    rng = np.random.default_rng(7)
    for trial in range(8):
        n = 11
        a = (rng.random((n, n)) < 0.3) * rng.integers(1, 4, (n, n))
        a[np.arange(n), rng.permutation(n)] = rng.integers(1, 4, n)
        want = orc.exact_perman(a)
        got, leaves = sup.decompose(a.astype(np.int32), lambda m: float(orc.exact_perman(m.astype(np.int64))),
                                    compress=True, min_n=4)
        assert got == float(want), trial
        # leaves stop at n <= min_n or at minimum degree >= 5 (main.cpp:1007)
        for m in leaves:
            deg = min((m != 0).sum(0).min(), (m != 0).sum(1).min())
            assert m.shape[0] <= 4 or deg >= 5
    # rank deficient after singleton removal -> 0 without any leaf
    z = np.eye(6, dtype=np.int32)
    z[2, 2] = 0
    z[2, 3] = 1
    got, leaves = sup.decompose(z, lambda m: 1.0, compress=True)
    assert got == 0.0 and leaves == []


def test_scaling_divides_out(sup, orc):
    rng = np.random.default_rng(8)
    a = rng.integers(1, 6, (9, 9)).astype(np.float64)
    exact = float(orc.exact_perman(a.astype(np.int64)))
    for thr in (1, 4, 100):
        got, leaves = sup.decompose(a, lambda m: float(orc.exact_perman(m)), compress=False, scale=thr)
        assert len(leaves) == 1 and rel(got, exact) < 1e-12
        assert np.allclose(leaves[0].sum(1), thr)  # rows scaled to the threshold (last pass)


@pytest.mark.parametrize("name,min_n,thr", [r for r in REDUCE if r[0] not in ("chesapeake.mtx", "will57.mtx")])
def test_reduced_cpu_engine_vs_reference(sup, golden, name, min_n, thr):
    key = f"mtx/{name}|reduce|n{min_n}|u{thr}|t8"
    if key not in golden:
        pytest.skip("no reference result for this reduction")
    a, _, _ = sup.read_matrix(fixture_path("mtx/" + name))
    got, st = sup.perman_reduced(a, cpu=True, threads=8, compress=True, scale=thr if thr > 0 else None, min_n=min_n,
                                 return_stats=True)
    assert rel(got, golden[key]) < 1e-10
    assert st["leaves"] == golden[f"mtx/{name}|leaves|n{min_n}|u{thr}"]["count"]


def test_leaf_too_large(sup):
    # n > 64 is accepted by the reductions, but a leaf must end at n <= 64
    a = np.ones((70, 70), np.int32)
    with pytest.raises(sup.SupError) as e:
        sup.perman_reduced(a, cpu=True, compress=True)
    assert e.value.code == -7


def test_cli_compression(sup):
    exe = sup._lib.PERMAN_BIN
    f = fixture_path("mtx/can_24_ps.mtx")
    r = subprocess.run([exe, "-f", f, "-c", "-o", "-t", "4", "-v"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("Result: parallel_perman64 ")
    assert float(r.stdout.splitlines()[1].split()[1]) == pytest.approx(56892084785.0, rel=1e-12)
    r = subprocess.run([exe, "-f", f, "-c", "-o", "-u", "4", "-t", "4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and float(r.stdout.splitlines()[1].split()[1]) == pytest.approx(56892084785.0,
                                                                                            rel=1e-12)


def test_reduction_option_bounds(sup, orc):
    # d34 splits rows of degree 3 or 4 only (main.cpp:1007 hard-codes minDeg < 5):
    # max_deg > 5 would split a degree-5+ row on its first four nonzeros, and
    # min_n < 4 recurses into n = 0 leaves.  Both are refused up front.
    rng = np.random.default_rng(11)
    a = (rng.random((8, 8)) < 0.8) * rng.integers(1, 6, (8, 8))
    a[np.arange(8), rng.permutation(8)] = 1
    a = a.astype(np.int32)
    for kw in ({"max_deg": 6}, {"max_deg": 7}, {"max_deg": 0}, {"min_n": 3}, {"min_n": 0}):
        with pytest.raises(sup.SupError) as e:
            sup.decompose(a, lambda m: float(orc.exact_perman(m.astype(np.int64))), compress=True,
                          **{"min_n": 4, "max_deg": 5, **kw})
        assert e.value.code == -1 and ("max_deg" in str(e.value) or "min_n" in str(e.value))
    with pytest.raises(sup.SupError):
        sup.perman_reduced(a, cpu=True, compress=True, min_n=2)
    # the widest accepted options still give the exact permanent
    want = float(orc.exact_perman(a.astype(np.int64)))
    got, _ = sup.decompose(a, lambda m: float(orc.exact_perman(m.astype(np.int64))), compress=True, min_n=4,
                           max_deg=5)
    assert got == want


def test_repeated_leaves_memo(sup):
    """The batched decomposition (sup_perman_reduced) gives a leaf equal to an
    earlier one that leaf's value without computing it again: the result is
    the callback fold's bit for bit, and the exact form (which sums every leaf,
    repeats included) still equals the direct exact permanent."""
    import collections
    rng = np.random.default_rng(25)
    n = 26
    a = np.where(rng.random((n, n)) < 0.14, rng.integers(1, 3, (n, n)), 0).astype(np.float64)
    a[np.arange(n), rng.permutation(n)] = 1
    seen = collections.Counter()

    def leaf(m):
        seen[hashlib.sha1(m.tobytes()).hexdigest()] += 1
        return sup.perman_cpu(m, threads=2)

    via_cb, _ = sup.decompose(a, leaf, compress=True, min_n=10)
    assert sum(seen.values()) > len(seen)  # this reduction repeats a leaf
    got, st = sup.perman_reduced(a, cpu=True, threads=2, compress=True, min_n=10, return_stats=True)
    assert got == via_cb and st["leaves"] == sum(seen.values())
    assert sup.perman_reduced_exact(a, cpu=True, threads=2, min_n=10) == sup.perman_exact(a, cpu=True, threads=2)
