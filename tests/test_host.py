"""Host logic of the product: reader, CSR/CSC, orders, layout, and the CPU walk
(`-c`), which must be bit-identical to the oracle's mirror of the engine
schedule (and therefore to the GPU kernels)."""
import os

import numpy as np
import pytest

from conftest import FIX, fixture_path, rel


def test_read_matrix_types(sup):
    a, typ, nnz = sup.read_matrix(fixture_path("int__30_0.50_0"))
    assert typ == "int" and a.dtype == np.int32 and a.shape == (30, 30)
    assert int((a != 0).sum()) == nnz
    d, typ, nnz = sup.read_matrix(fixture_path("double__30_0.50_0"))
    assert typ == "double" and d.dtype == np.float64 and int((d != 0).sum()) == nnz
    f, typ, _ = sup.read_matrix(fixture_path("float__30_0.50_0"))
    assert typ == "float" and f.dtype == np.float32
    b, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"), binary=True)
    assert set(np.unique(b)) <= {0.0, 1.0} and int(b.sum()) == nnz


def test_read_matrix_errors(sup, tmp_path):
    p = tmp_path / "bad"
    p.write_text("3 2 int\n0 0 1\n5 1 1\n")
    with pytest.raises(sup.SupError):
        sup.read_matrix(str(p))
    p.write_text("3 2 complex\n")
    with pytest.raises(sup.SupError):
        sup.read_matrix(str(p))
    with pytest.raises(sup.SupError):
        sup.read_matrix(str(tmp_path / "missing"))
    # malformed lines are skipped (util.h:351)
    p.write_text("2 2 double\n0 0 1.5\ngarbage\n1 1 2\n")
    a, _, _ = sup.read_matrix(str(p))
    assert a.tolist() == [[1.5, 0.0], [0.0, 2.0]]


def test_compress(sup):
    rng = np.random.default_rng(3)
    a = np.where(rng.random((9, 9)) < 0.3, rng.standard_normal((9, 9)), 0.0)
    c = sup.compress(a)
    for j in range(9):
        rows = c["rows"][c["cptrs"][j]:c["cptrs"][j + 1]]
        assert list(rows) == list(np.nonzero(a[:, j])[0])
        assert np.array_equal(c["cvals"][c["cptrs"][j]:c["cptrs"][j + 1]], a[rows, j])
        cols = c["cols"][c["rptrs"][j]:c["rptrs"][j + 1]]
        assert list(cols) == list(np.nonzero(a[j])[0])


def test_orders_are_permutations(sup):
    rng = np.random.default_rng(4)
    a = np.where(rng.random((12, 12)) < 0.3, rng.integers(1, 5, (12, 12)), 0).astype(np.int32)
    s, cp = sup.sort_order(a)
    assert np.array_equal(s, a[:, cp])
    nnz = (a != 0).sum(0)[cp]
    assert all(nnz[i] <= nnz[i + 1] for i in range(11))
    k, rp, cp2 = sup.skip_order(a)
    assert sorted(rp) == list(range(12)) and sorted(cp2) == list(range(12))
    assert np.array_equal(k, a[np.ix_(rp, cp2)])


def test_layout_matches_oracle(sup, orc):
    for n in range(1, 65):
        assert sup.layout(n) == orc.engine_layout(n), n
        L, m, h = sup.layout(n)
        assert L + m + h == n - 1 and L <= 6 and m <= 31 and (h <= 20 or m == 31)


@pytest.mark.parametrize("kind", ["dense", "sparse", "skip"])
def test_cpu_walk_bitexact_vs_oracle_mirror(sup, orc, kind):
    rng = np.random.default_rng(7)
    for n in (1, 2, 3, 6, 7, 8, 11, 16, 19):
        for d in (0.5, 0.2):
            pat = rng.random((n, n)) < d
            pat[np.arange(n), rng.permutation(n)] = True
            a = np.where(pat, rng.integers(1, 4, (n, n)), 0).astype(np.float64)
            if kind == "skip":
                a, _, _ = sup.skip_order(a)
            got = sup.perman_cpu(a, kind, threads=3)
            want = orc.engine_perman_as(sup, a, kind, threads=2)
            assert got == want or (np.isnan(got) and np.isnan(want)), (n, d, got, want)


def test_cpu_walk_known_answers(sup, orc):
    import math
    for n in (1, 2, 4, 8, 13, 17):
        assert sup.perman_cpu(np.ones((n, n)), "dense", 4) == pytest.approx(math.factorial(n), rel=1e-13)
        assert sup.perman_cpu(np.ones((n, n)), "skip", 4) == pytest.approx(math.factorial(n), rel=1e-13)
    p = np.eye(10)[np.random.default_rng(0).permutation(10)]
    for k in ("dense", "sparse", "skip"):
        assert sup.perman_cpu(p, k, 2) == 1.0
    z = np.ones((9, 9))
    z[4] = 0
    for k in ("dense", "sparse", "skip"):
        assert sup.perman_cpu(z, k, 2) == 0.0


def test_cpu_walk_corpus_n30(sup, orc, golden):
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    got = sup.perman_cpu(a, "dense", 8)
    key = "double__30_0.50_0|dense_q|r0|b0|t8"
    if key in golden:
        assert rel(got, golden[key]) < 1e-9
    assert rel(got, golden["double__30_0.50_0|dense|r0|b0|t8"]) < 1e-8


def test_nw_start_matches_oracle(sup, orc):
    a = np.random.default_rng(9).random((13, 13))
    x, p = sup.nw_start(a)
    xo, po = orc.nw_start(a)
    assert np.array_equal(x, xo) and p == po


def test_config5_fixtures_reproducible(sup, tmp_path):
    # BASELINE config 5 has no reference file: the committed inputs must be
    # exactly what tests/fixtures/gen_config5.py generates
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_config5", os.path.join(FIX, "gen_config5.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    for typ in ("int", "double"):
        a, _ = g.generate(44, 0.15, typ)
        g.write_v1(str(tmp_path / typ), a, typ)
        assert open(tmp_path / typ).read() == open(fixture_path(f"synth44_0.15_{typ}")).read()
        b, t, _ = sup.read_matrix(fixture_path(f"synth44_0.15_{typ}"))
        assert t == typ and np.array_equal(a, b)
        assert (b != 0).any(0).all() and (b != 0).any(1).all()


def test_skipper_column_search(sup):
    """SkipPer's column map for long integer walks (engine.cpp
    skip_walk_order): config 5 takes a searched map, the same in every process
    (the plan must not depend on the host or the device count), with a lower
    prefix cost than SkipOrder's map; a non-integer matrix and a short walk keep
    SkipOrder's map (engine bit e = column e)."""
    import subprocess
    import sys
    from conftest import ROOT
    a = sup.skip_order(sup.read_matrix(fixture_path("synth44_0.15_int"))[0])[0]
    info = sup.plan_info(a, "skip", jit=-1)
    assert info["kind"] == "skip"
    cm = [int(c) for c in info["colmap"]]
    assert sorted(cm) == list(range(a.shape[0] - 1))
    assert cm != list(range(a.shape[0] - 1))
    assert info["est_ops_per_step"] < 25.5
    code = ("import sys; sys.path.insert(0, %r); import superman_amd as S; "
            "a = S.skip_order(S.read_matrix(%r)[0])[0]; "
            "print(' '.join(map(str, S.plan_info(a, 'skip', jit=-1)['colmap'])))") % (
        ROOT, fixture_path("synth44_0.15_int"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env=dict(os.environ, OMP_NUM_THREADS="3")).stdout.split()
    assert [int(c) for c in out] == cm
    real = sup.skip_order(sup.read_matrix(fixture_path("synth44_0.15_double"))[0])[0]
    assert [int(c) for c in sup.plan_info(real, "skip", jit=-1)["colmap"]] == list(range(43))
    short = sup.skip_order(sup.read_matrix(fixture_path("int__30_0.20_0"))[0])[0]
    assert [int(c) for c in sup.plan_info(short, "skip", jit=-1)["colmap"]] == list(range(29))
