"""The drop-in boundary exercised as the reference's caller would: the
RunAlgo<T> GPU branch (main.cu:30-155) retargeted to the reference-named
sup_gpu_perman64_* wrappers (tests/c_abi/runalgo_gpu.c, built by the csrc
Makefile), with CSR/CSC built by sup_compress after SortOrder / SkipOrder.
Each wrapper must equal sup_perman with the same kernel family and device
policy bit for bit, and the manual distribution (-p66) the one-device walk."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, fixture_path

EXE = os.path.join(ROOT, "superman_amd", "bin", "runalgo_gpu")


def run(*args) -> dict:
    out = subprocess.run([EXE, *map(str, args)], capture_output=True, text=True, timeout=300, check=True).stdout
    res = {}
    for line in out.splitlines():
        key, _, rest = line.partition(":")
        res[key] = rest.split()
    return res


CASES = [  # (fixture, algo, sparse, -r)
    ("int__30_0.20_0", 4, 0, 0), ("int__30_0.20_0", 5, 0, 0), ("int__30_0.20_0", 6, 0, 0),
    ("int__30_0.20_0", 66, 0, 0),
    ("double__30_0.20_0", 4, 1, 1), ("double__30_0.20_0", 5, 1, 1), ("double__30_0.20_0", 6, 1, 1),
    ("double__30_0.20_0", 66, 1, 1),
    ("int__30_0.20_0", 7, 1, 2), ("int__30_0.20_0", 8, 1, 2),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,algo,sparse,prep", CASES)
def test_runalgo_wrappers_equal_engine(sup, name, algo, sparse, prep):
    res = run(fixture_path(name), algo, sparse, prep, 1)
    assert "Error" not in res, res
    assert res["Result"][1] == res["Check"][0]  # wrapper == sup_perman, %.17e
    a = sup.read_matrix(fixture_path(name))[0]
    if prep == 1:
        a = sup.sort_order(a)[0]
    elif prep == 2:
        a = sup.skip_order(a)[0]
    got = float(res["Result"][1])
    # the same request through the Python mirror (one device: -p66's eight
    # pieces are subtrees of the one-device reduction tree)
    want = sup.perman(a, algo=4 if algo == 66 else algo, sparse=bool(sparse))
    assert got == want


@pytest.mark.gpu
def test_runalgo_exact_integer(sup):
    """int/30_0.20_0 through -p66 -s against the exact integer (rel 1e-12)."""
    res = run(fixture_path("int__30_0.20_0"), 66, 1, 1, 1)
    a = sup.read_matrix(fixture_path("int__30_0.20_0"))[0]
    exact = sup.perman_exact(a)
    assert abs(float(res["Result"][1]) - exact) <= 1e-12 * abs(exact)


def test_runalgo_refuses_csc_without_negative_entries(tmp_path):
    """A CSC built with the reference's `> 0` test (util.h:537) drops the
    negative entries; the wrapper refuses it (SUP_EINVAL) instead of walking a
    different matrix than `mat` — checked before any device work, so this runs
    without a GPU."""
    n = 6
    rng = np.random.default_rng(3)
    a = rng.integers(-3, 4, (n, n))
    a[np.arange(n), np.arange(n)] = 5
    a[0, 1] = -2
    path = tmp_path / "neg"
    nz = [(i, j, a[i, j]) for i in range(n) for j in range(n) if a[i, j] != 0]
    path.write_text(f"{n} {len(nz)} int\n" + "".join(f"{i} {j} {v}\n" for i, j, v in nz))
    res = run("--bad-csc", path)
    assert res["Error"][0] == "-1", res
    assert "sup_compress" in " ".join(res["Error"])
