"""The fused fold (walk_common.hpp chunk_store): the walk kernels fold their own
chunk partials into the 64-way pairwise tree launch_pairwise_reduce builds,
so no reduction launch follows the walk.  Every walk family, chunk counts
from 1 to 2^17 (growing, so the arrival counters are reallocated between
calls), the visited sums and the -R slot path give the same bits with the fold
as with the reduction launches (SUP_FOLD=0, read once per process: each mode
runs in a child process), and each call leaves every arrival counter at zero
(SUP_FOLD_CHECK)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, fixture_path

pytestmark = pytest.mark.gpu

_CODE = r"""
import json, sys
import numpy as np
import superman_amd as S
out = []
for path, kern, jit, algo, sparse, rccl in json.loads(sys.argv[1]):
    a = np.load(path)
    if kern == "skip":
        a = S.skip_order(a)[0]
    for _ in range(2):  # the second call reuses the context's buffers
        v, st = S.perman(a, algo=algo, sparse=sparse, jit=jit, kernel=kern, use_rccl=rccl, return_stats=True)
        out.append([v.hex(), st["visited_steps"], st["walk_kind"]])
print(json.dumps(out))
"""


def _cases(tmp_path):
    rng = np.random.default_rng(2026)
    cases = []
    # (n, density, integer): chunk counts 1 (n = 8) up to 2^17 (n = 40)
    for n, d, integer in ((8, 0.6, False), (14, 0.5, False), (20, 0.5, False), (24, 0.3, True), (28, 0.5, False),
                          (30, 0.2, True), (32, 0.5, False)):
        if integer:
            a = np.where(rng.random((n, n)) < d, rng.integers(1, 6, (n, n)), 0).astype(np.float64)
            a[np.arange(n), rng.permutation(n)] = 1.0
        else:
            a = np.where(rng.random((n, n)) < d, rng.random((n, n)), 0.0)
            a[np.arange(n), rng.permutation(n)] = 0.5
        p = str(tmp_path / f"m{n}.npy")
        np.save(p, a)
        for kern, jit, algo, sparse in (("dense_plain", -1, 4, False), ("dense", -1, 4, False), ("sparse", -1, 4, True),
                                        ("dense", 1, 4, False)):
            cases.append([p, kern, jit, algo, sparse, False])
        if integer:
            cases.append([p, "skip", -1, 7, True, False])
    c5 = str(tmp_path / "config5.npy")
    np.save(c5, np.ascontiguousarray(__import__("superman_amd").read_matrix(fixture_path("synth44_0.15_int"))[0]))
    cases.append([c5, "skip", 1, 8, True, False])  # segmented walk with chunk skip (visited sums)
    p40 = fixture_path("double__40_0.20_0")
    a40 = str(tmp_path / "d40.npy")
    np.save(a40, __import__("superman_amd").read_matrix(p40)[0])
    cases.append([a40, "dense", 1, 4, False, False])
    cases.append([str(tmp_path / "m28.npy"), "dense", 1, 4, False, 2])  # -R (RCCL slot): the result through d_result
    return cases


def _run(cases, **env):
    e = dict(os.environ, PYTHONPATH=ROOT, **env)
    r = subprocess.run([sys.executable, "-c", _CODE, json.dumps(cases)], capture_output=True, text=True, env=e,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_fused_fold_same_bits(tmp_path):
    cases = _cases(tmp_path)
    fused, log = _run(cases, SUP_FOLD="1", SUP_FOLD_CHECK="1")
    assert "after a fused walk" not in log, log[-2000:]  # every arrival counter back at zero
    assert log.count("SUP_FOLD_CHECK: kind") >= len(cases)  # the fold ran
    launched, _ = _run(cases, SUP_FOLD="0")
    assert fused == launched
    # the two calls of each case agree, and the walk families ran as asked
    for i in range(0, len(fused), 2):
        assert fused[i] == fused[i + 1]
    assert {w for _, _, w in fused} >= {0, 1, 2, 3}
