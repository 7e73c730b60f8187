"""Every form of the ahead-of-time SkipPer kernel (walk_skip.hip; reference
kernel_xshared_coalescing_mshared_skipper, gpu_exact_sparse.cu:555-670) gives
the same bits and visits the same states.  The launch takes the most
specialised form whose compile-time block counts cover the walk's own (form 3:
the 15 steps inside a 16-step segment straight-line; 2: walk bits 0-2 on one
block; 1: bits 0-1; 0: every block count at run time); SUP_SKIP_FORM caps the
form, read once per process, so each form runs in a child process.  The
default form is pinned against the oracle's mirror by test_gpu_parity.py."""
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
for path in sys.argv[1:]:
    a = np.load(path)
    k = S.skip_order(a)[0]
    v, st = S.perman(k, 7, sparse=True, jit=-1, return_stats=True)
    out.append([v.hex(), st["visited_steps"], st["walk_kind"]])
print(json.dumps(out))
"""


def _mats(tmp_path):
    rng = np.random.default_rng(606)
    paths = []
    for n, d in ((18, 0.3), (24, 0.15), (26, 0.25), (28, 0.5), (30, 0.12)):
        a = np.where(rng.random((n, n)) < d, rng.integers(1, 6, (n, n)), 0).astype(np.float64)
        a[np.arange(n), rng.permutation(n)] = 1.0
        paths.append(tmp_path / f"m{n}_{d}.npy")
        np.save(paths[-1], a)
    c5 = np.ascontiguousarray(__import__("superman_amd").read_matrix(fixture_path("synth44_0.15_int"))[0])
    paths.append(tmp_path / "config5.npy")
    np.save(paths[-1], c5)
    return paths


def test_skip_forms_same_bits(tmp_path):
    paths = [str(p) for p in _mats(tmp_path)]
    runs = {}
    for form in ("0", "1", "2", "3"):
        env = dict(os.environ, SUP_SKIP_FORM=form, PYTHONPATH=ROOT)
        r = subprocess.run([sys.executable, "-c", _CODE, *paths], capture_output=True, text=True, env=env,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        runs[form] = json.loads(r.stdout.strip().splitlines()[-1])
    for form in ("1", "2", "3"):
        assert runs[form] == runs["0"], form
    assert all(w == 2 for _, _, w in runs["0"])  # the SkipPer kernel ran
