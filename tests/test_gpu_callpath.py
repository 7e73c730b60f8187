"""GPU: the per-call completion path (engine.cpp run_range, round 4).

The host waits on the sequence number the reduction's last pass stores beside
the result in mapped host memory instead of in hipStreamSynchronize.  The
choice is read once per process (SUP_FLAG_WAIT), so each leg runs in its own
process: both legs return the same bits and a positive kernel time, back-to-back calls
see their own results (the sequence number, not a stale one), and a long walk
(past the 2 ms spin) falls back to the stream sync with the same result.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, sys
sys.path.insert(0, %r)
import numpy as np
import superman_amd as S
rng = np.random.default_rng(11)
out = []
# alternate two matrices and two walks, so a stale result would show
mats = [rng.random((26, 26)), rng.random((28, 28)) * (rng.random((28, 28)) < 0.6) + np.eye(28)]
for i in range(12):
    a = mats[i %% 2]
    v, st = S.perman(a, jit=1 if i %% 4 < 2 else -1, return_stats=True)
    out.append([v.hex(), st["kernel_ms"], st["walk_kind"]])
big = S.read_matrix(%r)[0]
v, st = S.perman(big, jit=1, return_stats=True)  # ~18 ms walk: the wait outlasts the spin
out.append([v.hex(), st["kernel_ms"], st["walk_kind"]])
sh = [S.perman_shard(big, k, 4, jit=1) for k in range(4)]
out.append([float(x).hex() for x in sh])
print(json.dumps(out))
"""


def _leg(env_extra):
    env = dict(os.environ, **env_extra)
    big = os.path.join(ROOT, "tests", "fixtures", "double__40_0.20_0")
    r = subprocess.run([sys.executable, "-c", SCRIPT % (ROOT, big)], capture_output=True, text=True, env=env,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_call_path_legs_bit_identical():
    legs = {"flag": _leg({}), "sync": _leg({"SUP_FLAG_WAIT": "0"})}
    ref = legs["sync"]
    for name, got in legs.items():
        assert len(got) == len(ref), name
        for i, (g, r) in enumerate(zip(got[:-1], ref[:-1])):
            assert g[0] == r[0], (name, i)  # same bits
            assert g[2] == r[2], (name, i)  # same walk
            assert g[1] > 0.0, (name, i)  # a kernel time was measured
        assert got[-1] == ref[-1], name  # shards
    # the two matrices really differ (a stale result would repeat the other's bits)
    assert ref[0][0] != ref[1][0]
    # calls on one matrix with one walk agree among themselves
    assert ref[0][0] == ref[4][0] and ref[1][0] == ref[5][0]


def test_deferred_kernel_time():
    """sup_opts.timing = 0 (the bench's timed steps): the call returns once its
    result is there and leaves its walk's HIP events to sup_kernel_time — the
    same bits, one deferred time per call, each close to the per-call time."""
    import superman_amd as S

    a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "double__32_0.50_0"))[0]
    S.prepare(a, "dense", jit=1)
    eager = S.ShardCall(a, 0, 1, kernel="dense", jit=1)
    lazy = S.ShardCall(a, 0, 1, kernel="dense", jit=1, timing=False)
    S.kernel_time(0)
    ref, k_ref = [], []
    for _ in range(5):
        v, k = eager()
        ref.append(v)
        k_ref.append(k)
    assert S.kernel_time(0) == (0.0, 0)  # eager calls leave nothing deferred
    got = []
    for _ in range(300):  # past the 256 pending pairs the call reads the finished ones itself
        v, k = lazy()
        assert k == 0.0
        got.append(v)
    total, n = S.kernel_time(0)
    assert n == 300 and set(got) == set(ref) and len(set(ref)) == 1
    assert 0.5 * min(k_ref) < total / n < 2.0 * max(k_ref)
    assert S.kernel_time(0) == (0.0, 0)
