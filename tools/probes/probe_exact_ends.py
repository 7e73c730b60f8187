"""Exact (residue) walks with the chunk-end check (round 5): the direct exact
permanent of config 5 against its committed exact integer, and the -o -E
reductions (exact leaves) of the MatrixMarket fixtures, with wall times.

    python3 tools/probes/probe_exact_ends.py [matrix.mtx ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import superman_amd as S  # noqa: E402

ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "synth44_0.15_int"))[0]
t = time.perf_counter()
v, st = S.perman_exact(a.astype(np.int32), return_stats=True)
print(f"config 5 exact: {time.perf_counter() - t:.2f} s (kernel {st['kernel_ms'] / 1e3:.2f} s), "
      f"equal to the committed integer: {str(v) == ex['_integers']['synth44_0.15_int']['integer']}", flush=True)
for name in sys.argv[1:] or ["chesapeake.mtx", "will57.mtx"]:
    m = S.read_mtx(os.path.join(ROOT, "tests", "fixtures", "mtx", name))[0]
    t = time.perf_counter()
    v, st = S.perman_reduced_exact(m.astype(np.int32), return_stats=True)
    print(f"{name} -o -E: {time.perf_counter() - t:.2f} s, {st['leaves']} leaves, permanent {v}", flush=True)
