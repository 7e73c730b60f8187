"""Double-double walk timings (round 5, prefix-blocked walk_dd_blocked where its
cost model wins): -q on the bench matrix against its exact permanent, and -o -q
on the MatrixMarket fixtures.  Prints as it goes.

    python3 tools/probes/probe_quad_blocked.py [matrix.mtx ...]
"""
import json
import os
import sys
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
for name in ("double__40_0.50_0", "double__40_0.20_0"):
    a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", name))[0]
    info = S.plan_info(a, "sparse", jit=-1)
    t = time.perf_counter()
    (hi, lo), st = S.perman_quad(a, return_stats=True)
    print(f"{name} -q: {time.perf_counter() - t:.2f} s (kernel {st['kernel_ms'] / 1e3:.2f} s), {hi!r} {lo!r}, "
          f"|hi - exact|/exact {abs(hi - ex[name]) / abs(ex[name]):.2e}", flush=True)
for name in sys.argv[1:]:
    m = S.read_mtx(os.path.join(ROOT, "tests", "fixtures", "mtx", name))[0]
    t = time.perf_counter()
    (hi, lo), st = S.perman_reduced_quad(m, return_stats=True)
    print(f"{name} -o -q: {time.perf_counter() - t:.2f} s, {hi!r} {lo!r}", flush=True)
