"""Walks of config 5 (n = 44 d = 0.15 integer, SkipOrder) whose column map is
searched for chunk ends (round 5): the ahead-of-time SpaRyser walk (`-p4 -s
--jit -1`), the exact walk and the double-double walk, against exact values.

    python3 tools/probes/probe_chunk_end_search.py
"""
import json
import os
import sys
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import superman_amd as S  # noqa: E402

ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "synth44_0.15_int"))[0]
c = S.skip_order(a)[0]
truth = int(ex["_integers"]["synth44_0.15_int"]["integer"])
for label, fn in (
        ("SpaRyser -p4 -s --jit -1", lambda: S.perman(c, algo=4, sparse=True, jit=-1, return_stats=True)),
        ("exact", lambda: S.perman_exact(c.astype(np.int32), return_stats=True)),
        ("double-double", lambda: S.perman_quad(c, return_stats=True))):
    t = time.perf_counter()
    v, st = fn()
    wall = time.perf_counter() - t
    val = Fraction(v[0]) + Fraction(v[1]) if isinstance(v, tuple) else (Fraction(v) if not isinstance(v, int) else v)
    print(f"{label}: {wall:.2f} s (kernel {st['kernel_ms'] / 1e3:.2f} s), walk_kind {st.get('walk_kind')}, "
          f"rel. err vs exact {float(abs(val - truth) / truth):.2e}", flush=True)
