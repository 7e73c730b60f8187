"""GPU probe of fp64 accuracy per walk at n = 30-40: every walk kind on the
corpus matrices whose exact permanent is known (tests/golden/exact_corpus.json,
from tools/probe_exact_decimal.py), relative error against it.  The plain dense
walk has the reference kernel's structure (x_j += col_j, product of all n rows
per step); the others reorder the same products (prefix blocks, product trees,
paired steps)."""
import json
import os
import sys
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

exact = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
runs = [("plain", "dense_plain", -1, None), ("prefix", "sparse", -1, None), ("seg cc0", "seg", 1, "0"),
        ("seg cc1", "seg", 1, "1"), ("seg cc2", "seg", 1, "2"), ("skipper", "skip", -1, None)]
for name in [k for k in exact if not k.startswith("_")]:
    a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", name))[0]
    e = Fraction(exact[name])
    row = []
    for label, kernel, jit, cc in runs:
        if cc is None:
            os.environ.pop("SUP_JIT_CC", None)
        else:
            os.environ["SUP_JIT_CC"] = cc
        t = time.perf_counter()
        v, st = S.perman(a, kernel=kernel, jit=jit, return_stats=True)
        dt = time.perf_counter() - t
        err = float(abs(Fraction(v) - e) / abs(e))
        row.append(f"{label} {err:.2e} ({st['kernel_ms']:.0f} ms)")
    os.environ.pop("SUP_JIT_CC", None)
    print(f"{name} n={a.shape[0]}: " + " | ".join(row), flush=True)
