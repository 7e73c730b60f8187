"""GPU probe of fp64 accuracy per walk at n = 30-40: every walk kind on the
corpus matrices whose exact permanent is known (tests/golden/exact_corpus.json,
from tools/probes/probe_exact_decimal.py), relative error against it.  The plain dense
walk has the reference kernel's structure (x_j += col_j, product of all n rows
per step); the others reorder the same products (prefix blocks, product trees,
paired steps)."""
import json
import os
import sys
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

exact = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
runs = [("plain", "dense_plain", -1, None), ("prefix", "sparse", -1, None), ("seg cc0", "seg", 1, "0"),
        ("seg cc1", "seg", 1, "1"), ("seg cc2", "seg", 1, "2"), ("seg cc3", "seg", 1, "3"),
        ("seg (plan)", "seg", 1, None), ("skipper", "skip", -1, None)]
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

# random integer matrices (values 1..5, a permutation's diagonal forced nonzero):
# the exact integer path gives the ground truth
import numpy as np  # noqa: E402

geo = {label: [] for label, *_ in runs}
for n, d, seeds in ((36, 0.5, range(6)), (38, 0.3, range(6, 10))):
    for seed in seeds:
        rng = np.random.default_rng(1000 + seed)
        mask = rng.random((n, n)) < d
        mask[np.arange(n), rng.permutation(n)] = True
        a = np.where(mask, rng.integers(1, 6, (n, n)), 0).astype(np.float64)
        e = S.perman_exact(a)
        row = []
        for label, kernel, jit, cc in runs:
            if cc is None:
                os.environ.pop("SUP_JIT_CC", None)
            else:
                os.environ["SUP_JIT_CC"] = cc
            v = S.perman(a, kernel=kernel, jit=jit)
            err = float(abs(Fraction(v) - e) / e)
            geo[label].append(max(err, 1e-18))
            row.append(f"{label} {err:.1e}")
        os.environ.pop("SUP_JIT_CC", None)
        print(f"random int n={n} d={d} seed={seed}: " + " | ".join(row), flush=True)
print("geometric mean rel.err over the random matrices: " +
      " | ".join(f"{k} {float(np.exp(np.mean(np.log(v)))):.1e}" for k, v in geo.items()), flush=True)
