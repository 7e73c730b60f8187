"""Double-double walk (sup_perman_quad) throughput and accuracy on one MI355X.

For each corpus matrix: Gray steps/s of walk_dd, the fp64 op rate of its cost
model (16n + 13 ops per Gray step), and — where exact ground truth exists —
the error of hi + lo and of the fp64 engine.  The reference's own quad
calculation (v2 -q, parallel_perman64<__float128>) ran at 3.0e6 Gray steps/s
on 8 host cores here."""
import json
import os
import sys
import time
from fractions import Fraction

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import superman_amd as S  # noqa: E402

FIX = os.path.join(os.path.dirname(__file__), "..", "..", "tests", "fixtures")
EX = json.load(open(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "exact_corpus.json")))
PEAK = 78.6e12

import numpy as np  # noqa: E402

rng = np.random.default_rng(28)
a28 = np.where(rng.random((28, 28)) < 0.5, rng.uniform(0.0, 5.0, (28, 28)), 0.0)
(hi28, _), st28 = S.perman_quad(a28, return_stats=True)
print(json.dumps({"matrix": "random n=28 d=0.5", "n": 28, "kernel_ms": round(st28["kernel_ms"], 3),
                  "gray_steps_per_s": float(1 << 27) / (st28["kernel_ms"] / 1e3)}), flush=True)

for name in ["double__30_0.50_0", "double__32_0.50_0", "int__36_0.20_0", "double__40_0.20_0", "double__40_0.50_0"]:
    a = S.read_matrix(os.path.join(FIX, name))[0]
    n = a.shape[0]
    S.perman_quad(a) if n <= 32 else None  # warm (module load) on small ones
    t0 = time.perf_counter()
    (hi, lo), st = S.perman_quad(a, return_stats=True)
    wall = time.perf_counter() - t0
    steps = float(1 << (n - 1))
    ops = 16 * n + 13
    line = {"matrix": name, "n": n, "kernel_ms": round(st["kernel_ms"], 3), "wall_ms": round(wall * 1e3, 3),
            "gray_steps_per_s": steps / (st["kernel_ms"] / 1e3), "model_ops_per_step": ops,
            "issue_frac": steps * ops / (st["kernel_ms"] / 1e3) / (PEAK / 2), "hi": hi, "lo": lo}
    if name in EX:
        line["rel_err_hi_vs_exact_rounded"] = abs(hi - EX[name]) / abs(EX[name])
        f64 = S.perman(a, algo=4, jit=1)
        line["fp64_engine_rel_err"] = abs(f64 - EX[name]) / abs(EX[name])
    if a.dtype.kind == "i":
        e = S.perman_exact(a)
        line["rel_err_hi_plus_lo_vs_exact"] = float(abs(Fraction(hi) + Fraction(lo) - e) / abs(e))
        f64 = S.perman(a, algo=4, jit=1)
        line["fp64_engine_rel_err"] = float(abs(Fraction(f64) - e) / abs(e))
    print(json.dumps(line), flush=True)
