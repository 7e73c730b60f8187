"""Exact ground truth for every BASELINE config matrix (and the d = 0.9 dense
point), for the -m gpu tests that pin the benchmarked segmented walk.

Corpus `double` files hold 6-digit decimals, so perm(A) = perm(round(1e6 A)) /
1e6^n exactly; integer files are exact as they are.  sup_perman_exact (residue
walk modulo primes + CRT, with its built-in 2^(n-1) divisibility self-check)
gives the integer; the fp64 segmented walk (jit = 1, the bench's walk) and the
engine's choice for the request are printed beside it with their true relative
errors.  Output: one JSON line per matrix to stdout, and the whole record to
gpurun_out/exact_truth.json (merge into tests/golden/exact_corpus.json).

    python3 tools/probes/probe_exact_truth.py [name ...]
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

FIX = os.path.join(ROOT, "tests", "fixtures")
# name -> (-r preprocessing, kernel of the request) as bench.py times it
CASES = {"double__32_0.50_0": (0, "dense"), "double__36_0.20_0": (1, "sparse"),
         "double__40_0.90_0": (0, "dense"), "synth44_0.15_int": (2, "skip")}


def main():
    names = sys.argv[1:] or list(CASES)
    out = {}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for name in names:
        prep, kern = CASES.get(name, (0, "dense"))
        a, typ, _ = S.read_matrix(os.path.join(FIX, name))
        n = a.shape[0]
        if typ == "int":
            ai, scale = a.astype(np.int64), 1
        else:
            ai = np.rint(a * 1e6).astype(np.int64)
            assert np.all(np.abs(ai - a * 1e6) < 1e-3), "entries are not 6-digit decimals"
            scale = 10 ** (6 * n)
        t = time.perf_counter()
        e, st = S.perman_exact(ai.astype(np.float64), return_stats=True)
        dt = time.perf_counter() - t
        exact = Fraction(e, scale)
        b = a
        if prep == 1:
            b = S.sort_order(a)[0]
        elif prep == 2:
            b = S.skip_order(a)[0]
        seg = S.perman(b, algo=8 if kern == "skip" else 4, sparse=prep > 0, jit=1)
        err = lambda v: float(abs(Fraction(v) - exact) / abs(exact))  # noqa: E731
        rec = {"name": name, "n": n, "exact_fp64": float(exact), "exact_integer": str(e),
               "scale": "1e6^n" if scale != 1 else "1", "exact_s": round(dt, 2),
               "kernel_ms": st["kernel_ms"], "seg_jit1": seg, "seg_rel_err": err(seg)}
        print(json.dumps(rec), flush=True)
        out[name] = rec
        with open(os.path.join(ROOT, "gpurun_out", "exact_truth.json"), "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
