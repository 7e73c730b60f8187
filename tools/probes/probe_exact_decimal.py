"""Ground truth for the fp64 corpus matrices: their entries are decimals with
6 digits, so perm(A) = perm(round(1e6 A)) / 1e6^n exactly, and the exact
integer path (sup_perman_exact) gives the true permanent of the file's
matrix.  Prints it next to the fp64 GPU results (segmented and prefix
walks) and their true relative errors."""
import os
import sys
import time
from fractions import Fraction

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import superman_amd as S  # noqa: E402

FIX = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "fixtures")
for name in sys.argv[1:] or ["double__30_0.50_0", "double__40_0.20_0", "double__40_0.50_0"]:
    a = S.read_matrix(os.path.join(FIX, name))[0]
    n = a.shape[0]
    ai = np.rint(a * 1e6).astype(np.int64)
    assert np.all(np.abs(ai - a * 1e6) < 1e-3), "entries are not 6-digit decimals"
    t = time.perf_counter()
    e, st = S.perman_exact(ai.astype(np.float64), return_stats=True)
    dt = time.perf_counter() - t
    exact = Fraction(e, 10 ** (6 * n))
    seg = S.perman(a, algo=4, jit=1)
    blk = S.perman(a, algo=4, jit=-1)
    err = lambda v: float(abs(Fraction(v) - exact) / abs(exact))  # noqa: E731
    print(f"{name} n={n}: exact={float(exact):.17e} (integer {len(str(abs(e)))} digits, exact path "
          f"{dt:.1f} s, kernel {st['kernel_ms']:.0f} ms) | fp64 segmented {seg:.17e} rel.err {err(seg):.2e} | "
          f"fp64 prefix-blocked {blk:.17e} rel.err {err(blk):.2e}", flush=True)
