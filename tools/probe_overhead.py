"""GPU probe: host-side cost of one C-ABI call (sup_perman through the Python
mirror) on small matrices, where the walk itself takes microseconds: wall time
per call minus the walk kernel's hipEvent time, averaged over repeated calls on
one matrix (plan cached after the first)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import superman_amd as S  # noqa: E402

rng = np.random.default_rng(5)
for n, jit in ((16, -1), (24, -1), (30, -1), (30, 1), (32, 1)):
    a = rng.random((n, n))
    for _ in range(3):
        S.perman(a, jit=jit)
    reps = 300
    kms = 0.0
    t = time.perf_counter()
    for _ in range(reps):
        _, st = S.perman(a, jit=jit, return_stats=True)
        kms += st["kernel_ms"]
    wall = (time.perf_counter() - t) / reps * 1e6
    print(f"n={n} jit={jit}: {wall:.1f} us per call, kernel {kms / reps * 1e3:.1f} us, "
          f"host/launch overhead {wall - kms / reps * 1e3:.1f} us", flush=True)
