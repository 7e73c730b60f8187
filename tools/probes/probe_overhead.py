"""GPU probe: host-side cost of one C-ABI call (sup_perman through the Python
mirror) on small matrices, where the walk itself takes microseconds: wall time
per call minus the walk kernel's hipEvent time, averaged over repeated calls on
one matrix (plan cached after the first)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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

# a new matrix every call, as the -o leaves are: planning + table upload each time
# (round 3: staging the uploads through pinned memory measured no difference,
# 158 against 160 us at n = 24 and 269 against 274 us at n = 30 — the time is
# the host's planning, profiles/r3/probe_overhead_newmatrix.log)
for n in (24, 30):
    mats = [rng.random((n, n)) * (rng.random((n, n)) < 0.4) + np.eye(n) for _ in range(200)]
    S.perman(mats[0])
    kms = 0.0
    t = time.perf_counter()
    for a in mats:
        _, st = S.perman(a, return_stats=True)
        kms += st["kernel_ms"]
    wall = (time.perf_counter() - t) / len(mats) * 1e6
    print(f"n={n} new matrix per call: {wall:.1f} us per call, kernel {kms / len(mats) * 1e3:.1f} us, "
          f"host/launch overhead {wall - kms / len(mats) * 1e3:.1f} us", flush=True)

# the bench's own call on config 2 (double/32_0.50_0, sup_perman_shard, segmented walk):
# VERDICT r3 next-7 asks ms_per_step - kernel_ms <= 25 us
a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "double__32_0.50_0"))[0]
S.prepare(a, "dense", jit=1)
for _ in range(5):
    S.perman_shard(a, 0, 1, jit=1)
for label, stats in (("return_stats", True), ("value only", False)):
    reps, kms = 300, 0.0
    t = time.perf_counter()
    for _ in range(reps):
        if stats:
            _, st = S.perman_shard(a, 0, 1, jit=1, return_stats=True)
            kms += st["kernel_ms"]
        else:
            S.perman_shard(a, 0, 1, jit=1)
    wall = (time.perf_counter() - t) / reps * 1e6
    k = kms / reps * 1e3 if stats else float("nan")
    print(f"config 2 perman_shard ({label}): {wall:.1f} us per call, kernel {k:.1f} us, "
          f"host/launch overhead {wall - k:.1f} us", flush=True)

# where the config 2 per-call cost goes: Python wrapper vs the C ABI call (its own wall clock, sup_stats.wall_ms)
# vs the walk kernel (hipEvents around the walk only)
import ctypes as C  # noqa: E402
from superman_amd import _lib  # noqa: E402
lib = _lib.load()
b, dt, n = S._mat(a)
o = S._opts(jit=1)
out, st = C.c_double(0.0), _lib.SupStats()
args = (b.ctypes.data, dt, n, S._KERNELS["dense"], 0, 1, C.byref(o), C.byref(out), C.byref(st))
for _ in range(5):
    lib.sup_perman_shard(*args)
reps, cw, kk = 300, 0.0, 0.0
t = time.perf_counter()
for _ in range(reps):
    lib.sup_perman_shard(*args)
    cw += st.wall_ms
    kk += st.kernel_ms
wall = (time.perf_counter() - t) / reps * 1e6
print(f"config 2 bare ctypes call: {wall:.1f} us per call; C ABI wall {cw / reps * 1e3:.1f} us; walk kernel "
      f"{kk / reps * 1e3:.1f} us; inside the C call but outside the walk {(cw - kk) / reps * 1e3:.1f} us; "
      f"Python wrapper {wall - cw / reps * 1e3:.1f} us", flush=True)
