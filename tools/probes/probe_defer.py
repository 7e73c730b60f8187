"""Eager against deferred walk timing (sup_opts.timing), alternating in one process: wall per call and the
walk-kernel time (per call, or read afterwards with kernel_time) for config 2 and config 3's bench steps."""
import os
import statistics as st
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

for name, prep, kern, reps in (("double__32_0.50_0", 0, "dense", 500), ("double__36_0.20_0", 1, "sparse", 150)):
    a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", name))[0]
    if prep:
        a = S.sort_order(a)[0]
    S.prepare(a, kern, jit=1)
    calls = {t: S.ShardCall(a, 0, 1, kernel=kern, jit=1, timing=t) for t in (True, False)}
    for rnd in range(3):
        for t in (True, False):
            c = calls[t]
            for _ in range(20):
                c()
            S.kernel_time(0)
            ks = []
            t0 = time.perf_counter()
            for _ in range(reps):
                ks.append(c()[1])
            wall = (time.perf_counter() - t0) / reps * 1e3
            tot, n = S.kernel_time(0)
            k = tot / n if n else st.mean(ks)
            print(f"{name} {'eager' if t else 'deferred'}: {wall:.4f} ms per call, kernel {k:.4f} ms, "
                  f"beyond {(wall - k) * 1e3:.1f} us", flush=True)
