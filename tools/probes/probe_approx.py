"""GPU probe: throughput of the randomized estimators (samples/s) vs host threads."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402
from oracle import approx as A  # noqa: E402

for (m, n) in ((8, 8), (12, 12), (36, 36)):
    g = S.grid_graph(m, n)
    t = A.domino_tilings(m, n) if m * n <= 144 else None
    for algo, samples in ((1, 1 << 24), (2, 1 << 21)):
        if m == 36:
            samples >>= 6
        S.approx(g, algo, samples=1 << 12, seed=1)
        t0 = time.perf_counter()
        est, st = S.approx(g, algo, samples=samples, seed=2, return_stats=True)
        dt = time.perf_counter() - t0
        cs = max(samples >> 8, 64 * 16)
        t1 = time.perf_counter()
        S.approx(g, algo, samples=cs, seed=2, cpu=True, threads=16)
        ct = time.perf_counter() - t1
        print(f"grid {m}x{n} (nov {g.shape[0]}) algo {algo}: est {est:.6g} +- {st['std_error']:.2g} "
              f"(tilings {t}) kernel {st['kernel_ms']:.1f} ms wall {dt * 1e3:.1f} ms "
              f"-> {st['samples'] / (st['kernel_ms'] * 1e-3):.3e} samples/s GPU, "
              f"{cs / ct:.3e} samples/s on 16 host threads", flush=True)
