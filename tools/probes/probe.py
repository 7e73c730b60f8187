"""GPU probe: throughput of each walk on the benchmark matrices (one process)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import superman_amd as S  # noqa: E402

rng = np.random.default_rng(0)
a = rng.random((16, 16))
for k in ("dense", "dense_plain", "sparse", "skip"):
    g = S.perman(a, algo=7 if k == "skip" else 4, sparse=k in ("sparse", "skip")) if k != "dense_plain" else None
print("n16 ok", flush=True)


def run(label, m, kernel, reps=2):
    n = m.shape[0]
    kind = kernel
    if kind == "seg":
        print(f"  prepare: {S.prepare(m, 'seg')}", flush=True)
    S.perman_shard(m, 0, 1, kernel=kind)
    best = None
    for _ in range(reps):
        t = time.perf_counter()
        v, st = S.perman_shard(m, 0, 1, kernel=kind, return_stats=True)
        dt = time.perf_counter() - t
        best = st if best is None or st["kernel_ms"] < best["kernel_ms"] else best
    steps = 2 ** (n - 1)
    ks = best["kernel_ms"] * 1e-3
    print(f"{label:28s} {kernel:11s} walk={best['walk_kind']} est_ops={best['est_ops_per_step']:.1f} "
          f"kernel={best['kernel_ms']:.1f}ms wall={dt*1e3:.1f}ms steps/s={steps/ks:.3e} "
          f"nominal-frac={2*n*steps/ks/78.6e12:.3f} visited={best['visited_steps']:.3e} grid={best['grid']}",
          flush=True)


only = sys.argv[1:]  # optional subset of fixture names
for path, prep in (("double__32_0.50_0", 0), ("double__36_0.20_0", 1), ("double__40_0.50_0", 0),
                   ("int__36_0.20_0", 2), ("synth44_0.15_int", 2), ("synth44_0.15_double", 2)):
    if only and path not in only:
        continue
    m, _, _ = S.read_matrix(os.path.join("tests/fixtures", path))
    if prep == 1:
        m = S.sort_order(m)[0]
    if prep == 2:
        m = S.skip_order(m)[0]
    for kernel in (("sparse", "seg", "skip") if m.shape[0] > 40 else
                   ("dense_plain", "dense", "sparse", "seg") + (("skip",) if prep == 2 else ())):
        run(f"{path} r{prep}", m, kernel, reps=1 if m.shape[0] > 40 else 2)

if only:
    sys.exit(0)
# strong-scaling rehearsal on one GPU: the 8 shards of the n=40 bench, one by one
m, _, _ = S.read_matrix("tests/fixtures/double__40_0.50_0")
full = S.perman_shard(m, 0, 1, jit=1)
parts, times = [], []
for world in (2, 4, 8):
    parts, times = [], []
    for r in range(world):
        v, st = S.perman_shard(m, r, world, return_stats=True, jit=1)
        parts.append(v)
        times.append(st["kernel_ms"])
    import math
    tot = math.fsum(parts)
    print(f"shards={world}: kernel ms per shard min {min(times):.1f} max {max(times):.1f} "
          f"(1-GPU {1152.0 if False else 0:.0f}) sum rel-diff vs full {abs(tot - full) / abs(full):.2e}", flush=True)
