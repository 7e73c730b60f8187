"""Wall time of the -o reductions on one MI355X against the walk-kernel time
they contain (sup_perman_reduced, leaves through the engine): how much of a
reduction is GPU work and how much per-leaf overhead.

    python3 tools/probes/probe_reduce.py [matrix.mtx ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

FIX = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "fixtures", "mtx")
names = sys.argv[1:] or ["chesapeake.mtx", "will57.mtx"]
warm = S.read_mtx(os.path.join(FIX, "chesapeake.mtx"))[0]
for algo, sparse in ((4, False), (4, True)):
    S.perman_reduced(warm, algo=algo, sparse=sparse)  # n = 30 kernels loaded once
BATCHES = os.environ.get("PROBE_BATCHES", "1,16").split(",")  # leaves per launch (SUP_LEAF_BATCH; 1 = one each)
WORKERS = os.environ.get("PROBE_WORKERS", "1,4,8").split(",")
SPARSE = [s == "1" for s in os.environ.get("PROBE_SPARSE", "0,1").split(",")]
for name in names:
    a = S.read_mtx(os.path.join(FIX, name))[0]
    # concurrent GPU leaves (context lanes, SUP_LEAF_WORKERS) x leaves per launch (SUP_LEAF_BATCH)
    for (algo, sparse), batch, workers in [((4, sp), b, w) for sp in SPARSE for b in BATCHES for w in WORKERS]:
        os.environ["SUP_LEAF_WORKERS"] = workers
        os.environ["SUP_LEAF_BATCH"] = batch
        t = time.perf_counter()
        v, st = S.perman_reduced(a, algo=algo, sparse=sparse, return_stats=True)
        wall = time.perf_counter() - t
        print(f"{name} n={a.shape[0]} algo={algo}{' -s' if sparse else ''} batch={batch} workers={workers}: "
              f"{st['leaves']} leaves, wall {wall:.3f} s, walk kernels {st['kernel_ms'] / 1e3:.3f} s "
              f"({st['kernel_ms'] / 1e3 / wall:.0%}), {st['gray_steps'] / wall:.3e} Gray steps/s, perm {v!r}",
              flush=True)
