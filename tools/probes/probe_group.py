"""Walk-kernel time against the wave's chunk group (SUP_WALK_GROUP: chunks
dequeued per atomic and stored as one group, 1..64): the tail of the dynamic
queue (a wave may finish one group after the others) against the partial-store
width (group x 8 B) and the number of queue atomics.

    python3 tools/probes/probe_group.py [fixture] [group ...]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "double__40_0.50_0"
# settings: "G" forces the group, "tT" the tail group (0 = no tail phase)
groups = sys.argv[2:] or ["t0", "t4", "t2", "t1", "8", "4"]
a = S.read_matrix(os.path.join("tests", "fixtures", name))[0]
n = a.shape[0]
S.prepare(a, "dense", jit=1)
ref = None
for g in ["default"] + groups:
    os.environ.pop("SUP_WALK_GROUP", None)
    os.environ.pop("SUP_WALK_TAIL", None)
    if g.startswith("t"):
        os.environ["SUP_WALK_TAIL"] = g[1:]
    elif g != "default":
        os.environ["SUP_WALK_GROUP"] = g
    ks = []
    for _ in range(5):
        v, st = S.perman_shard(a, 0, 1, kernel="dense", jit=1, return_stats=True)
        ks.append(st["kernel_ms"])
    ref = v if ref is None else ref
    print(f"{name} group {g}: kernel median {statistics.median(ks):.2f} ms (min {min(ks):.2f}) "
          f"same sum: {v == ref}", flush=True)
