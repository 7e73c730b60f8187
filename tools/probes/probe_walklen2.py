"""Walk length (m walk bits per wave-chunk) of the segmented walk on the bench
matrices, interleaved: kernel medians of 5 launches through sup_perman_shard
per setting; 0 = the planner's choice.

    python3 tools/probes/probe_walklen2.py [m ...]
"""
import os
import statistics
import sys

import torch  # noqa: F401  (torch's hiprtc, as bench.py)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

ms = [int(x) for x in sys.argv[1:]] or [0, 14, 15, 0, 14, 15]
for name in os.environ.get("PROBE_CASES", "double__40_0.50_0,double__40_0.90_0").split(","):
    a = S.read_matrix(os.path.join("tests", "fixtures", name))[0]
    for wl in ms:
        info = S.plan_info(a, "dense", jit=1, walk_log2=wl)
        S.perman_shard(a, 0, 1, kernel="dense", jit=1, walk_log2=wl)
        ks = []
        for _ in range(5):
            v, st = S.perman_shard(a, 0, 1, kernel="dense", jit=1, walk_log2=wl, return_stats=True)
            ks.append(st["kernel_ms"])
        print(f"{name} m={wl or info['m']}{'' if wl else ' (planner)'}: ops {info['est_ops_per_step']:.3f} "
              f"kernel median {statistics.median(ks):.3f} ms (min {min(ks):.3f}) sum {v!r}", flush=True)
