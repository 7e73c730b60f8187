"""Walk-kernel time of the segmented walk at fixed live-value budgets
(SUP_JIT_BUDGET, no compiler check) next to the budget the compiler check
picks, on one matrix: which scratch the kernels keep (codescan) and what it
costs in time.

    python3 tools/probes/probe_budgets.py [fixture] [budget ...]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "double__40_0.50_0"
budgets = [int(b) for b in sys.argv[2:]] or [184, 190, 196, 202, 208, 214, 220]
a = S.read_matrix(os.path.join("tests", "fixtures", name))[0]
n = a.shape[0]


def timed(label):
    info = S.plan_info(a, "seg", jit=1)
    S.perman_shard(a, 0, 1, kernel="seg", jit=1)  # compile + warm
    ks, v = [], None
    for _ in range(5):
        v, st = S.perman_shard(a, 0, 1, kernel="seg", jit=1, return_stats=True)
        ks.append(st["kernel_ms"])
    k = statistics.median(ks)
    print(f"{name} {label}: ops/step {info['est_ops_per_step']:.4f} cc {info['cached']} b {info['pair_bits']} "
          f"kernel median {k:.2f} ms (min {min(ks):.2f}) {2 ** (n - 1) / (k * 1e-3):.4e} steps/s sum {v!r}",
          flush=True)


timed("checked (default)")
for b in budgets:
    os.environ["SUP_JIT_BUDGET"] = str(b)
    timed(f"budget {b}")
del os.environ["SUP_JIT_BUDGET"]
