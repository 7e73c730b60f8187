"""One walk launch for profiling: python tools/probes/run_one.py <fixture> <prep 0|1|2> <kernel> [reps] [jit]

Runs the engine's whole Gray walk for tests/fixtures/<fixture> (after -r <prep>)
`reps` times through sup_perman_shard (one launch each) and prints the kernel
time and rate; meant to sit under rocprofv3 --pmc / --stats.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

name, prep, kernel = sys.argv[1], int(sys.argv[2]), sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
jit = int(sys.argv[5]) if len(sys.argv) > 5 else 0  # -1: the ahead-of-time kernel itself
a, _, _ = S.read_matrix(os.path.join("tests", "fixtures", name))
if prep == 1:
    a = S.sort_order(a)[0]
elif prep == 2:
    a = S.skip_order(a)[0]
n = a.shape[0]
for _ in range(reps):
    v, st = S.perman_shard(a, 0, 1, kernel=kernel, jit=jit, return_stats=True)
    print(f"{name} r{prep} {kernel}: walk={st['walk_kind']} est_ops={st['est_ops_per_step']:.1f} "
          f"kernel={st['kernel_ms']:.1f} ms steps/s={2 ** (n - 1) / (st['kernel_ms'] * 1e-3):.3e} "
          f"visited={st['visited_steps']:.3e}", flush=True)
