"""Kernel time against the wave-chunk's walk length (walk_log2 = m walk bits).

python tools/probes/probe_walklen.py [m ...]   (0 = the default layout)

Each (matrix, m) is planned and compiled once, then timed best-of-3 through
sup_perman_shard; prints the kernel time, nominal Gray steps/s and the chunk
count, so the per-chunk start cost (row copies, trees, column sums of the
start index) can be weighed against tail balance.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd as S  # noqa: E402

CASES = [("double__40_0.50_0", 0, "dense"), ("double__40_0.20_0", 0, "dense"), ("double__40_0.90_0", 0, "dense"),
         ("double__32_0.50_0", 0, "dense"), ("double__36_0.20_0", 1, "sparse"), ("synth44_0.15_int", 2, "sparse")]
if os.environ.get("PROBE_CASES"):
    CASES = [c for c in CASES if c[0] in os.environ["PROBE_CASES"].split(",")]
ms = [int(v) for v in sys.argv[1:]] or [0, 11, 12, 13, 14, 15, 16]
for name, prep, kernel in CASES:
    a, _, _ = S.read_matrix(os.path.join("tests", "fixtures", name))
    if prep == 1:
        a = S.sort_order(a)[0]
    elif prep == 2:
        a = S.skip_order(a)[0]
    n = a.shape[0]
    for m in ms:
        if m and m > n - 1 - 6:
            continue
        best, v = None, None
        for _ in range(4):
            v, st = S.perman_shard(a, 0, 1, kernel=kernel, walk_log2=m, jit=1, return_stats=True)
            k = st["kernel_ms"]
            best = k if best is None or k < best else best
        print(f"{name} m={m or 'default'} walk={st['walk_kind']} est_ops={st['est_ops_per_step']:.3f} "
              f"kernel={best:.3f} ms steps/s={2 ** (n - 1) / (best * 1e-3):.4e} perm={v:.15e}", flush=True)
