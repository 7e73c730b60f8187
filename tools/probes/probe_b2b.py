"""Back-to-back bench steps of one walk under the environment it is started with (code-generation knobs:
SUP_JIT_*): python3 tools/probes/probe_b2b.py <fixture> <prep> <kernel> [calls].  Prints wall per call and the
walk-kernel time (deferred HIP events), as bench.py's config legs time them."""
import os
import sys
import time

if os.environ.get("PROBE_IMPORT_TORCH"):  # as bench.py: torch (and its HIP runtime) loaded first
    import torch  # noqa: F401
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

name, prep, kern = sys.argv[1], int(sys.argv[2]), sys.argv[3]
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 500
a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", name))[0]
if prep == 1:
    a = S.sort_order(a)[0]
elif prep == 2:
    a = S.skip_order(a)[0]
S.prepare(a, kern, jit=1)
c = S.ShardCall(a, 0, 1, kernel=kern, jit=1, timing=False)
for _ in range(min(50, calls)):
    v = c()[0]
S.kernel_time(0)
res = []
for rnd in range(3):
    t0 = time.perf_counter()
    for _ in range(calls):
        c()
    wall = (time.perf_counter() - t0) / calls * 1e3
    tot, n = S.kernel_time(0)
    res.append(f"{wall:.4f}/{tot / n:.4f}")
knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items())
                 if k.startswith("SUP_JIT_") or k in ("SUP_RESULT_SYS", "SUP_FOLD", "SUP_WALK_TAIL", "PROBE_IMPORT_TORCH"))
print(f"{name} [{knobs or 'default'}] ms per call / kernel: {' '.join(res)}  value {v!r}", flush=True)
