"""A/B of two builds of the library on one box: python3 tools/probes/probe_ab_lib.py <package root> [label].
Walks the headline (double__40_0.50_0, --jit 1) 5 times, config 2's bench step 300 times and config 3's 100 times through
the package under <package root> (e.g. a git worktree of an earlier commit, built in place) and prints
the walk-kernel times; run the roots alternately in separate processes."""
import os
import statistics as st
import sys
import time

root = os.path.abspath(sys.argv[1])
sys.path.insert(0, root)
import superman_amd as S  # noqa: E402

assert os.path.dirname(os.path.abspath(S.__file__)).startswith(root), S.__file__
fx = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "fixtures")
out = []
for name, reps, prep, kern in (("double__40_0.50_0", 5, 0, "dense"), ("double__32_0.50_0", 300, 0, "dense"),
                               ("double__36_0.20_0", 100, 1, "sparse")):
    a = S.read_matrix(os.path.join(fx, name))[0]
    if prep:
        a = S.sort_order(a)[0]
    S.prepare(a, kern, jit=1)
    call = S.ShardCall(a, 0, 1, kernel=kern, jit=1)
    for _ in range(2 if reps < 10 else 30):
        call()
    ks, ws = [], []
    for _ in range(reps):
        t = time.perf_counter()
        v, k = call()
        ws.append((time.perf_counter() - t) * 1e3)
        ks.append(k)
    out.append(f"{name}: kernel median {st.median(ks):.4f} ms, wall median {st.median(ws):.4f} ms, value {v!r}")
print(sys.argv[2] if len(sys.argv) > 2 else root, "|", " | ".join(out), flush=True)
