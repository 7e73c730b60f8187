"""GPU probe: where a short walk's per-call cost goes.  Calls config 2's bench
step (sup_perman_shard on double__32_0.50_0, --jit 1) back to back through the
prepared ShardCall, as bench.py times it, and prints the wall time per call
beside the walk kernel's.  Under `rocprofv3 --kernel-trace` the dispatch
timestamps split the rest: walk end -> reduction passes -> the next walk's
start (host: flag wait, Python, launch).  Analyse the trace with
`python3 tools/probes/probe_callgap.py --trace <kernel_trace.csv>`.

usage: python3 tools/probes/probe_callgap.py [calls] [fixture]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def analyse(path):
    import csv
    import statistics as st
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    walks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("sup_walk")]
    walks = walks[len(walks) // 4:]  # steady state
    cols = {"walk": [], "walk_end->next": [], "after_walk_kernels": [], "gpu_busy_between": [], "idle_between": []}
    for a, b in zip(walks, walks[1:]):
        w = rows[a]
        ws, we = int(w["Start_Timestamp"]), int(w["End_Timestamp"])
        cols["walk"].append((we - ws) / 1e3)
        cols["walk_end->next"].append((int(rows[b]["Start_Timestamp"]) - we) / 1e3)
        mid = rows[a + 1:b]
        cols["after_walk_kernels"].append(len(mid))
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in mid) / 1e3
        cols["gpu_busy_between"].append(busy)
        last = max([int(r["End_Timestamp"]) for r in mid] + [we])
        cols["idle_between"].append((int(rows[b]["Start_Timestamp"]) - last) / 1e3)
    names = sorted({rows[i]["Kernel_Name"][:60] for w in walks for i in range(w + 1, w + 3) if i < len(rows)})
    print("kernels after a walk:", names)
    for k, v in cols.items():
        print(f"{k:>22}: median {st.median(v):9.2f}  min {min(v):9.2f}  max {max(v):9.2f}  (us or count)")
    if len(walks) > 1:
        gaps = []
        for a in walks:
            for i in range(a + 1, min(a + 4, len(rows))):
                if rows[i]["Kernel_Name"].startswith("sup_walk"):
                    break
                prev_end = int(rows[i - 1]["End_Timestamp"])
                gaps.append((rows[i]["Kernel_Name"][:40], (int(rows[i]["Start_Timestamp"]) - prev_end) / 1e3,
                             (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3))
        by = {}
        for nm, g, d in gaps:
            by.setdefault(nm, []).append((g, d))
        for nm, v in by.items():
            print(f"  {nm}: gap before median {st.median(x for x, _ in v):.2f} us, duration median "
                  f"{st.median(y for _, y in v):.2f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--trace":
        analyse(sys.argv[2])
        sys.exit(0)
    import superman_amd as S
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    fixture = sys.argv[2] if len(sys.argv) > 2 else "double__32_0.50_0"
    a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", fixture))[0]
    S.prepare(a, "dense", jit=1)
    call = S.ShardCall(a, 0, 1, kernel="dense", jit=1)
    for _ in range(50):
        call()
    walls, kms = [], []
    t0 = time.perf_counter()
    for _ in range(calls):
        t = time.perf_counter()
        _, k = call()
        walls.append((time.perf_counter() - t) * 1e3)
        kms.append(k)
    total = (time.perf_counter() - t0) * 1e3
    walls.sort()
    kms.sort()
    print(f"{fixture}: {calls} calls, {total / calls:.4f} ms per call; wall median {walls[len(walls) // 2]:.4f} ms, "
          f"walk kernel median {kms[len(kms) // 2]:.4f} ms, beyond the walk {(walls[len(walls) // 2] - kms[len(kms) // 2]) * 1e3:.1f} us",
          flush=True)
