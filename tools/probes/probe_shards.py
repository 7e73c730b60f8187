"""GPU probe: the 8 bench shards of the n = 40 headline (sup_perman_shard, the
per-rank call of `bench.py --gpus 8`), walked one after another on one device:
per-shard kernel time against the whole walk, and their sum == the whole
permanent's raw sum (pairwise subtrees)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

# the n = 40 headline, and config 5 (n = 44 d = 0.15 int, -p8 -s -r2: the
# segmented walk skips 87 % of its wave-chunks; the planner's column order
# keeps the shards' skip patterns equal, engine.cpp make_plan)
cases = [("dense n=40 d=0.5 (bench)", S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "double__40_0.50_0"))[0],
          "dense"),
         ("config 2 n=32 d=0.5", S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "double__32_0.50_0"))[0], "dense"),
         ("d=0.2 n=40", S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "double__40_0.20_0"))[0], "dense"),
         ("config 5 n=44 d=0.15 int -p8 -s -r2",
          S.skip_order(S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "synth44_0.15_int"))[0])[0], "skip")]
for name, a, kern in cases:
    S.prepare(a, kern, jit=1, gpu_num=8)
    whole, st = S.perman_shard(a, 0, 1, kernel=kern, jit=1, return_stats=True)
    whole, st = S.perman_shard(a, 0, 1, kernel=kern, jit=1, return_stats=True)
    print(f"{name}: whole walk: kernel {st['kernel_ms']:.1f} ms", flush=True)
    for world in (2, 4, 8):
        for r in range(world):  # warm each shard's call (its tables, flags)
            S.perman_shard(a, r, world, kernel=kern, jit=1)
        parts, kms, walls, vis = [], [], [], []
        for r in range(world):
            t = time.perf_counter()
            p, s = S.perman_shard(a, r, world, kernel=kern, jit=1, return_stats=True)
            walls.append((time.perf_counter() - t) * 1e3)
            parts.append(p)
            kms.append(s["kernel_ms"])
            vis.append(s["visited_steps"])
        while len(parts) > 1:  # pairwise, as the reduction tree
            parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
        print(f"  {world} shards: kernel ms {min(kms):.2f}-{max(kms):.2f}, call ms {min(walls):.2f}-{max(walls):.2f}, "
              f"visited {min(vis)}-{max(vis)}, ideal speedup {st['kernel_ms'] / max(kms):.2f}x, "
              f"pairwise sum == whole: {parts[0] == whole}", flush=True)
