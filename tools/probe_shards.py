"""GPU probe: the 8 bench shards of the n = 40 headline (sup_perman_shard, the
per-rank call of `bench.py --gpus 8`), walked one after another on one device:
per-shard kernel time against the whole walk, and their sum == the whole
permanent's raw sum (pairwise subtrees)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "double__40_0.50_0"))[0]
S.prepare(a, "dense", jit=1, gpu_num=8)
whole, st = S.perman_shard(a, 0, 1, kernel="dense", jit=1, return_stats=True)
whole, st = S.perman_shard(a, 0, 1, kernel="dense", jit=1, return_stats=True)
print(f"whole walk: kernel {st['kernel_ms']:.1f} ms", flush=True)
for world in (2, 4, 8):
    parts, kms, walls = [], [], []
    for r in range(world):
        t = time.perf_counter()
        p, s = S.perman_shard(a, r, world, kernel="dense", jit=1, return_stats=True)
        walls.append((time.perf_counter() - t) * 1e3)
        parts.append(p)
        kms.append(s["kernel_ms"])
    while len(parts) > 1:  # pairwise, as the reduction tree
        parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
    print(f"{world} shards: kernel ms {min(kms):.2f}-{max(kms):.2f}, call ms {min(walls):.2f}-{max(walls):.2f}, "
          f"ideal speedup {st['kernel_ms'] / max(kms):.2f}x, pairwise sum == whole: {parts[0] == whole}", flush=True)
