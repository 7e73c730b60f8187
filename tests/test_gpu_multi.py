"""The bench's one-process-per-GPU path with the HIP kernel on the card: N
ranks (gloo, all on device 0 — the rehearsal form of bench.py --rehearse)
each plan on their own, agree on the plan fingerprint, walk their contiguous
shard of wave-chunks with sup_perman_shard (the segmented walk, as the bench
times it) and combine with the bench's one-slot-per-rank all-reduce.  The
result equals the single-process walk bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, fixture_path

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, q):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    import superman_amd as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = S.read_matrix(path)[0]
        S.prepare(a, "dense", jit=1, gpu_num=world)
        bench.check_plans_agree(S.plan_key(a, "dense", jit=1, gpu_num=world), rank, world, "cpu")
        part, st = S.perman_shard(a, rank, world, kernel="dense", jit=1, return_stats=True)
        total = bench.combine(part, rank, world, "cpu")
        out = (total, st["walk_kind"], st["gray_steps"])
        if rank == 0:
            whole, st1 = S.perman_shard(a, 0, 1, kernel="dense", jit=1, return_stats=True)
            out = out + (whole, st1["gray_steps"])
        q.put((rank, out))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, ("error", repr(e))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gpu_shards_allreduce_bitwise(world):
    path = fixture_path("double__32_0.50_0")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r][0] != "error", res[r]
    total, kind, steps, whole, whole_steps = res[0]
    assert kind == 3  # the segmented walk the bench times
    assert steps * world == whole_steps == 1 << 31
    assert total == whole  # power-of-two shards are subtrees of the fixed pairwise tree
    assert all(res[r][0] == total for r in range(world))


def _bench(args, env=None):
    import json
    import subprocess
    import sys
    e = dict(os.environ, **(env or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, env=e)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


_QUICK = ["--steps", "1", "--warmup", "0", "--configs", "0", "--cpu-seconds", "0", "--pmc", "0", "--cold", "0",
          "--also", ""]


def test_bench_gpus_flag_launches_ranks():
    """`python3 bench.py --gpus 2` from plain python (no torchrun, no
    WORLD_SIZE) starts the 2 ranks itself (torch.distributed.run as a child):
    one JSON line with n_gpus 2, the ranks' plan keys equal, the permanent
    bit-equal to the one-rank run."""
    r2, out2 = _bench(["--gpus", "2", "--rehearse", *_QUICK])
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert len(out2) == 1, r2.stdout
    rec2 = out2[0]
    assert rec2["n_gpus"] == 2
    keys = rec2["plan_keys_per_rank"]
    assert len(keys) == 2 and keys[0] == keys[1]
    r1, out1 = _bench(["--gpus", "1", *_QUICK])
    assert r1.returncode == 0, r1.stderr[-3000:]
    assert len(out1) == 1 and out1[0]["n_gpus"] == 1
    assert out1[0]["plan_keys_per_rank"] == [keys[0]]
    assert rec2["permanent"] == out1[0]["permanent"]


def test_bench_gpus_flag_refuses_missing_gpus():
    """Without --rehearse, --gpus N on a node with fewer GPUs fails loudly
    instead of measuring one rank."""
    import torch
    n = torch.cuda.device_count() + 1
    r, out = _bench(["--gpus", str(n), *_QUICK])
    assert r.returncode != 0 and not out
    assert "GPU" in r.stderr
