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
