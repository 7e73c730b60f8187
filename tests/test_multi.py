"""N > 1 path on CPU: gloo, world_size 2, 4 and 8 — the bench's shard
arithmetic and its single all-reduce reproduce the 1-device sum bit for bit.
Each rank's shard is walked by the oracle's mirror of the engine schedule (the
CPU stand-in for the GPU kernel, which is bit-identical to it)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mat, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch

    import bench
    import oracle
    import superman_amd as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = mat.shape[0]
    c0, c1 = bench.shard_chunks(n, rank, world)
    info = S.plan_info(mat, "dense")  # the plan sup_perman_shard runs
    part, _ = oracle.engine_range(mat, info["kind"], c0, c1, info["L"], info["m"], info["colmap"], 1,
                                  info["cached"], info["pair_bits"])
    total = bench.combine(part, rank, world, "cpu")
    el = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put(((4 * (n & 1) - 2) * total, float(el.item()), (c0, c1)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_allreduce_matches_single(world, orc):
    n = 22
    mat = np.random.default_rng(5).random((n, n))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mat, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    got, max_rank, _ = res
    assert max_rank == world - 1
    import superman_amd as S
    want = orc.engine_perman_as(S, mat, "dense", threads=2)
    # bitwise: the shards are the top subtrees of the engine's pairwise tree,
    # the one-slot-per-rank all-reduce is exact and the fold is that tree's top
    assert got == want


def test_shard_chunks_cover_space():
    import bench
    import superman_amd as S
    for n in (8, 20, 33, 40):
        for world in (1, 2, 3, 4, 8):
            L, m, h = S.layout(n)
            b = [bench.shard_chunks(n, r, world) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == 1 << h
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            if world in (1, 2, 4, 8) and (1 << h) >= world:
                assert all((c1 - c0) == (1 << h) // world for c0, c1 in b)


def test_pairwise_fold_is_engine_tree():
    import bench
    v = np.random.default_rng(1).random(8).tolist()
    assert bench.pairwise(v) == ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]))
    assert bench.pairwise(v[:3]) == (v[0] + v[1]) + (v[2] + 0.0)
    assert bench.pairwise([2.5]) == 2.5


def _plan_worker(rank, world, port, mat, perturb, q):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    import superman_amd as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = mat.copy()
    if perturb and rank == world - 1:
        a[0, 0] += 1.0  # this rank would walk another matrix's plan
    # what bench.timed does before its warmup: plan (+ compile), then the key
    S.prepare(a, "dense", jit=1, gpu_num=world)
    info = S.plan_info(a, "dense", jit=1, gpu_num=world)
    key = S.plan_key(a, "dense", jit=1, gpu_num=world)
    try:
        keys = bench.check_plans_agree(key, rank, world, "cpu")
        out = ("ok", keys, info["kind"])
    except RuntimeError as e:
        out = ("mismatch", str(e), info["kind"])
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("perturb", [False, True])
def test_bench_plan_fingerprint_guard(perturb):
    """bench.py all-gathers every rank's plan fingerprint (sup_plan_key) after
    S.prepare and aborts when ranks planned different walks — a mismatch would
    otherwise sum shards of two enumerations into a silently wrong permanent."""
    n, world = 24, 2
    rng = np.random.default_rng(17)
    mat = np.where(rng.random((n, n)) < 0.5, rng.random((n, n)) * 5, 0.0)
    mat[np.arange(n), rng.permutation(n)] = 1.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, mat, perturb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        status, detail, kind = res[r]
        assert kind == "seg"
        if perturb:
            assert status == "mismatch" and "planned different walks" in detail
        else:
            assert status == "ok" and len(set(detail)) == 1


def _auto_worker(rank, world, port, mat, dirs, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["SUP_JIT_CACHE_DIR"] = dirs[rank]
    import bench
    import superman_amd as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    naive = S.plan_info(mat, "dense", jit=0, gpu_num=world)["kind"]  # this rank's own auto decision
    jit = bench.auto_decision(S, mat, "dense", rank, world, 0, "cpu")
    key = S.plan_key(mat, "dense", jit=jit, gpu_num=world)
    try:
        bench.check_plans_agree(key, rank, world, "cpu")
        status = "ok"
    except RuntimeError as e:
        status = str(e)
    q.put((rank, (naive, jit, status)))
    dist.destroy_process_group()


def test_bench_auto_mode_decided_by_rank0(tmp_path):
    """Auto mode (jit = 0) decides from the disk cache's state, which ranks see
    at different moments: here rank 1's cache already holds the bench matrix's
    segmented-walk choices (warm: specialise when it saves > 0.1 s) and rank
    0's is empty (cold: > 3 s), so on their own they would plan different
    walks.  bench.auto_decision makes rank 0's choice everyone's."""
    import superman_amd as S
    from conftest import fixture_path
    a, _, _ = S.read_matrix(fixture_path("double__40_0.50_0"))
    warm, cold = tmp_path / "warm", tmp_path / "cold"
    warm.mkdir()
    cold.mkdir()
    os.environ["SUP_JIT_CACHE_DIR"] = str(warm)
    try:  # record the pattern's choices (a scaled copy: same pattern, not in this process's plan cache)
        assert S.plan_info(0.125 * a, "dense", jit=1)["kind"] == "seg"
    finally:
        del os.environ["SUP_JIT_CACHE_DIR"]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    dirs = [str(cold), str(warm)]
    procs = [ctx.Process(target=_auto_worker, args=(r, world, port, a, dirs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][0] == "sparse" and res[1][0] == "seg"  # left alone, the ranks disagree
    for r in range(world):
        assert res[r][1] == -1 and res[r][2] == "ok"  # rank 0's choice (the ahead-of-time walk) for all
