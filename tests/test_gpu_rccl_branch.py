"""The RCCL code the driver's N-GPU bench run takes, executed on the real
device at world 1 (a one-GPU box cannot hold two RCCL ranks: RCCL refuses two
ranks on one GPU).

bench.py --pg creates the process group exactly as the N-rank run does
(`init_process_group("nccl", device_id=cuda:<local rank>)` under
torch.distributed.run) and runs every collective of that branch on `cuda:`
tensors: the plan-key all-gather (check_plans_agree), the shard combine's
one-slot-per-rank all-reduce, the steps / elapsed MAX all-reduces, the
visited-count all-reduce of the config lines and the kernel-time all-gather.
Its JSON line must be bit-equal to the run without a process group.  The
library's own RCCL combine (-p5 / -p6 / -p8 with use_rccl = 2, one
communicator from ncclCommInitAll) then runs in a process that already holds
torch's RCCL communicator.  The reference sums its device partials on the
host (gpu_exact_dense.cu:847-901); DESIGN.md §5."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT, fixture_path

pytestmark = pytest.mark.gpu

_QUICK = ["--steps", "1", "--warmup", "1", "--cpu-seconds", "0", "--pmc", "0", "--cold", "0", "--also", ""]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return e


def _launch(script_args, extra_env=None, timeout=420):
    """torch.distributed.run, one rank on this box's GPU, as the driver's
    N-GPU bench run starts every rank."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", *script_args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=dict(_env(), **(extra_env or {})))
    return r, [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_rccl_branch_world1_bitwise():
    """The headline and the BASELINE config lines through bench.py's
    process-group branch on RCCL, bit-equal to the same run without it."""
    r, out = _launch([os.path.join(ROOT, "bench.py"), "--gpus", "1", "--pg", *_QUICK])
    assert r.returncode == 0, r.stderr[-4000:]
    assert len(out) == 1, r.stdout[-2000:]
    pg = out[0]
    r0 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *_QUICK],
                        capture_output=True, text=True, timeout=420, env=_env())
    assert r0.returncode == 0, r0.stderr[-4000:]
    plain = [json.loads(ln) for ln in r0.stdout.splitlines() if ln.startswith("{")][0]
    assert pg["process_group"] == "nccl" and plain["process_group"] is None
    assert pg["n_gpus"] == plain["n_gpus"] == 1
    assert pg["permanent"] == plain["permanent"]
    assert pg["plan_keys_per_rank"] == plain["plan_keys_per_rank"]
    assert len(pg["kernel_ms_per_rank"]) == 1
    assert len(pg["configs"]) == len(plain["configs"]) == 4
    for c_pg, c0 in zip(pg["configs"], plain["configs"]):
        assert c_pg["config"] == c0["config"]
        if c_pg["walk"] == c0["walk"]:  # auto mode (config 5, jit 0) is decided by rank 0 under a group
            assert c_pg["permanent"] == c0["permanent"], c_pg["config"]
            assert c_pg["visited_frac"] == c0["visited_frac"], c_pg["config"]
    # the first three lines pin their walk (--jit 1 / -1): no decision to differ
    assert [c["walk"] for c in pg["configs"][:3]] == [c["walk"] for c in plain["configs"][:3]]


_IN_PG = r"""
import json, os, sys
sys.path.insert(0, os.environ["SUP_ROOT"])
import torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
v = torch.ones(4, dtype=torch.float64, device="cuda:0")
dist.all_reduce(v)
import superman_amd as S
a = S.read_matrix(os.environ["SUP_M1"])[0]
k = S.skip_order(S.read_matrix(os.environ["SUP_M2"])[0])[0]
out = {"torch_allreduce": v.cpu().tolist(),
       "p4": S.perman(a, 4), "p5_rccl": S.perman(a, 5, gpu_num=1, use_rccl=2),
       "p6_rccl": S.perman(a, 6, gpu_num=1, use_rccl=2),
       "p6_rccl_items": S.perman(a, 6, gpu_num=1, use_rccl=2, chunk_log2=2),
       "p7": S.perman(k, 7, sparse=True, jit=-1),
       "p8_rccl": S.perman(k, 8, sparse=True, gpu_num=1, use_rccl=2, jit=-1)}
dist.all_reduce(v)  # torch's communicator still works after the library's
out["torch_allreduce_after"] = v.cpu().tolist()
dist.destroy_process_group()
print(json.dumps(out), flush=True)
"""


def test_library_rccl_combine_inside_torch_process_group(tmp_path):
    """The library's in-process RCCL combine (ncclCommInitAll + slot
    all-reduce) beside torch's RCCL communicator in one rank: bit-equal to the
    single-device walk, and torch's collective still runs afterwards."""
    script = tmp_path / "in_pg.py"
    script.write_text(_IN_PG)
    r, out = _launch([str(script)], {"SUP_ROOT": ROOT, "SUP_M1": fixture_path("double__32_0.50_0"),
                                     "SUP_M2": fixture_path("int__30_0.20_0")})
    assert r.returncode == 0, r.stderr[-4000:]
    d = out[0]
    assert d["torch_allreduce"] == [1.0] * 4 and d["torch_allreduce_after"] == [1.0] * 4
    assert d["p5_rccl"] == d["p4"] and d["p6_rccl"] == d["p4"] and d["p6_rccl_items"] == d["p4"]
    assert d["p8_rccl"] == d["p7"]


def _cli(args, env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.run([os.path.join(ROOT, "superman_amd", "bin", "perman"), *args], capture_output=True,
                          text=True, timeout=300, env=env)


def test_cli_combine_choice(tmp_path):
    """The CLI's multi-device combine: RCCL whenever the -d devices are
    distinct GPUs, else the host pairwise tree, named by -v.  On one GPU the
    shared map takes the host tree (and -R, which insists on RCCL, is refused);
    the single device has nothing to combine."""
    m = fixture_path("double__30_0.50_0")
    cache = {"SUP_JIT_CACHE_DIR": str(tmp_path)}
    one = _cli(["-f", m, "-g", "-p4", "-v"], cache)
    assert one.returncode == 0, one.stderr
    shared = _cli(["-f", m, "-g", "-p6", "-d2", "-v"], dict(cache, SUP_DEVICE_MAP="0,0"))
    assert shared.returncode == 0, shared.stderr
    assert "Combine: host pairwise tree over 2 devices (devices share a GPU)" in shared.stdout
    perm = [ln for ln in one.stdout.splitlines() if ln.startswith("Permanent:")]
    assert perm and perm == [ln for ln in shared.stdout.splitlines() if ln.startswith("Permanent:")]
    forced = _cli(["-f", m, "-g", "-p5", "-d2", "-R"], dict(cache, SUP_DEVICE_MAP="0,0"))
    assert forced.returncode != 0 and "distinct physical devices" in forced.stderr
    single = _cli(["-f", m, "-g", "-p6", "-d1", "-v"], cache)
    assert "Combine: host pairwise tree over 1 device\n" in single.stdout
