"""bench.py's entry point (no GPU needed): `--gpus N` and the launcher's
WORLD_SIZE must agree, and `--gpus N > 1` without torchrun and without N GPUs
fails loudly instead of silently measuring one rank.  The
launch itself (N ranks from plain python) is tests/test_gpu_multi.py."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=120, env=e)


def test_world_size_disagrees_with_gpus():
    r = _run(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
    assert not r.stdout.strip()


def test_gpus_without_devices_fails_loudly():
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip("this host has the GPUs")
    r = _run(["--gpus", "2", "--steps", "1"])
    assert r.returncode == 3
    assert "--rehearse" in r.stderr
    assert not r.stdout.strip()


def test_gpus_zero_refused():
    r = _run(["--gpus", "0"])
    assert r.returncode == 2


def test_hbm_profiles_found_for_every_bench_walk():
    """Every committed FETCH_SIZE / WRITE_SIZE profile of round 5 is found by
    the lookup the bench line uses, under the kernel name the bench reports
    (`sup::walk_skip<44>` for the ahead-of-time SkipPer kernel, whose profile
    records `walk_skip<44>`)."""
    import glob
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r5", "pmc_hbm_*.json")))
    assert paths
    for p in paths:
        d = json.load(open(p))
        kernel = d["kernel"] if d["kernel"].startswith("sup_") else "sup::" + d["kernel"]
        rec = b.pmc_record(d["n"], kernel, d["plan_key"])
        assert rec is not None, p
        assert b.hbm_traffic(rec) > d["algorithmic_bytes_per_launch"], p
