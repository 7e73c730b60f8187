"""The in-process multi-device schedulers (reference -p5 / -p6 / -p66 / -p8 with
one OpenMP thread per device, gpu_exact_dense.cu:701-990,
gpu_exact_sparse.cu:1192-1400) run with G > 1 on a one-GPU box.

SUP_DEVICE_MAP="0,0,0,0" presents four logical devices on physical device 0,
each with its own context (stream, buffers, chunk queue), so the per-device
threads, their kernels (concurrently on one GPU), the item queue with several
takers and the host combine all run as they would on four GPUs.  Results must
equal the one-device walk bit for bit: pieces and queue items are aligned
subtrees of the one fixed pairwise reduction.  RCCL (-R)
needs distinct physical devices and is refused under such a map."""
import os
from contextlib import contextmanager

import numpy as np
import pytest

from conftest import fixture_path

pytestmark = pytest.mark.gpu


@contextmanager
def device_map(spec: str):
    old = os.environ.get("SUP_DEVICE_MAP")
    os.environ["SUP_DEVICE_MAP"] = spec
    try:
        yield
    finally:
        if old is None:
            del os.environ["SUP_DEVICE_MAP"]
        else:
            os.environ["SUP_DEVICE_MAP"] = old


def test_device_map_count(sup):
    phys = sup.device_count()
    with device_map(",".join(["0"] * 4)):
        assert sup.device_count() == 4
    with device_map(str(phys)):  # a physical id that does not exist
        assert sup.device_count() == 0
    assert sup.device_count() == phys


@pytest.mark.parametrize("jit", [-1, 1])
def test_dense_multidevice_threads(sup, jit):
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    one, st1 = sup.perman(a, 4, jit=jit, return_stats=True)
    with device_map("0,0,0,0"):
        for G in (2, 3, 4):
            r5, st = sup.perman(a, 5, gpu_num=G, jit=jit, return_stats=True)
            assert st["devices_used"] == G
            if G != 3:  # power-of-two pieces are subtrees of the one-device tree
                assert r5 == one, (G, r5, one)
            else:
                assert abs(r5 - one) <= 1e-12 * abs(one)
            r6, st = sup.perman(a, 6, gpu_num=G, jit=jit, return_stats=True)
            assert r6 == one, (G, r6, one)
            assert st["devices_used"] == G
        # dynamic queue with the hybrid CPU worker beside four device threads
        r6c, st = sup.perman(a, 6, gpu_num=4, cpu=True, threads=4, jit=jit, return_stats=True)
        assert r6c == one
        # -p66: eight pieces owned {0,0,0,1,1,1,2,3}
        assert sup.perman(a, 66, gpu_num=4, jit=jit) == one
    if jit == 1:
        assert st1["walk_kind"] == 3  # the segmented walk ran on every logical device


def test_sparse_and_skipper_multidevice_threads(sup):
    a, _, _ = sup.read_matrix(fixture_path("int__30_0.20_0"))
    s = sup.sort_order(a)[0]
    k = sup.skip_order(a)[0]
    sp1 = sup.perman(s, 4, sparse=True)
    sk1 = sup.perman(k, 7, sparse=True, jit=-1)
    with device_map("0,0,0,0"):
        assert sup.perman(s, 5, sparse=True, gpu_num=4) == sp1
        assert sup.perman(s, 6, sparse=True, gpu_num=4) == sp1
        assert sup.perman(s, 6, sparse=True, gpu_num=4, cpu=True, threads=4) == sp1
        assert sup.perman(k, 8, sparse=True, gpu_num=4, jit=-1) == sk1
        assert sup.perman(k, 8, sparse=True, gpu_num=4, jit=-1, cpu=True, threads=4) == sk1


def test_exact_quad_approx_multidevice(sup):
    rng = np.random.default_rng(31)
    n = 26
    a = np.where(rng.random((n, n)) < 0.4, rng.integers(1, 4, (n, n)), 0).astype(np.int32)
    ex1 = sup.perman_exact(a)
    q1 = sup.perman_quad(a)
    g = sup.grid_graph(6, 6)
    e1 = sup.approx(g, 1, samples=64 * 256, seed=5)
    with device_map("0,0,0,0"):
        assert sup.perman_exact(a, gpu_num=4) == ex1
        assert sup.perman_exact(a, gpu_num=3, cpu_worker=True, threads=4) == ex1
        assert sup.perman_quad(a, gpu_num=4) == q1
        assert sup.approx(g, 3, samples=64 * 256, seed=5, gpu_num=4) == e1  # -a 3: the multi-device Rasmussen


def test_rccl_refused_on_shared_device(sup):
    a, _, _ = sup.read_matrix(fixture_path("synth/22_0.50_double"))
    with device_map("0,0"):
        with pytest.raises(sup.SupError) as e:
            sup.perman(a, 5, gpu_num=2, use_rccl=True)
        assert "distinct physical devices" in str(e.value)
        # the host combine still runs
        assert sup.perman(a, 5, gpu_num=2) == sup.perman(a, 4)


def _cli(args, cache, devices=8, extra_env=None):
    """Run the drop-in CLI under SUP_DEVICE_MAP (all logical devices on GPU 0)
    with the device-placement assertions on; (Permanent line, stats dict)."""
    import subprocess
    from conftest import ROOT
    env = dict(os.environ, SUP_JIT_CACHE_DIR=str(cache), SUP_CHECK_DEVICE="1",
               SUP_DEVICE_MAP=",".join(["0"] * devices), **(extra_env or {}))
    r = subprocess.run([os.path.join(ROOT, "superman_amd", "bin", "perman"), *args, "-v"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, (args, r.stdout[-2000:], r.stderr[-2000:])
    lines = r.stdout.splitlines()
    perm = [ln for ln in lines if ln.startswith("Permanent:")][0]
    stats = [ln for ln in lines if ln.startswith("Stats:")][0].split()[1:]
    return perm, {stats[i]: stats[i + 1] for i in range(0, len(stats) - 1, 2)}


@pytest.mark.parametrize("jit", ["1", "-1"])
def test_baseline_config4_cli_p6_d8(tmp_path, jit):
    """BASELINE config 4 as written: `perman -f double/40_0.50_0 -g -p6 -d8`,
    on 8 logical devices (one host thread, context and chunk queue taker
    each), bit-equal to `-p4` with the same --jit; and with the hybrid CPU
    worker (-c) as a ninth taker.  Every allocation, module load and launch
    passes the SUP_CHECK_DEVICE assertion (gpu_exact_dense.cu:776-904)."""
    m = fixture_path("double__40_0.50_0")
    one, s1 = _cli(["-f", m, "-g", "-p4", "--jit", jit], tmp_path, devices=1)
    eight, s8 = _cli(["-f", m, "-g", "-p6", "-d8", "--jit", jit], tmp_path)
    assert eight == one
    assert s8["devices"] == "8" and s8["walk_kind"] == s1["walk_kind"] == ("3" if jit == "1" else "1")
    assert int(s8["device_checks"]) >= 8 * 3  # every device thread: buffers, launch, reduction
    hybrid, sh = _cli(["-f", m, "-g", "-c", "-p6", "-d8", "--jit", jit], tmp_path)
    assert hybrid == one and sh["devices"] == "8"


@pytest.mark.parametrize("jit", ["1", "-1"])
def test_baseline_config5_cli_p8_d8(tmp_path, jit):
    """BASELINE config 5 as written: `perman -f synth44_0.15_int -g -p8 -s -r2
    -d8` (SkipPer request, SkipOrder) on 8 logical devices, bit-equal to -d1
    with the same --jit (1: the segmented walk with the chunk skip; -1: the
    SkipPer kernel itself) and with the hybrid CPU worker
    (gpu_exact_sparse.cu:1192-1324)."""
    m = fixture_path("synth44_0.15_int")
    one, s1 = _cli(["-f", m, "-g", "-p8", "-s", "-r2", "-d1", "--jit", jit], tmp_path, devices=1)
    eight, s8 = _cli(["-f", m, "-g", "-p8", "-s", "-r2", "-d8", "--jit", jit], tmp_path)
    assert eight == one
    assert s8["devices"] == "8" and s8["walk_kind"] == s1["walk_kind"] == ("3" if jit == "1" else "2")
    assert s8["visited"] == s1["visited"]
    assert int(s8["device_checks"]) >= 8 * 3
    if jit == "1":  # the CPU worker's item of the SkipPer kernel's walk would take minutes on the host
        hybrid, sh = _cli(["-f", m, "-g", "-c", "-p8", "-s", "-r2", "-d8", "--jit", jit], tmp_path)
        assert hybrid == one


def test_device_checks_in_process(tmp_path):
    """The in-process schedulers under SUP_CHECK_DEVICE=1 (read once per
    process, so in a child): -p5/-p6/-p8 on 4 logical devices, the exact,
    double-double and estimator multi-device forms; checks counted."""
    import subprocess
    import sys
    from conftest import ROOT
    code = (
        "import numpy as np, superman_amd as S\n"
        "from conftest import fixture_path\n"
        "a = S.read_matrix(fixture_path('double__30_0.50_0'))[0]\n"
        "one = S.perman(a, 4, jit=1)\n"
        "assert S.perman(a, 5, gpu_num=4, jit=1) == one and S.perman(a, 6, gpu_num=4, jit=1) == one\n"
        "assert S.perman(a, 6, gpu_num=4, jit=-1, cpu=True, threads=4) == S.perman(a, 4, jit=-1)\n"
        "k = S.skip_order(S.read_matrix(fixture_path('int__30_0.20_0'))[0])[0]\n"
        "assert S.perman(k, 8, sparse=True, gpu_num=4, jit=-1) == S.perman(k, 7, sparse=True, jit=-1)\n"
        "i = np.where(np.random.default_rng(3).random((24, 24)) < 0.4, 2, 0).astype(np.int32)\n"
        "np.fill_diagonal(i, 1)\n"
        "assert S.perman_exact(i, gpu_num=4) == S.perman_exact(i)\n"
        "assert S.perman_quad(i, gpu_num=4) == S.perman_quad(i)\n"
        "g = S.grid_graph(6, 6)\n"
        "assert S.approx(g, 3, samples=64 * 256, seed=5, gpu_num=4) == S.approx(g, 1, samples=64 * 256, seed=5)\n"
        "print('checks', S._lib.load().sup_device_checks())\n")
    env = dict(os.environ, SUP_CHECK_DEVICE="1", SUP_DEVICE_MAP="0,0,0,0", SUP_JIT_CACHE_DIR=str(tmp_path),
               PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert int(r.stdout.split("checks")[1]) > 50
