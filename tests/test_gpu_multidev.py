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
