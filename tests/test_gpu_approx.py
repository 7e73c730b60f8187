"""GPU estimators (approx.hip) against the host threads and the restatement.

A sample's estimate depends only on (seed, sample index), and block sums are
folded in a fixed pairwise order, so the GPU result must equal the CPU result
bit for bit, for one device, the multi-device form and the hybrid CPU worker.
"""
import numpy as np
import pytest

from oracle import approx as A

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu(sup):
    if sup.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")


def _cases(sup):
    rng = np.random.default_rng(31)
    a = (rng.random((20, 20)) < 0.3).astype(np.int32)
    a[np.arange(20), rng.permutation(20)] = 1
    return [a, sup.grid_graph(8, 8), sup.grid_graph(10, 13), sup.grid_graph(36, 36)]


@pytest.mark.parametrize("algo", [1, 2])
def test_gpu_equals_cpu_bitwise(sup, algo):
    for g in _cases(sup):
        samples = 64 * 50 if g.shape[0] > 300 else 64 * 2000
        c = sup.approx(g, algo, samples=samples, seed=17, cpu=True, threads=16)
        r, st = sup.approx(g, algo, samples=samples, seed=17, return_stats=True)
        assert r == c, (g.shape, algo)
        assert st["devices"] == 1 and st["kernel_ms"] > 0
        # multi-device form (-p3 / -p4) and the hybrid CPU worker give the same bits
        assert sup.approx(g, algo + 2, samples=samples, seed=17, gpu_num=1, cpu_worker=True, threads=4) == c


def test_gpu_block_matches_restatement(sup):
    a = _cases(sup)[0][:10, :10].copy()
    a[np.arange(10), np.arange(10)] = 1
    for algo, method in ((1, "rasmussen"), (2, "scaling")):
        want = A.block_sums(a, method, seed=5, block=0)
        assert sup.approx(a, algo, samples=64, seed=5) == want[0] / 64.0


def test_gpu_unbiased_grid(sup):
    g = sup.grid_graph(8, 8)
    t = A.domino_tilings(8, 8)
    for algo in (1, 2):
        est, st = sup.approx(g, algo, samples=1 << 22, seed=23, return_stats=True)
        assert abs(est - t) < 5 * st["std_error"], (algo, est, t, st["std_error"])
        assert st["std_error"] < 0.01 * t


@pytest.mark.parametrize("algo", [1, 2])
def test_gpu_coop_equals_per_lane(sup, monkeypatch, algo):
    """The cooperative form (one wave per sample, factors in LDS; approx.hip
    approx_coop) gives every block sum of the per-lane form bit for bit."""
    for g, samples in ((sup.grid_graph(10, 13), 4096), (sup.grid_graph(16, 16), 2048), (sup.grid_graph(36, 36), 256)):
        got = {}
        for form in ("0", "1"):
            monkeypatch.setenv("SUP_APPROX_COOP", form)
            got[form] = sup.approx(g, algo, samples=samples, seed=29, return_stats=True)
        assert got["0"][0] == got["1"][0]
        assert got["0"][1]["std_error"] == got["1"][1]["std_error"]
