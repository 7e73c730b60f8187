"""The seeded random sweep of test_gpu_fuzz.py on the host walks (no GPU): the
CPU worker's walks (sup_perman_cpu: the same plans on host threads, what the
hybrid -c worker runs) bit-exact against the oracle's mirror, and the engine's
exact path on host threads equal to the oracle's own residue Ryser."""
import numpy as np
import pytest

from test_gpu_fuzz import _case, _walks

SEEDS = list(range(36))  # n <= 24


@pytest.mark.parametrize("seed", SEEDS)
def test_host_walks_bitexact_vs_mirror(sup, orc, seed):
    a, integer = _case(seed)
    n = a.shape[0]
    for kernel, jit in _walks(n):
        kind = sup.plan_info(a, kernel, jit=jit)["kind"]
        want = orc.engine_perman_as(sup, a, kernel, threads=8, jit=jit)
        assert sup.perman_cpu(a, "seg" if kind == "seg" else kernel, threads=8) == want, (seed, n, kernel)
    if (a >= 0).all():
        for order, kernel in ((sup.sort_order, "sparse"), (sup.skip_order, "skip")):
            b = order(a)[0]
            want = orc.engine_perman_as(sup, b, kernel, threads=8, jit=-1)
            assert sup.perman_cpu(b, kernel, threads=8) == want, (seed, n, kernel)
    if integer and n <= 20:
        ai = a.astype(np.int64)
        assert sup.perman_exact(ai.astype(np.int32), cpu=True) == orc.exact_perman_crt(ai, threads=8), (seed, n)
