"""Maximum order (n = 64, the engine's limit; n = 63 for the odd sign) on the
GPU: aligned Gray-index ranges, including ranges whose chunk index sets the
top bits of the 2^63 space, through every kernel family.

* bit-exact against the oracle's mirror of the engine schedule (dense,
  SpaRyser, SkipPer: oracle/oracle.c orc_engine_range);
* within 1e-9 of the reference chunk helpers restated (cpu_perman64 /
  cpu_perman64_sparse / cpu_perman64_skipper, gpu_exact_dense.cu:6-69,
  gpu_exact_sparse.cu:6-191), the segmented walk included;
* orders above 64 are refused.
A whole n = 64 permanent is 2^63 Gray steps (~35 days on one MI355X at 3e12 steps/s), so the
full size is covered by ranges, as the reference's own chunk helpers cover it."""
import numpy as np
import pytest

from conftest import rel

pytestmark = pytest.mark.gpu


def _mat(n, d, seed, ints):
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < d
    mask[np.arange(n), rng.permutation(n)] = True
    vals = rng.integers(1, 6, (n, n)) if ints else rng.random((n, n)) * 2.0
    return np.where(mask, vals, 0).astype(np.float64)


def _layout(sup, n, s, e):
    L, m, _ = sup.layout(n)
    al = min((v & -v).bit_length() - 1 for v in (s, e))
    return L, min(m, al - L)


Q = 1 << 22
# chunk index k of [k Q, (k + 1) Q): the first, one with scattered bits, and the
# last but one below 2^62 (bits 22-61 of the Gray index set)
KS = (1, 0x5A5A5A5, (1 << 40) - 2)


@pytest.mark.parametrize("n", [63, 64])
def test_dense_max_order(sup, orc, n):
    a = _mat(n, 0.5, 100 + n, ints=False)
    for k in KS:
        s, e = k * Q, (k + 1) * Q
        got = sup.partial(a, s, e, kernel="dense_plain")
        assert rel(got, orc.ref_dense_partial(a, s, e, 8)) < 1e-9, k
        L, ml = _layout(sup, n, s, e)
        mir, _ = orc.engine_range(a, "dense", s >> (L + ml), e >> (L + ml), L, ml, None, 8)
        assert got == mir, k
        # the prefix-blocked and the segmented walk: the same range, other operation orders
        for kind in ("sparse", "seg"):
            assert rel(sup.partial(a, s, e, kernel=kind), got) < 1e-9, (k, kind)


@pytest.mark.parametrize("n", [63, 64])
def test_sparse_skip_max_order(sup, orc, n):
    a = sup.skip_order(_mat(n, 0.15, 200 + n, ints=True))[0]
    for k in KS:
        s, e = k * Q, (k + 1) * Q
        L, ml = _layout(sup, n, s, e)
        for kind, fn in (("sparse", orc.ref_sparse_partial), ("skip", orc.ref_skip_partial)):
            got = sup.partial(a, s, e, kernel=kind)
            want = fn(a, s, e, 8)
            assert abs(got - want) <= 1e-9 * max(abs(want), 1e-300) or got == want, (k, kind, got, want)
            mir, _ = orc.engine_range(a, kind, s >> (L + ml), e >> (L + ml), L, ml, None, 8)
            assert got == mir, (k, kind)


def test_order_limit(sup):
    for call in (lambda a: sup.perman(a), lambda a: sup.partial(a, 0, 64)):
        with pytest.raises((ValueError, sup.SupError)):
            call(np.ones((65, 65)))
