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


def _dense_mat(n, d):
    """tools/probes/sweep_large_n.py's matrices: Bernoulli(d), U(0,5), a permutation diagonal."""
    rng = np.random.default_rng(1000 * n + int(round(100 * d)))
    a = np.where(rng.random((n, n)) < d, rng.random((n, n)) * 5, 0.0)
    a[np.arange(n), rng.permutation(n)] = 1.0 + rng.random(n)
    return a


@pytest.mark.parametrize("n,d", [(56, 0.5), (56, 0.9), (64, 0.5), (64, 0.9)])
def test_seg_large_dense(sup, orc, n, d):
    """Large dense n: the segmented walk plans and compiles at n = 56 and at
    the maximum order 64 (before
    round 4 hiprtc refused d = 0.9 patterns from n = 46 on: a region's pinned
    SGPR pieces exceeded the wave's SGPRs) and its walk loop has no scratch
    (the plan's compiler check).  (1) The planned kernel (searched walk order,
    budget ladder) on one wave-chunk of 2^25 Gray steps through the bench's
    entry point, bit-exact against the oracle's mirror of that plan (n = 56:
    a shard index is a C int, and n = 64 has 2^38 wave-chunks); (2) the
    reference-order range [k 2^25, (k+1) 2^25) through sup_partial, bit-exact
    against the mirror and within 1e-9 of the reference chunk helper
    cpu_perman64 restated (gpu_exact_dense.cu:6-69)."""
    wl = 19
    a = _dense_mat(n, d)
    info = sup.plan_info(a, "dense", jit=1, walk_log2=wl)
    assert info["kind"] == "seg" and info["m"] == wl
    assert info["est_ops_per_step"] < 0.95 * sup.plan_info(a, "dense", jit=-1)["est_ops_per_step"]
    r = 0x2A5A5A5
    if n - 1 - info["L"] - wl <= 30:  # one wave-chunk per shard (shard counts are C ints: n = 64 has 2^38 chunks)
        nshards = 1 << (n - 1 - info["L"] - wl)
        part, st = sup.perman_shard(a, r, nshards, kernel="dense", jit=1, walk_log2=wl, return_stats=True)
        assert st["walk_kind"] == 3 and st["gray_steps"] == 1 << (info["L"] + wl)
        assert (st["seg_cached_bits"], st["seg_pair_bits"]) == (info["cached"], info["pair_bits"])
        mir, _ = orc.engine_range(a, "seg", r, r + 1, info["L"], wl, info["colmap"], 16, info["cached"],
                                  info["pair_bits"])
        assert part == mir
    s = r << (info["L"] + wl)
    e = s + (1 << (info["L"] + wl))
    got, st2 = sup.partial(a, s, e, kernel="seg", return_stats=True)
    assert st2["walk_kind"] == 3
    L, ml = _layout(sup, n, s, e)
    mir2, _ = orc.engine_range(a, "seg", s >> (L + ml), e >> (L + ml), L, ml, None, 16, st2["seg_cached_bits"],
                               st2["seg_pair_bits"])
    assert got == mir2
    assert rel(got, orc.ref_dense_partial(a, s, e, 16)) < 1e-9
