"""-o / -u leaves computed concurrently on the GPU (sup_perman_reduced): the
decomposition hands each leaf to one of SUP_LEAF_WORKERS host threads, each on
its own context lane (stream, buffers), and folds the combine afterwards in
the sequential order — so any worker count returns the bits of one leaf at a
time and of the callback path (sup_decompose with the engine's own leaf
permanent), and an error in any leaf surfaces."""
import os
from contextlib import contextmanager

import pytest

from conftest import fixture_path

pytestmark = pytest.mark.gpu


@contextmanager
def workers(k):
    old = os.environ.get("SUP_LEAF_WORKERS")
    os.environ["SUP_LEAF_WORKERS"] = str(k)
    try:
        yield
    finally:
        if old is None:
            del os.environ["SUP_LEAF_WORKERS"]
        else:
            os.environ["SUP_LEAF_WORKERS"] = old


@pytest.mark.parametrize("name,algo,sparse,prep,scale", [
    ("mtx/chesapeake.mtx", 4, False, 0, None),
    ("mtx/chesapeake.mtx", 4, True, 1, None),
    ("mtx/will57.mtx", 4, False, 0, None),
    ("mtx/can_24_ps.mtx", 4, False, 0, 4),
])
def test_concurrent_leaves_bitwise(sup, name, algo, sparse, prep, scale):
    a = sup.read_mtx(fixture_path(name))[0]
    kw = dict(algo=algo, sparse=sparse, preprocessing=prep, compress=True, scale=scale, min_n=20 if scale else 30)
    with workers(1):
        one, st1 = sup.perman_reduced(a, return_stats=True, **kw)
    for k in (2, 4, 8):
        with workers(k):
            got, st = sup.perman_reduced(a, return_stats=True, **kw)
        assert got == one, (name, k, got, one)
        assert st["leaves"] == st1["leaves"] and st["gray_steps"] == st1["gray_steps"]
    # the callback path: the same leaves, one at a time through sup_decompose
    if scale is None and prep == 0 and not sparse:
        via_cb = sup.decompose(a, lambda m: sup.perman(m, algo), compress=True)[0]
        assert via_cb == one


def test_concurrent_leaves_error_surfaces(sup):
    a = sup.read_mtx(fixture_path("mtx/will57.mtx"))[0]
    with workers(4):
        with pytest.raises(sup.SupError):
            sup.perman_reduced(a, algo=4, device_id=7)  # no such device: every leaf fails
        assert sup.perman_reduced(a, algo=4) == sup.perman_reduced(a, algo=4)  # and the engine is fine after


@contextmanager
def batch(k):
    old = os.environ.get("SUP_LEAF_BATCH")
    os.environ["SUP_LEAF_BATCH"] = str(k)
    try:
        yield
    finally:
        if old is None:
            del os.environ["SUP_LEAF_BATCH"]
        else:
            os.environ["SUP_LEAF_BATCH"] = old


@pytest.mark.parametrize("name,sparse,prep,scale", [
    ("mtx/chesapeake.mtx", False, 0, None),
    ("mtx/chesapeake.mtx", True, 1, None),
    ("mtx/will57.mtx", False, 0, None),
    ("mtx/can_24_ps.mtx", False, 0, 4),
    ("mtx/ibm32_p.mtx", False, 0, None),
])
def test_leaf_batches_bitwise(sup, name, sparse, prep, scale):
    """Several leaves of one order per launch (walk_sparse_batch /
    walk_dense_batch, run_range_batch; round 4): each leaf's chunk partials
    are those of its own launch and are folded by the same pairwise tree, so
    every batch size and worker count returns the one-leaf-at-a-time bits."""
    a = sup.read_mtx(fixture_path(name))[0]
    kw = dict(algo=4, sparse=sparse, preprocessing=prep, compress=True, scale=scale, min_n=20 if scale else 30)
    with batch(1), workers(1):
        one, st1 = sup.perman_reduced(a, return_stats=True, **kw)
    for b, k in ((4, 1), (16, 1), (32, 1), (16, 8), (3, 8)):
        with batch(b), workers(k):
            got, st = sup.perman_reduced(a, return_stats=True, **kw)
        assert got == one, (name, b, k, got, one)
        assert st["leaves"] == st1["leaves"] and st["gray_steps"] == st1["gray_steps"]
