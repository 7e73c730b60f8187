"""GPU parity: the gfx950 kernels, called through the C ABI, against the oracle.

* bit-exact against the oracle's mirror of the engine schedule (same fp64
  operations in the same order) — dense, SpaRyser, SkipPer;
* within fp64 tolerance of the reference's own results (golden.json) and of
  the reference algorithm restated in oracle/ (orc_ref_*);
* chunk partials against the reference chunk helpers' semantics
  (gpu_exact_dense.cu:6-69 cpu_perman64 over [start, end));
* at full benchmark size (n = 40), size-independent properties: bitwise row
  scaling by powers of two, chunk-partial additivity, permutation invariance.
"""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import fixture_path, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu(sup):
    if sup.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")


def _partial_layout(sup, n, s, e):
    """Layout sup_partial uses for [s, e): the default one, with the walk
    shortened until a wave-chunk divides both ends (capi.cpp sup_partial)."""
    L, m, _ = sup.layout(n)
    space = 1 << (n - 1)
    al = min((n - 1) if v in (0, space) else (v & -v).bit_length() - 1 for v in (s, e))
    return L, min(m, al - L)


def _synth(sup, golden):
    names = sorted({k.split("|")[0] for k in golden if k.startswith("synth/")})
    return [(nm, sup.read_matrix(fixture_path(nm))[0]) for nm in names]


KINDS = [("dense", 4, False), ("sparse", 4, True), ("skip", 7, True)]


@pytest.mark.parametrize("kind,algo,sparse", KINDS)
def test_bitexact_vs_engine_mirror(sup, orc, golden, kind, algo, sparse):
    for name, a in _synth(sup, golden):
        if kind == "skip":
            a = sup.skip_order(a)[0]
        got, st = sup.perman(a, algo=algo, sparse=sparse, return_stats=True)
        want = orc.engine_perman_as(sup, a, kind, threads=4)
        assert got == want, (name, kind, got, want)
        assert st["devices_used"] == 1 and st["kernel_ms"] > 0.0


@pytest.mark.parametrize("kind,algo,sparse", KINDS)
def test_matches_reference_goldens(sup, golden, kind, algo, sparse):
    for name, a in _synth(sup, golden):
        q = golden.get(f"{name}|dense_q|r0|b0|t4")
        f = golden[f"{name}|dense|r0|b0|t4"]
        b = sup.skip_order(a)[0] if kind == "skip" else a
        got = sup.perman(b, algo=algo, sparse=sparse)
        ref = q if q is not None else f
        # as close to the quad golden as the reference's own fp64 result (or 1e-13)
        assert abs(got - ref) <= max(4 * abs(f - ref), 1e-13 * abs(ref), 1e-12), (name, got, f, q)


def test_known_answers(sup):
    # J_n = all ones: perm = n!.  Ryser cancels heavily on J_n (x entries are
    # +-1/2 sums, terms up to (n/2)^n), so fp64 keeps ~12 digits at n = 24.
    for n in (1, 2, 3, 7, 8, 12, 20, 24):
        tol = 1e-13 if n <= 12 else 1e-11
        for algo, sparse in ((4, False), (4, True), (7, True)):
            assert sup.perman(np.ones((n, n)), algo=algo, sparse=sparse) == pytest.approx(math.factorial(n),
                                                                                          rel=tol)
    p = np.eye(22)[np.random.default_rng(2).permutation(22)]
    assert sup.perman(p) == 1.0
    assert sup.perman(p, algo=7, sparse=True) == 1.0
    # a zero column: perm = 0; the terms it pairs up cancel only up to fp64
    # rounding of the running sum, so compare against the term scale
    z = np.random.default_rng(3).random((18, 18))
    z[:, 5] = 0
    scale = float(np.prod(z.sum(1)))
    for algo, sparse in ((4, False), (4, True), (7, True)):
        assert abs(sup.perman(z, algo=algo, sparse=sparse)) <= 1e-13 * scale
    z[2, :] = 0  # a zero row: every x_2 term is exactly 0
    for algo, sparse in ((4, False), (4, True), (7, True)):
        assert sup.perman(z, algo=algo, sparse=sparse) == 0.0


@pytest.mark.parametrize("name", ["int__30_0.50_0", "double__30_0.50_0", "float__30_0.50_0",
                                  "double__30_0.20_0", "int__30_0.20_0"])
def test_corpus_n30(sup, orc, golden, name):
    a, typ, _ = sup.read_matrix(fixture_path(name))
    got = sup.perman(a, algo=4)
    assert got == orc.engine_perman_as(sup, a, "dense", threads=16)
    q = golden.get(f"{name}|dense_q|r0|b0|t8")
    f = golden[f"{name}|dense|r0|b0|t8"]
    assert rel(got, q if q is not None else f) < 1e-8
    if q is not None:
        assert abs(got - q) <= max(2 * abs(f - q), 1e-14 * abs(q))


def test_sparse_orders_corpus(sup, orc, golden):
    for name in ("double__30_0.20_0", "int__30_0.20_0"):
        a, _, _ = sup.read_matrix(fixture_path(name))
        s1 = sup.sort_order(a)[0]
        s2 = sup.skip_order(a)[0]
        g1 = sup.perman(s1, algo=4, sparse=True)
        g2 = sup.perman(s2, algo=7, sparse=True)
        assert g1 == orc.engine_perman_as(sup, s1, "sparse", threads=16)
        assert g2 == orc.engine_perman_as(sup, s2, "skip", threads=16)
        ref = golden.get(f"{name}|dense_q|r0|b0|t8", golden[f"{name}|sparse|r1|b0|t8"])
        assert rel(g1, ref) < 1e-8 and rel(g2, ref) < 1e-8


def test_partials_match_reference_chunk_helper(sup, orc):
    # cpu_perman64 (gpu_exact_dense.cu:6-69) returns sum_{i in [s,e)} (-1)^i prod x(gray(i))
    a, _, _ = sup.read_matrix(fixture_path("synth/22_0.50_double"))
    n = 22
    end = 1 << (n - 1)
    for s, e in ((1 << 12, 1 << 14), (1 << 18, (1 << 18) + (1 << 16)), (1 << 20, end)):
        got = sup.partial(a, s, e)
        want = orc.ref_dense_partial(a, s, e, 4)
        assert rel(got, want) < 1e-10, (s, e, got, want)
        L, ml = _partial_layout(sup, n, s, e)
        mir, _ = orc.engine_range(a, "dense", s >> (L + ml), e >> (L + ml), L, ml, None, 4)
        assert got == mir
    # index 0 carries the p0 term
    x0, p0 = orc.nw_start(a)
    g0 = sup.partial(a, 0, 64)
    assert rel(g0, p0 + orc.ref_dense_partial(a, 1, 64, 1)) < 1e-12
    with pytest.raises(sup.SupError):
        sup.partial(a, 3, 64)


@pytest.mark.parametrize("kind", ["sparse", "skip"])
def test_sparse_partials(sup, orc, kind):
    a, _, _ = sup.read_matrix(fixture_path("synth/22_0.20_int"))
    a = sup.skip_order(a)[0]
    s, e = 1 << 14, 1 << 17
    got = sup.partial(a, s, e, kernel=kind)
    fn = orc.ref_sparse_partial if kind == "sparse" else orc.ref_skip_partial
    assert rel(got, fn(a, s, e, 4)) < 1e-9


def test_schedulers_agree_bitwise(sup):
    # -p4 / -p5 / -p6 and the reference-named wrappers give identical bits
    # (fixed pairwise reduction over aligned power-of-two chunk ranges)
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    r4 = sup.perman(a, 4)
    assert sup.perman(a, 5, gpu_num=1) == r4
    assert sup.perman(a, 6, gpu_num=1) == r4
    assert sup.perman(a, 6, gpu_num=1, chunk_log2=3) == r4
    assert sup.gpu_perman64_xshared_coalescing_mshared(a) == r4
    for algo in (0, 1, 2, 3):
        assert sup.perman(a, algo) == r4


def test_rccl_combine_single_device(sup):
    # in-process RCCL path (ncclCommInitAll + ncclAllReduce) of -p5/-p6 -R,
    # exercised on one device.  The all-reduced buffer has one slot per device
    # (-p5) or per queue item (-p6), each with a single nonzero addend, so the
    # merged vector is folded by the host's pairwise tree: bit-identical.
    a, _, _ = sup.read_matrix(fixture_path("synth/22_0.50_double"))
    r4 = sup.perman(a, 4)
    assert sup.perman(a, 5, gpu_num=1, use_rccl=2) == r4
    assert sup.perman(a, 6, gpu_num=1, use_rccl=2) == r4
    assert sup.perman(a, 6, gpu_num=1, use_rccl=2, chunk_log2=2) == r4
    b = sup.skip_order(a)[0]
    assert sup.perman(b, 8, sparse=True, gpu_num=1, use_rccl=2) == sup.perman(b, 7, sparse=True)


def test_shards_sum_to_full(sup):
    # sup_perman_shard: the bench's per-rank unit; 2^k shards are subtrees of
    # the fixed reduction, so pairing them reproduces the single-launch bits
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    full = sup.perman_shard(a, 0, 1)
    for world in (2, 4, 8):
        parts = [sup.perman_shard(a, r, world) for r in range(world)]
        while len(parts) > 1:
            parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
        assert parts[0] == full
    assert -2 * full == sup.perman(a, 4)  # n even: perm = -2 * sum


def test_hybrid_cpu_worker(sup):
    a, _, _ = sup.read_matrix(fixture_path("synth/22_0.50_double"))
    r4 = sup.perman(a, 4)
    r, st = sup.perman(a, 6, gpu_num=1, cpu=True, threads=4, chunk_log2=2, return_stats=True)
    assert r == r4  # CPU worker items are bit-identical to GPU items


def test_int_float_double_storage(sup):
    rng = np.random.default_rng(11)
    ai = rng.integers(0, 6, (21, 21)).astype(np.int32)
    assert sup.perman(ai) == sup.perman(ai.astype(np.float64)) == sup.perman(ai.astype(np.float32))


def test_n40_properties(sup):
    # full benchmark size: properties that hold independent of a CPU oracle
    a, _, _ = sup.read_matrix(fixture_path("double__40_0.50_0"))
    r = sup.perman(a)
    assert np.isfinite(r) and r > 0  # permanent of a nonnegative matrix
    b = a.copy()
    b[7] *= 2.0
    b[31] *= 0.5
    b[0] *= 4.0
    assert sup.perman(b) == r * 4.0  # power-of-two row scaling is exact
    # chunk partials add up (each aligned range is a subtree of the fixed reduction)
    n = 40
    q = 1 << (n - 3)
    parts = [sup.partial(a, k * q, (k + 1) * q) for k in range(4)]
    tot = ((parts[0] + parts[1]) + (parts[2] + parts[3]))
    assert sup.partial(a, 0, 4 * q) == tot
    # column permutation invariance (rounding-level)
    perm = np.random.default_rng(5).permutation(n)
    assert rel(sup.perman(a[:, perm]), r) < 1e-9


@pytest.mark.parametrize("typ", ["int", "double"])
def test_config5_n44(sup, orc, typ):
    # BASELINE config 5 (n = 44, d = 0.15, synthetic: tests/fixtures/gen_config5.py).
    # Aligned 2^23-step ranges against the reference chunk helpers restated
    # (cpu_perman64_sparse / _skipper, gpu_exact_sparse.cu:6-191) and bit-exact
    # against the engine mirror; the full 2^43 walk through properties.
    a, _, _ = sup.read_matrix(fixture_path(f"synth44_0.15_{typ}"))
    b = sup.skip_order(a)[0]
    n, q = 44, 1 << 23
    for k in (1, 777, 1 << 19, (1 << 20) - 1):
        s, e = k * q, (k + 1) * q
        for kind, fn in (("sparse", orc.ref_sparse_partial), ("skip", orc.ref_skip_partial)):
            got = sup.partial(b, s, e, kernel=kind)
            assert rel(got, fn(b, s, e, 8)) < 1e-9, (kind, k)
            L, ml = _partial_layout(sup, n, s, e)
            mir, _ = orc.engine_range(b, kind, s >> (L + ml), e >> (L + ml), L, ml, None, 8)
            assert got == mir, (kind, k)
    r_sp = sup.perman(b, algo=4, sparse=True)
    r_sk, st = sup.perman(b, algo=8, sparse=True, return_stats=True, jit=-1)  # the SkipPer kernel itself
    assert st["walk_kind"] == 2
    assert np.isfinite(r_sp) and r_sp > 0 and rel(r_sk, r_sp) < 1e-9
    if typ == "int":
        assert st["visited_steps"] < 0.5 * 2.0 ** 43  # SkipPer jumps over exact-zero rows
    # default SkipPer request: the engine measures SkipPer's visited fraction on a
    # sample of its chunks (integer input; non-integer input has no exact zeros)
    # and runs the segmented walk, which is cheaper here either way; same sum
    r_def, st_def = sup.perman(b, algo=8, sparse=True, return_stats=True)
    assert st_def["walk_kind"] == 3
    assert rel(r_def, r_sp) < 1e-9
    c = b.astype(np.float64)
    c[5] *= 2.0
    assert sup.perman(c, algo=4, sparse=True) == 2.0 * r_sp  # power-of-two row scaling is exact


def test_cli_gpu(sup, orc):
    exe = sup._lib.PERMAN_BIN
    f = fixture_path("double__30_0.50_0")
    r = subprocess.run([exe, "-f", f, "-g", "-p4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("Result: gpu_perman64_xshared_coalescing_mshared ")
    val = float(r.stdout.splitlines()[1].split()[1])
    a, _, _ = sup.read_matrix(f)
    assert val == sup.perman(a)
    r = subprocess.run([exe, "-f", fixture_path("int__30_0.20_0"), "-s", "-r2", "-p7"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "skipper" in r.stdout
    r = subprocess.run([exe, "-f", f, "-g", "-p6", "-d1", "-v"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ChunkID" in r.stdout


# (pores_1_r.mtx is left out: entries of both signs up to 2.5e7 cancel so
# badly in fp64 Ryser that neither the reference nor this engine keeps a
# correct digit — 9.9e139 vs 5.3e138)
MTX_DIRECT = ["Tina_DisCog_p.mtx", "Trefethen_20_s.mtx", "can_24_ps.mtx", "mycielskian5_ps.mtx", "ex5_rs.mtx",
              "GD02_a_p.mtx", "Ragusa16.mtx", "Ragusa18.mtx"]


@pytest.mark.parametrize("name", MTX_DIRECT)
def test_mtx_direct_vs_reference(sup, golden, name):
    # MatrixMarket inputs (revised_perman/matrices) on the dense GPU path vs the
    # reference CPU (parallel_perman64<double>) on the reference reader's matrix
    a, _, _ = sup.read_matrix(fixture_path("mtx/" + name))
    want = golden[f"mtx/{name}|dense|r0|b0|t8"]
    got = sup.perman(a)
    if want == 0.0:
        assert abs(got) <= 1e-6 * max(1.0, float(np.prod(np.abs(a).sum(1))) ** 0.5)
    else:
        assert rel(got, want) < 1e-8, (name, got, want)


@pytest.mark.parametrize("algo,sparse,prep", [(4, False, 0), (4, True, 1), (7, True, 2), (6, False, 0)])
def test_reduced_gpu_vs_reference(sup, golden, algo, sparse, prep):
    # -o / -u with every leaf on the GPU vs the reference's reductions + CPU
    for name, min_n, thr in [("can_24_ps.mtx", 20, -1), ("can_24_ps.mtx", 20, 4), ("ibm32_p.mtx", 20, -1),
                             ("ibm32_p.mtx", 20, 4), ("mycielskian5_ps.mtx", 20, -1), ("Tina_DisCog_p.mtx", 30, -1)]:
        a, _, _ = sup.read_matrix(fixture_path("mtx/" + name))
        got, st = sup.perman_reduced(a, algo=algo, sparse=sparse, preprocessing=prep, compress=True,
                                     scale=thr if thr > 0 else None, min_n=min_n, return_stats=True)
        assert rel(got, golden[f"mtx/{name}|reduce|n{min_n}|u{thr}|t8"]) < 1e-10, (name, algo, prep)
        assert st["leaves"] == golden[f"mtx/{name}|leaves|n{min_n}|u{thr}"]["count"]


def test_chesapeake(sup):
    # n = 39 pattern matrix (elektrik_matrices/known_perman): directly on the
    # GPU; the reference's older SpaRyser runs report 1.31734973e13 (their
    # float-X results spread ~1e-5: sparyser/RealResults/chesapeake.mtx.a3s1.out)
    a, _, _ = sup.read_matrix(fixture_path("mtx/chesapeake.mtx"))
    r = sup.perman(a)
    assert r == pytest.approx(13173497329080.0, rel=2e-5)
    assert abs(r - round(r)) < 1e-3 * abs(r) ** 0.5  # an integer, up to fp64 rounding of the sum
    assert rel(sup.perman(a, algo=4, sparse=True), r) < 1e-12


def test_dense_lds_bitexact(sup, orc):
    """The north star's LDS-staged dense kernel (walk_lds.hip) does walk_dense's
    arithmetic with X in LDS: bit-identical results, full and partial."""
    rng = np.random.default_rng(17)
    for n in (3, 9, 16, 23, 30):
        a = rng.random((n, n)) * 5
        got, st = sup.perman(a, algo=4, kernel="dense_lds", return_stats=True)
        assert st["walk_kind"] == 4
        assert got == sup.perman(a, algo=4, kernel="dense_plain"), n
        assert got == orc.engine_perman_as(sup, a, "dense_lds", threads=16), n
    a, _, _ = sup.read_matrix(fixture_path("double__32_0.50_0"))
    assert sup.perman(a, algo=4, kernel="dense_lds") == sup.perman(a, algo=4, kernel="dense_plain")
    s, e = 1 << 24, 1 << 25
    assert sup.partial(a, s, e, kernel="dense_lds") == sup.partial(a, s, e, kernel="dense_plain")
