"""GPU parity of the segmented walk (pattern-specialised kernel compiled with
hiprtc, superman_amd/csrc/jit.cpp) through the C ABI:

* bit-exact against the oracle's mirror of the segmented enumeration
  (oracle/oracle.c kind 3) and against the host-thread walk (sup_perman_cpu);
* within fp64 tolerance of the reference's goldens;
* schedulers (-p5/-p6, RCCL combine, CPU worker) and shards bit-identical;
* at the bench size (n = 40) against the prefix-blocked walk (1e-9) and
  through exact properties (power-of-two row scaling, shard additivity).
"""
import numpy as np
import pytest

from conftest import fixture_path, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu(sup):
    if sup.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")


def _synth(sup, golden, min_n=10):
    names = sorted({k.split("|")[0] for k in golden if k.startswith("synth/")})
    out = []
    for nm in names:
        a = sup.read_matrix(fixture_path(nm))[0]
        if a.shape[0] >= min_n:
            out.append((nm, a))
    return out


def test_seg_bitexact_vs_mirror_and_cpu(sup, orc, golden):
    cases = _synth(sup, golden)
    assert len(cases) >= 10
    for name, a in cases:
        got, st = sup.perman(a, algo=4, kernel="seg", return_stats=True)
        assert st["walk_kind"] == 3, name
        want = orc.engine_perman_as(sup, a, "seg", threads=4)
        assert got == want, (name, got, want)
        assert sup.perman_cpu(a, "seg", threads=4) == got, name
        q = golden.get(f"{name}|dense_q|r0|b0|t4")
        f = golden[f"{name}|dense|r0|b0|t4"]
        ref = q if q is not None else f
        assert abs(got - ref) <= max(4 * abs(f - ref), 1e-13 * abs(ref), 1e-12), (name, got, f, q)


@pytest.mark.parametrize("name", ["double__30_0.50_0", "double__30_0.20_0", "int__30_0.50_0"])
def test_seg_corpus_n30(sup, orc, golden, name):
    a, _, _ = sup.read_matrix(fixture_path(name))
    got = sup.perman(a, algo=4, kernel="seg")
    assert got == orc.engine_perman_as(sup, a, "seg", threads=16)
    q = golden.get(f"{name}|dense_q|r0|b0|t8")
    f = golden[f"{name}|dense|r0|b0|t8"]
    assert rel(got, q if q is not None else f) < 1e-8
    if q is not None:
        assert abs(got - q) <= max(2 * abs(f - q), 1e-14 * abs(q))


def test_seg_sparse_orders(sup, orc):
    for name in ("double__30_0.20_0", "int__30_0.20_0"):
        a, _, _ = sup.read_matrix(fixture_path(name))
        for b in (sup.sort_order(a)[0], sup.skip_order(a)[0]):
            got = sup.perman(b, algo=4, sparse=True, kernel="seg")
            assert got == orc.engine_perman_as(sup, b, "seg", threads=16)
            assert rel(got, sup.perman(b, algo=4, sparse=True, jit=-1)) < 1e-10


def test_seg_schedulers_and_shards(sup):
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    r4 = sup.perman(a, 4, kernel="seg")
    assert sup.perman(a, 5, gpu_num=1, kernel="seg") == r4
    assert sup.perman(a, 6, gpu_num=1, chunk_log2=3, kernel="seg") == r4
    assert sup.perman(a, 6, gpu_num=1, use_rccl=2, chunk_log2=2, kernel="seg") == r4
    # hybrid CPU worker: host-thread items are bit-identical to the kernel's
    assert sup.perman(a, 6, gpu_num=1, cpu=True, threads=4, chunk_log2=4, kernel="seg") == r4
    # jit=1: the dense request takes the segmented walk when its cost model wins
    info = sup.plan_info(a, "dense", jit=1)
    if info["kind"] == "seg":
        assert sup.perman(a, 4, jit=1) == r4
        full = sup.perman_shard(a, 0, 1, jit=1)
        parts = [sup.perman_shard(a, r, 4, jit=1) for r in range(4)]
        assert (parts[0] + parts[1]) + (parts[2] + parts[3]) == full
        assert -2 * full == r4


def test_seg_known_answers(sup):
    import math
    for n in (10, 12, 16, 20):
        assert sup.perman(np.ones((n, n)), algo=4, kernel="seg") == pytest.approx(math.factorial(n), rel=1e-12)
    p = np.eye(22)[np.random.default_rng(2).permutation(22)]
    assert sup.perman(p, algo=4, kernel="seg") == 1.0
    z = np.random.default_rng(3).random((18, 18))
    z[2, :] = 0
    assert sup.perman(z, algo=4, kernel="seg") == 0.0
    with pytest.raises(sup.SupError):
        sup.perman(np.ones((9, 9)), algo=4, kernel="seg")  # needs >= 3 walk bits


def test_seg_n40_bench_matrix(sup):
    a, _, _ = sup.read_matrix(fixture_path("double__40_0.50_0"))
    r_seg, st = sup.perman(a, algo=4, jit=1, return_stats=True)
    assert st["walk_kind"] == 3
    r_blk = sup.perman(a, algo=4, jit=-1)
    assert rel(r_seg, r_blk) < 1e-9
    b = a.copy()
    b[3] *= 2.0
    b[20] *= 0.25
    assert sup.perman(b, algo=4, kernel="seg") == r_seg * 0.5  # exact under power-of-two row scaling
    # the bench's shards (strong scaling at 2/4/8 ranks) pair up to the full sum bit for bit
    full = sup.perman_shard(a, 0, 1, jit=1)
    for world in (2, 8):
        parts = [sup.perman_shard(a, r, world, jit=1) for r in range(world)]
        while len(parts) > 1:
            parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
        assert parts[0] == full
    assert -2 * full == r_seg


@pytest.mark.parametrize("cc", [0, 1, 2, 3, 4])
def test_seg_cached_bits_bitexact(sup, orc, monkeypatch, cc):
    """Each cached-walk-bit count (SUP_JIT_CC forces it) on the GPU: bit-exact
    against the oracle's per-state mirror and the host twin."""
    monkeypatch.setenv("SUP_JIT_CC", str(cc))
    rng = np.random.default_rng(40 + cc)
    for n, d in ((24, 0.5), (26, 0.3)):
        a = np.where(rng.random((n, n)) < d, rng.random((n, n)) * 5, 0.0)
        a[np.arange(n), rng.permutation(n)] = 1.0
        assert sup.plan_info(a, "seg")["cached"] == cc
        got = sup.perman(a, algo=4, kernel="seg")
        assert got == orc.engine_perman_as(sup, a, "seg", threads=16), (n, d)
        assert got == sup.perman_cpu(a, "seg", threads=16), (n, d)


def test_seg_n40_d02_companion(sup):
    """The bench's density-0.2 companion (double/40_0.20_0): segmented walk vs
    the prefix-blocked walk, and exact under power-of-two row scaling."""
    a, _, _ = sup.read_matrix(fixture_path("double__40_0.20_0"))
    r_seg, st = sup.perman(a, algo=4, jit=1, return_stats=True)
    assert st["walk_kind"] == 3
    assert rel(r_seg, sup.perman(a, algo=4, jit=-1)) < 1e-9
    b = a.copy()
    b[7] *= 4.0
    assert sup.perman(b, algo=4, jit=1) == r_seg * 4.0
    # cheap steps: the plan lengthens the wave-chunks (engine.cpp make_seg_plan);
    # the shards of that layout still pair up to the full sum bit for bit
    assert sup.plan_info(a, "dense", jit=1)["m"] > sup.layout(40)[1]
    full = sup.perman_shard(a, 0, 1, jit=1)
    parts = [sup.perman_shard(a, r, 8, jit=1) for r in range(8)]
    while len(parts) > 1:
        parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
    assert parts[0] == full and -2 * full == r_seg


def test_seg_config3_long_chunks(sup, golden):
    """Config 3 (double/36_0.20_0, SortOrder, SpaRyser request): the segmented
    walk on lengthened wave-chunks against the reference's golden, and
    bit-identical to the same walk length asked for explicitly (walk_log2)."""
    a = sup.sort_order(sup.read_matrix(fixture_path("double__36_0.20_0"))[0])[0]
    info = sup.plan_info(a, "sparse", jit=1)
    assert info["kind"] == "seg" and info["m"] > sup.layout(36)[1]
    got = sup.perman(a, algo=4, sparse=True, jit=1)
    assert rel(got, golden["double__36_0.20_0|sparse|r1|b0|t8"]) < 1e-9
    assert sup.perman(a, algo=4, sparse=True, jit=1, walk_log2=info["m"]) == got


@pytest.mark.parametrize("n,d,seed", [(24, 0.15, 4), (24, 0.15, 3)])
def test_seg_chunk_skip_gpu(sup, orc, n, d, seed):
    """Wave-chunks whose walk-untouched rows are exactly zero in every lane are
    skipped by the generated kernel: GPU == host twin (same skip) == oracle
    mirror (walks them) bit for bit, and the exact permanent."""
    from conftest import seg_skip_fraction
    from test_seg import _skip_case
    a = _skip_case(sup, n, d, seed)
    frac = seg_skip_fraction(sup, a, "seg")
    assert frac >= 0.25
    got, st = sup.perman(a, algo=4, kernel="seg", return_stats=True)
    assert st["walk_kind"] == 3
    # the kernel reports the states it walked: exactly the chunks not skipped
    assert st["visited_steps"] == round((1.0 - frac) * 2 ** (n - 1))
    assert got == sup.perman_cpu(a, "seg", threads=8) == orc.engine_perman_as(sup, a, "seg", threads=8)
    assert rel(got, float(orc.exact_perman_crt(a))) < 1e-12


def test_seg_shared_steps_and_lane_fold_gpu(sup, orc):
    """The n = 28 case of test_seg.py (shared steps, two-level lane sum) on the
    GPU: == host twin == oracle mirror bit for bit."""
    rng = np.random.default_rng(28)
    n = 28
    mask = rng.random((n, n)) < 0.15
    mask[np.arange(n), rng.permutation(n)] = True
    a = np.where(mask, rng.random((n, n)) * 3, 0).astype(np.float64)
    a = sup.sort_order(a)[0]
    got, st = sup.perman(a, algo=4, kernel="seg", return_stats=True)
    assert st["walk_kind"] == 3
    assert got == sup.perman_cpu(a, "seg", threads=8) == orc.engine_perman_as(sup, a, "seg", threads=8)


@pytest.mark.parametrize("b", [6, 7, 8])
def test_seg_pair_bits_bitexact_gpu(sup, orc, monkeypatch, b):
    """Specialised pair-bit counts above the old fixed 5 (the plan now picks
    5-8 by op count; SUP_JIT_B forces one): n = 30 (10 walk bits, so a shared
    step remains): GPU == host twin == oracle mirror bit for bit."""
    monkeypatch.setenv("SUP_JIT_B", str(b))
    rng = np.random.default_rng(300 + b)
    n = 30
    a = np.where(rng.random((n, n)) < 0.3, rng.random((n, n)) * 5, 0.0)
    a[np.arange(n), rng.permutation(n)] = 1.0
    info = sup.plan_info(a, "seg")
    assert info["pair_bits"] == b and info["m"] - 1 > b
    got = sup.perman(a, algo=4, kernel="seg")
    assert got == orc.engine_perman_as(sup, a, "seg", threads=16)
    assert got == sup.perman_cpu(a, "seg", threads=16)


def test_seg_storage_plan_invariance_gpu(sup, orc, monkeypatch):
    """The generated kernel at storage budgets 0 (every copy and node formed on
    demand inside its consumer), the default and 1000 (everything live): the
    same bits, equal to the oracle mirror, at n = 26 and n = 30."""
    rng = np.random.default_rng(77)
    for n, d in ((26, 0.5), (30, 0.3)):
        a = np.where(rng.random((n, n)) < d, rng.random((n, n)) * 5, 0.0)
        a[np.arange(n), rng.permutation(n)] = 1.0
        want = orc.engine_perman_as(sup, a, "seg", threads=16)
        for budget in (0, 1000):
            monkeypatch.setenv("SUP_JIT_STORAGE", str(budget))
            assert sup.perman(a, algo=4, kernel="seg") == want, (n, budget)
        monkeypatch.delenv("SUP_JIT_STORAGE")
        assert sup.perman(a, algo=4, kernel="seg") == want, n


_SCHED_KNOBS = (("SUP_JIT_ACCFLOAT", ("0", "1")), ("SUP_JIT_KP", ("1", "2", "4")),
                ("SUP_JIT_SCHED", ("max-ilp",)))


def test_seg_codegen_schedule_invariance_gpu(sup, orc, monkeypatch):
    """Scheduling-only code generation choices keep every bit of a given plan:
    accumulate chains floated into the next region or not (SUP_JIT_ACCFLOAT),
    step regions of 1, 2 or 4 SGPR pieces (SUP_JIT_KP), LLVM's max-ilp machine
    scheduler (SUP_JIT_SCHED).

    A knob can still change the plan itself: a short walk's 4-cached-bit
    kernel is compiled and re-planned with 3 cached bits when its walk loop
    touches scratch (jit.cpp build_seg), and whether it spills depends on the
    code the knob makes.  Round 4's red run (r4u: max-ilp with KP = 1 under
    torch's hiprtc) was that: the cc = 4 kernel came out clean, the plan walked
    cc = 4 with another walk order, and the test compared it with the mirror of
    the default knobs' cc = 3 plan.  So (1) with the plan pinned (SUP_JIT_CC = 3:
    no compiler check, the same walk order, trees and tables for every knob)
    every setting must give the same plan and the same bits; (2) unpinned, every
    setting must equal the mirror of the plan it actually walked."""
    rng = np.random.default_rng(91)
    n = 28
    a = np.where(rng.random((n, n)) < 0.5, rng.random((n, n)) * 5, 0.0)
    a[np.arange(n), rng.permutation(n)] = 1.0
    strip = lambda info: (info["kind"], info["colmap"].tolist(), info["L"], info["m"], info["cached"],  # noqa: E731
                          info["pair_bits"])
    # (1) pinned plan: scheduling knobs cannot move a bit
    monkeypatch.setenv("SUP_JIT_CC", "3")
    plan0 = strip(sup.plan_info(a, "seg"))
    want = orc.engine_perman_as(sup, a, "seg", threads=16)
    assert sup.perman(a, algo=4, kernel="seg") == want
    for knob, vals in _SCHED_KNOBS:
        for v in vals:
            monkeypatch.setenv(knob, v)
            assert strip(sup.plan_info(a, "seg")) == plan0, (knob, v)
            assert sup.perman(a, algo=4, kernel="seg") == want, (knob, v)
        monkeypatch.delenv(knob)
    monkeypatch.delenv("SUP_JIT_CC")
    # (2) unpinned: each setting against the mirror of its own plan
    for knob, vals in _SCHED_KNOBS:
        for v in vals:
            monkeypatch.setenv(knob, v)
            want = orc.engine_perman_as(sup, a, "seg", threads=16)
            assert sup.perman(a, algo=4, kernel="seg") == want, (knob, v)
        monkeypatch.delenv(knob)


def test_seg_config5_shards_balanced_gpu(sup):
    """Config 5 (n = 44 d = 0.15 int, -p8 -s -r2): with the skip-neutral high
    columns on the top chunk bits, the 8 contiguous shards of the engine's walk
    visit the same number of states (sup_stats.visited_steps), and they fold to
    the one-GPU sum bit for bit."""
    a = sup.skip_order(sup.read_matrix(fixture_path("synth44_0.15_int"))[0])[0]
    full, st = sup.perman_shard(a, 0, 1, kernel="skip", jit=1, return_stats=True)
    assert st["walk_kind"] == 3 and 0 < st["visited_steps"] < st["gray_steps"] // 2
    parts, vis = [], []
    for r in range(8):
        p, s = sup.perman_shard(a, r, 8, kernel="skip", jit=1, return_stats=True)
        parts.append(p)
        vis.append(s["visited_steps"])
    assert max(vis) == min(vis) and sum(vis) == st["visited_steps"]
    while len(parts) > 1:
        parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
    assert parts[0] == full


def test_cli_auto_mode_same_bits_cold_and_warm(tmp_path):
    """`perman -f double/40_0.50_0 -g -p4` (auto mode) with an empty cache,
    then a --jit 1 run (records the segmented plan's choices), then the first
    command again: the auto-mode runs print the same bits (the first decision
    is recorded)."""
    import os
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "superman_amd", "bin", "perman")
    env = dict(os.environ, SUP_JIT_CACHE_DIR=str(tmp_path))

    def run(*extra):
        out = subprocess.run([exe, "-f", fixture_path("double__40_0.50_0"), "-g", "-p4", *extra], capture_output=True,
                             text=True, timeout=300, env=env, check=True).stdout
        return [ln for ln in out.splitlines() if ln.startswith("Permanent:")][0]

    cold = run()
    jit1 = run("--jit", "1")
    warm = run()
    assert cold == warm
    assert rel(float(jit1.split()[1]), float(cold.split()[1])) < 1e-9


def test_cli_fresh_host_default_takes_benchmarked_walk(tmp_path):
    """the drop-in command `perman -f double/40_0.50_0 -g
    -p4` on a fresh host (empty plan cache, empty comgr cache, no recorded host
    speed) takes the segmented walk — the benchmarked kernel — and prints the
    --jit 1 bits; the warm run follows the recorded decision."""
    import os
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "superman_amd", "bin", "perman")

    def run(cache, *extra):
        env = dict(os.environ, SUP_JIT_CACHE_DIR=str(cache / "plans"), AMD_COMGR_CACHE_DIR=str(cache / "comgr"))
        env.pop("SUP_JIT_COLD_RATIO", None)
        out = subprocess.run([exe, "-f", fixture_path("double__40_0.50_0"), "-g", "-p4", "-v", *extra],
                             capture_output=True, text=True, timeout=300, env=env, check=True).stdout
        perm = [ln for ln in out.splitlines() if ln.startswith("Permanent:")][0]
        kind = [ln for ln in out.splitlines() if ln.startswith("Stats:")][0].split("walk_kind")[1].split()[0]
        return perm, kind

    cold, kind = run(tmp_path / "a")
    assert kind == "3", kind  # the segmented walk
    jit1, kind1 = run(tmp_path / "b", "--jit", "1")
    assert kind1 == "3" and jit1 == cold
    assert run(tmp_path / "a") == (cold, "3")


@pytest.mark.parametrize("n,d,seed", [(28, 0.9, 1), (30, 0.7, 1)])
def test_seg_shared_streams_bitexact_gpu(sup, orc, monkeypatch, n, d, seed):
    """Near-dense patterns (d = 0.7, 0.9) whose top specialised step and shared
    step re-form the same copies: one class reads the other's constant stream
    (jit.cpp share_streams, round 4).  Storage only: GPU == host twin ==
    oracle mirror bit for bit, and the same bits with sharing disabled."""
    rng = np.random.default_rng(seed)  # patterns where sharing applies (SUP_JIT_VERBOSE shows it)
    a = np.where(rng.random((n, n)) < d, rng.random((n, n)) * 5, 0.0)
    a[np.arange(n), rng.permutation(n)] = 1.0 + rng.random(n)
    got = sup.perman(a, algo=4, kernel="seg")
    assert got == orc.engine_perman_as(sup, a, "seg", threads=16)
    assert got == sup.perman_cpu(a, "seg", threads=16)
    monkeypatch.setenv("SUP_JIT_NOSHARE", "1")
    assert sup.perman(a, algo=4, kernel="seg") == got
