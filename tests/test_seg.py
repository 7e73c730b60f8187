"""Segmented walk on the CPU (no GPU needed): the host-thread walk of the
pattern-specialised enumeration is bit-exact against the oracle's independent
mirror (oracle/oracle.c kind 3); the planner picks it only where its cost model
wins; and the generated HIP source compiles for gfx950 with hiprtc for shapes
at the edges (n = 10 and 64, a zero walk column, no rest rows)."""
import numpy as np
import pytest

import os

from conftest import ROOT, fixture_path, rel


def _rand(n, d, seed, ints=True):
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < d
    mask[np.arange(n), rng.permutation(n)] = True
    vals = rng.integers(1, 6, (n, n)) if ints else rng.random((n, n)) * 5
    return np.where(mask, vals, 0).astype(np.float64)


@pytest.mark.parametrize("n,d,seed", [(10, 0.5, 1), (12, 0.3, 2), (14, 0.6, 3), (16, 0.2, 4), (17, 1.0, 5)])
def test_cpu_seg_vs_mirror_and_exact(sup, orc, n, d, seed):
    a = _rand(n, d, seed)
    got = sup.perman_cpu(a, "seg", threads=4)
    assert got == orc.engine_perman_as(sup, a, "seg", threads=4)
    assert sup.plan_info(a, "seg")["cached"] in (0, 1, 2, 3, 4)
    exact = float(orc.exact_perman(a))
    assert abs(got - exact) <= 1e-12 * max(abs(exact), 1.0)


@pytest.mark.parametrize("cc", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("n,d,seed", [(13, 0.5, 11), (16, 0.35, 12)])
def test_cpu_seg_cached_bits(sup, orc, monkeypatch, cc, n, d, seed):
    """Every cached-bit count (walk bits held in every state, SUP_JIT_CC forces
    it): host twin == oracle mirror bit for bit, and == the exact permanent."""
    monkeypatch.setenv("SUP_JIT_CC", str(cc))
    a = _rand(n, d, seed, ints=False)
    assert sup.plan_info(a, "seg")["cached"] == cc
    got = sup.perman_cpu(a, "seg", threads=4)
    assert got == orc.engine_perman_as(sup, a, "seg", threads=4)
    assert rel(got, float(orc.exact_perman(a))) < 1e-12


def test_cpu_seg_corpus_vs_sparse(sup, orc):
    a, _, _ = sup.read_matrix(fixture_path("synth/22_0.20_int"))
    b = sup.skip_order(a)[0]
    got = sup.perman_cpu(b, "seg", threads=8)
    assert got == orc.engine_perman_as(sup, b, "seg", threads=8)
    assert rel(got, sup.perman_cpu(b, "sparse", threads=8)) < 1e-12


def test_planner_choice(sup, tmp_path, monkeypatch):
    monkeypatch.setenv("SUP_JIT_CACHE_DIR", str(tmp_path))  # cold: nothing recorded yet
    a, _, _ = sup.read_matrix(fixture_path("double__40_0.50_0"))
    assert sup.plan_info(a, "dense", jit=-1)["kind"] == "sparse"
    # auto, cold, on a slow host (predicted cold plan 8x a GPU box's ~1.6-1.9 s): the n = 40 walk
    # saves ~0.5 s per run, under the plan's cost over 4 runs; n = 44 saves seconds
    monkeypatch.setenv("SUP_JIT_COLD_RATIO", "8")
    assert sup.plan_info(a, "dense", jit=0)["kind"] == "sparse"
    assert sup.plan_info(a, "dense", jit=0, gpu_num=8)["kind"] == "sparse"
    assert sup.plan_info(a, "dense", jit=1)["kind"] == "seg"
    monkeypatch.delenv("SUP_JIT_COLD_RATIO")
    # the jit = 1 plan left its choices (and kernel) in the disk cache, but auto mode's first decision for
    # this pattern is recorded too (round 4, AutoRecord): `a` and another matrix of its zero pattern keep it
    assert any(p.name.startswith("plan_") for p in tmp_path.iterdir())
    assert sup.plan_info(a, "dense", jit=0)["kind"] == "sparse"
    assert sup.plan_info(0.5 * a, "dense", jit=0)["kind"] == "sparse"
    # warm, no auto decision yet: a pattern whose choices a jit = 1 plan recorded first — rebuilding costs
    # ~ms, so auto mode's bar is 0.1 s and it takes the segmented walk (and records that)
    t = np.ascontiguousarray(a.T)
    assert sup.plan_info(t, "dense", jit=1)["kind"] == "seg"
    t2 = 0.5 * t
    assert sup.plan_info(t2, "dense", jit=0)["kind"] == "seg"
    assert sup.plan_key(t2, "dense", jit=0) == sup.plan_key(t2, "dense", jit=1)
    c, _, _ = sup.read_matrix(fixture_path("double__32_0.50_0"))
    assert sup.plan_info(c, "dense", jit=0)["kind"] == "sparse"  # 2^31 steps: ms saved
    b, _, _ = sup.read_matrix(fixture_path("synth44_0.15_int"))
    b = sup.skip_order(b)[0]
    assert sup.plan_info(b, "sparse", jit=0)["kind"] == "seg"  # 2^43 steps: worth compiling
    assert sup.plan_info(b, "skip", jit=1)["kind"] == "skip"   # SkipPer is never replaced
    # all-nonzero matrix: every step touches every row; the paired step and the
    # cached walk bits (held in both states, their steps only accumulate) keep
    # it below the plain walk's 2n + 1 ops
    _, st = sup.perman_cpu(np.ones((12, 12)), "seg", threads=2, return_stats=True)
    assert 8 <= st["est_ops_per_step"] < 2 * 12
    assert sup.plan_info(np.ones((12, 12)), "seg")["cached"] >= 1


def test_auto_cold_bar_follows_recorded_plan_cost(sup, tmp_path, monkeypatch):
    """Auto mode starts a segmented plan when the walk time it can save over 4
    runs covers the predicted cold plan cost: a model of n and the host's plan
    threads (fitted on a GPU box, empty plan and comgr caches), times this
    host's speed as its last cold plan measured it (cost_<toolchain>.txt:
    measured / modelled).  With no record the model stands: the n = 40 bench
    matrix (~0.5 s saved per run, ~1.6-1.9 s predicted on 8-16 threads)
    specialises on a fresh host."""
    monkeypatch.setenv("SUP_JIT_CACHE_DIR", str(tmp_path))
    monkeypatch.setenv("OMP_NUM_THREADS", "8")
    monkeypatch.delenv("SUP_JIT_COLD_RATIO", raising=False)
    a, _, _ = sup.read_matrix(fixture_path("double__40_0.50_0"))
    a = 0.75 * a  # values no other test plans in this process (the in-process plan cache)
    assert sup.plan_info(a, "dense", jit=0)["kind"] == "seg"  # no record: the model's bar
    cost = list(tmp_path.glob("cost_*.txt"))  # the cold plan recorded this host's speed
    assert len(cost) == 1
    tag, ver, ratio = cost[0].read_text().split()
    assert (tag, ver) == ("supcost", "2") and 0 < float(ratio) < 1000
    # each check on a new zero pattern: auto mode's first decision for a pattern is recorded on
    # disk and kept (test_auto_decision_recorded_across_processes)
    cost[0].write_text("supcost 2 8.0\n")  # a slow host: ~15 s predicted, ~3.9 s bar
    assert sup.plan_info(np.ascontiguousarray(a[::-1]), "dense", jit=0)["kind"] == "sparse"
    cost[0].write_text("supcost 2 0.25\n")  # a fast host
    b = np.ascontiguousarray(a[:, ::-1])
    assert sup.plan_info(b, "dense", jit=0)["kind"] == "seg"
    cost[0].write_text("supcost 2 8.0\n")
    assert sup.plan_info(0.25 * b, "dense", jit=0)["kind"] == "seg"  # b's pattern: its first decision stands
    cost[0].write_text("supcost 1 5.0\n")  # a round-4 record (seconds, not a ratio): ignored, the model
    assert sup.plan_info(np.ascontiguousarray(a.T), "dense", jit=0)["kind"] == "seg"


def test_auto_decision_recorded_across_processes(tmp_path):
    """Auto mode (jit = 0) decides from the cache's state; it records its first
    decision per matrix and request, so the same command gives the same walk —
    and the same bits — cold and warm.  A cold run on a
    slow host (SUP_JIT_COLD_RATIO: the plan would cost more than 4 runs save)
    keeps the ahead-of-time walk; a --jit 1 run then records the segmented
    plan's choices, which would lower the bar to 0.1 s; the next auto process
    still walks the ahead-of-time plan.  Where a --jit 1 run came first, auto
    mode's first decision is the segmented walk, and it stays.  On a host of
    the modelled speed, the first cold auto run specialises (VERDICT r4
    next-2).  Each step is its own process (a process keeps its plans in
    memory)."""
    import subprocess
    import sys
    code = ("import sys, numpy as np, superman_amd as S\n"
            "a = S.read_matrix(sys.argv[1])[0]\n"
            "if sys.argv[2] == 'T': a = np.ascontiguousarray(a.T)\n"
            "if sys.argv[2] == 'R': a = np.ascontiguousarray(a[::-1])\n"
            "print(S.plan_info(a, 'dense', jit=int(sys.argv[3]))['kind'])\n")
    env = dict(os.environ, SUP_JIT_CACHE_DIR=str(tmp_path), SUP_JIT_BUDGET="190", PYTHONPATH=ROOT,
               OMP_NUM_THREADS="8")
    env.pop("SUP_JIT_COLD_RATIO", None)

    def kind(tr, jit, ratio=None):
        e = dict(env, SUP_JIT_COLD_RATIO=ratio) if ratio else env
        r = subprocess.run([sys.executable, "-c", code, fixture_path("double__40_0.50_0"), tr, str(jit)],
                           capture_output=True, text=True, env=e, timeout=300)
        assert r.returncode == 0, r.stderr
        return r.stdout.strip()

    assert kind("N", 0, ratio="8") == "sparse"  # cold, slow host
    assert kind("N", 1) == "seg"                 # records the segmented plan's choices
    assert kind("N", 0) == "sparse"              # warm: the recorded first decision, not the 0.1 s bar
    assert len(list(tmp_path.glob("auto_*.txt"))) == 1
    assert kind("T", 1) == "seg"     # another pattern, --jit 1 first
    assert kind("T", 0) == "seg"     # warm bar: the first auto decision is the segmented walk
    assert kind("T", 0, ratio="8") == "seg"
    assert kind("R", 0, ratio="1") == "seg"  # a fresh pattern, cold, a host of the modelled speed
    assert kind("R", 0, ratio="8") == "seg"  # and kept
    assert len(list(tmp_path.glob("auto_*.txt"))) == 3
    assert not list(tmp_path.glob(".auto_*"))  # no temporaries left behind


def test_seg_cost_model_reported(sup):
    a, _, _ = sup.read_matrix(fixture_path("synth/22_0.20_int"))
    _, st_seg = sup.perman_cpu(a, "seg", threads=4, return_stats=True)
    _, st_blk = sup.perman_cpu(a, "sparse", threads=4, return_stats=True)
    assert st_seg["walk_kind"] == 3 and st_blk["walk_kind"] == 1
    assert 0 < st_seg["est_ops_per_step"] < st_blk["est_ops_per_step"]


@pytest.mark.parametrize("case", ["n10", "n64", "zero_walk_col", "no_rest", "shared_streams"])
def test_generated_kernel_compiles(sup, case, tmp_path, monkeypatch, capfd):
    monkeypatch.setenv("SUP_JIT_CACHE_DIR", str(tmp_path))
    if case == "n10":
        a = _rand(10, 0.5, 7)
    elif case == "n64":
        a = _rand(64, 0.1, 8, ints=False)
    elif case == "zero_walk_col":
        a = _rand(24, 0.3, 9)
        a[:, 3] = 0.0  # a column with no nonzero: its steps only accumulate
    elif case == "shared_streams":  # one step class reads another's constant stream (share_streams)
        rng = np.random.default_rng(1)
        a = np.where(rng.random((28, 28)) < 0.9, rng.random((28, 28)) * 5, 0.0)
        a[np.arange(28), rng.permutation(28)] = 1.0 + rng.random(28)
        monkeypatch.setenv("SUP_JIT_VERBOSE", "1")
    else:
        a = _rand(24, 0.9, 10)  # every row touched by the walk columns: no rest segment
    info = sup.prepare(a, "seg")
    assert info["kind"] == "seg"
    assert info["compile_ms"] > 0.0
    assert len(list(tmp_path.glob("seg_*.co"))) >= 1  # disk cache written (one per budget the plan compiled)
    again = sup.prepare(a, "seg")
    assert again["compile_ms"] == 0.0  # in-memory cache
    if case == "shared_streams":
        assert "reads another class's stream" in capfd.readouterr().err


def test_dense_lds_plan_and_cpu(sup, orc):
    """SUP_KERNEL_DENSE_LDS: the plain dense walk with X staged in LDS on the
    GPU; the plan (and so the host twin and the oracle mirror) is the dense one."""
    a = _rand(14, 0.5, 21, ints=False)
    assert sup.plan_info(a, "dense_lds")["kind"] == "lds"
    got = sup.perman_cpu(a, "dense_lds", threads=4)
    assert got == sup.perman_cpu(a, "dense_plain", threads=4)
    assert got == orc.engine_perman_as(sup, a, "dense_lds", threads=4)


def _skip_case(sup, n, d, seed):
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < d
    mask[np.arange(n), rng.permutation(n)] = True
    a = np.where(mask, rng.integers(1, 6, (n, n)), 0).astype(np.float64)
    return sup.skip_order(a)[0]


@pytest.mark.parametrize("n,d,seed", [(24, 0.15, 4), (24, 0.15, 3)])
def test_cpu_seg_chunk_skip(sup, orc, n, d, seed):
    """Integer matrices whose rows untouched by the walk are exactly zero in
    whole wave-chunks: the walk skips those chunks (66 % and 84 % here); the
    host twin (which skips the same chunks) == the oracle mirror (which walks
    them and gets +-0) == the exact permanent."""
    from conftest import seg_skip_fraction
    a = _skip_case(sup, n, d, seed)
    assert seg_skip_fraction(sup, a) >= 0.25
    got = sup.perman_cpu(a, "seg", threads=8)
    assert got == orc.engine_perman_as(sup, a, "seg", threads=8)
    assert rel(got, float(orc.exact_perman_crt(a))) < 1e-12



def _n28(sup):
    rng = np.random.default_rng(28)
    n = 28
    mask = rng.random((n, n)) < 0.15
    mask[np.arange(n), rng.permutation(n)] = True
    a = np.where(mask, rng.random((n, n)) * 3, 0).astype(np.float64)
    return sup.sort_order(a)[0]


@pytest.mark.parametrize("b", [3, 4, 5, 6])
def test_cpu_seg_shared_steps_and_lane_fold(sup, orc, monkeypatch, b):
    """n = 28 (8 walk bits, b specialised pair bits, SUP_JIT_B forces b): the
    shared step of the walk bits above them and the two-level lane sum (acc
    folds into the running total after each shared step) run on the CPU too;
    host twin == oracle mirror bit for bit, and the prefix walk to 1e-11."""
    monkeypatch.setenv("SUP_JIT_B", str(b))
    a = _n28(sup)
    info = sup.plan_info(a, "seg")
    assert info["pair_bits"] == b
    assert info["m"] - 1 > b  # more pair bits than specialised ones: shared steps + folds
    got = sup.perman_cpu(a, "seg", threads=8)
    assert got == orc.engine_perman_as(sup, a, "seg", threads=8)
    assert rel(got, sup.perman_cpu(a, "sparse", threads=8)) < 1e-11


def test_seg_pair_bits_chosen_by_cost(sup, monkeypatch):
    """Without SUP_JIT_B the plan takes the specialised pair-bit count (5-8,
    at most m - 1) whose generated code has the fewest ops per Gray step
    (measured on MI355X, profiles/r2/probe_b.log: 5 -> 6 on the n = 40 bench
    matrix, 2.06e12 -> 2.14e12 Gray steps/s, as the op count predicts)."""
    for name, kernel in (("double__40_0.50_0", "dense"), ("double__40_0.20_0", "dense")):
        a, _, _ = sup.read_matrix(fixture_path(name))
        auto = sup.plan_info(a, kernel, jit=1)
        assert auto["kind"] == "seg" and 5 <= auto["pair_bits"] <= min(8, auto["m"] - 1)
        forced = {}
        for b in (5, 6, 7, 8):
            monkeypatch.setenv("SUP_JIT_B", str(b))
            info = sup.plan_info(a, kernel, jit=1)
            assert info["pair_bits"] == b
            forced[b] = info["est_ops_per_step"]
        monkeypatch.delenv("SUP_JIT_B")
        # the chosen plan is at least as cheap as every forced b whose code fits
        assert auto["est_ops_per_step"] <= min(forced[5], forced[6]) + 1e-9, (name, auto, forced)
        assert auto["est_ops_per_step"] == pytest.approx(forced[auto["pair_bits"]], abs=1e-9)


def test_seg_walk_length_rule(sup):
    """Cheap segmented walks run on longer wave-chunks (engine.cpp
    make_seg_plan): a chunk's walk should cost >= 32 chunk starts, with at
    least 2^14 chunks left (2^15 until round 6).  Measured on MI355X
    (profiles/r2/probe_walklen.log, profiles/r6/cfg2_knobs.log, cfg3_m.log):
    config 3 2.94 -> 2.12 ms at m = 14 (1.905 at 15), config 2 0.580 -> 0.555 ms
    at m = 11, the d = 0.2 companion 36.1 -> 33.4 ms at m = 15; the bench matrix
    (12.7 ops per step) keeps m = 13."""
    cases = (("double__40_0.50_0", 0, "dense", 13, 13), ("double__40_0.20_0", 0, "dense", 14, 19),
             ("double__36_0.20_0", 1, "sparse", 13, 15), ("double__32_0.50_0", 0, "dense", 11, 11))
    for name, prep, kernel, lo, hi in cases:
        a = sup.read_matrix(fixture_path(name))[0]
        if prep:
            a = sup.sort_order(a)[0]
        info = sup.plan_info(a, kernel, jit=1)
        n = a.shape[0]
        assert info["kind"] == "seg" and info["L"] == 6 and lo <= info["m"] <= hi, (name, info["m"])
        assert n - 1 - 6 - info["m"] >= min(14, sup.layout(n)[2])
        if info["m"] > sup.layout(n)[1]:  # the walk's own steps now dwarf a chunk start, or the chunks ran out
            assert info["est_ops_per_step"] * 2.0 ** info["m"] >= 32 * 2048 or n - 1 - 6 - info["m"] == 14


@pytest.mark.parametrize("n,d,seed", [(16, 0.5, 31), (18, 0.35, 32)])
def test_cpu_seg_storage_plan_invariance(sup, orc, monkeypatch, tmp_path, n, d, seed):
    """Every value of the segmented walk is a pure function of x^0, so keeping a
    row or node copy live or forming it on demand changes ops and registers,
    never a bit.  Storage budgets from "everything on demand" (0) to
    "everything live" (1000) keep the walk order and the arithmetic (host twin
    == oracle mirror, which restate no storage plan), and every such kernel
    compiles for gfx950 (the GPU twin of this test checks the bits)."""
    monkeypatch.setenv("SUP_JIT_CACHE_DIR", str(tmp_path))
    a = _rand(n, d, seed, ints=False)
    want = orc.engine_perman_as(sup, a, "seg", threads=4)
    cm = sup.plan_info(a, "seg")["colmap"]
    for budget in (0, 40, 1000):
        monkeypatch.setenv("SUP_JIT_STORAGE", str(budget))
        assert (sup.plan_info(a, "seg")["colmap"] == cm).all()
        assert sup.perman_cpu(a, "seg", threads=4) == want, budget
        assert sup.prepare(a, "seg")["kind"] == "seg"


def test_seg_skip_aware_plan(sup, monkeypatch):
    """Integer matrices: the planner weighs each walk by its ops per Gray step
    times the fraction of wave-chunks it cannot skip (sampled); measured over
    every chunk (conftest.seg_skip_fraction, numpy), the chosen plan's effective
    cost is no worse than the op-count-only plan's."""
    from conftest import seg_skip_fraction
    for n, d, seed in ((24, 0.15, 4), (26, 0.15, 5)):
        a = _skip_case(sup, n, d, seed)
        eff = {}
        for polish in ("1", "0"):
            monkeypatch.setenv("SUP_JIT_POLISH", polish)
            info = sup.plan_info(a, "seg")
            eff[polish] = info["est_ops_per_step"] * (1.0 - seg_skip_fraction(sup, a, "seg"))
        assert eff["1"] <= eff["0"] * 1.05 + 1e-12, (n, eff)


def test_seg_uncompilable_pattern_falls_back(sup, tmp_path, monkeypatch):
    """A kernel hiprtc refuses (SUP_JIT_FAIL stands in for a register
    allocator that gives up): the plan check (jit.cpp build_seg) refuses the
    segmented walk, a dense request runs the ahead-of-time walk instead, an
    explicit segmented request fails loudly, and later kernels still compile
    in the same process (one at a time after a failure)."""
    monkeypatch.setenv("SUP_JIT_CACHE_DIR", str(tmp_path))
    a = _rand(36, 0.9, 1029, ints=False)  # a walk of >= 10 ms: planning compiles and checks the kernel
    monkeypatch.setenv("SUP_JIT_FAIL", "1")
    assert sup.plan_info(a, "dense", jit=1)["kind"] in ("dense", "sparse")
    with pytest.raises(sup.SupError):
        sup.plan_info(a, "seg", jit=1)
    monkeypatch.delenv("SUP_JIT_FAIL")
    assert sup.prepare(_rand(24, 0.5, 11), "seg")["kind"] == "seg"


def test_seg_near_dense_large_n_compiles(sup, tmp_path, monkeypatch):
    """The dense n = 60, d = 0.9 pattern hiprtc refused until round 3 ("inline
    assembly requires more registers than available": a region pinned all 8
    SGPR pieces of a near-dense D product beside the next region's prefetch)
    now gets a segmented plan whose walk loop has no scratch (the plan's
    compiler check)."""
    monkeypatch.setenv("SUP_JIT_CACHE_DIR", str(tmp_path))
    rng = np.random.default_rng(1029)
    n = 60
    a = np.where(rng.random((n, n)) < 0.9, rng.random((n, n)) * 5, 0.0)
    a[np.arange(n), rng.permutation(n)] = 1.0
    info = sup.plan_info(a, "seg", jit=1)
    assert info["kind"] == "seg"
    assert info["est_ops_per_step"] < sup.plan_info(a, "dense", jit=-1)["est_ops_per_step"]

def test_seg_shards_balanced_under_chunk_skip(sup):
    """Config 5 (n = 44 d = 0.15 int, SkipOrder): the segmented walk skips 87 %
    of its wave-chunks.  The high columns that touch no walk-untouched row never
    change a skip, and the planner puts them on the top chunk bits, so the
    contiguous shards of sup_perman_shard / -p5 walk equal chunk counts at 2, 4
    and 8 GPUs (before: the top bit alone decided, half the shards were empty).
    Restated in numpy from the plan's column map (conftest.seg_skipped_chunks)."""
    from conftest import seg_skipped_chunks
    a = sup.skip_order(sup.read_matrix(fixture_path("synth44_0.15_int"))[0])[0]
    walked = ~seg_skipped_chunks(sup, a, "sparse")
    assert 0.05 < walked.mean() < 0.5
    C = walked.size
    for world in (2, 4, 8):
        w = [int(walked[C * r // world:C * (r + 1) // world].sum()) for r in range(world)]
        assert max(w) == min(w), (world, w)


def test_seg_scheduling_knobs_keep_pinned_plan(sup, tmp_path, monkeypatch):
    """With the plan pinned (SUP_JIT_CC: no compiler check), the scheduling-only
    knobs (region pieces, accumulate float, LLVM scheduler strategy) leave the
    walk order, layout, cached and pair bits unchanged: only the kernel source
    and so the plan key move.  Unpinned, a knob may change the plan (the short
    walk's 4-cached-bit kernel is re-planned with 3 when its loop scratches), so
    GPU bit-parity is checked against the mirror of the plan walked
    (test_gpu_seg.py::test_seg_codegen_schedule_invariance_gpu)."""
    monkeypatch.setenv("SUP_JIT_CACHE_DIR", str(tmp_path))
    monkeypatch.setenv("SUP_JIT_CC", "3")
    rng = np.random.default_rng(91)
    n = 28
    a = np.where(rng.random((n, n)) < 0.5, rng.random((n, n)) * 5, 0.0)
    a[np.arange(n), rng.permutation(n)] = 1.0

    def strip(info):
        return (info["kind"], info["colmap"].tolist(), info["L"], info["m"], info["cached"], info["pair_bits"],
                info["est_ops_per_step"])
    base = strip(sup.plan_info(a, "seg"))
    keys = {sup.plan_key(a, "seg")}
    for knob, v in (("SUP_JIT_KP", "1"), ("SUP_JIT_ACCFLOAT", "0"), ("SUP_JIT_SCHED", "max-ilp")):
        monkeypatch.setenv(knob, v)
        assert strip(sup.plan_info(a, "seg")) == base, knob
        keys.add(sup.plan_key(a, "seg"))
        monkeypatch.delenv(knob)
    assert len(keys) == 4


def test_budget_ladder_helper_compiles_same_plan(tmp_path):
    """The budget ladder's candidates compiled ahead of the bisection by
    sup_rtc helper processes (one per host core; jit.cpp prefetch_compiles)
    give the plan the serial in-process bisection gives: the same plan key
    (walk, tables, kernel source), and every code object both runs compiled is
    byte-identical — the helper loads this process's own hiprtc."""
    import subprocess
    import sys
    code = ("import sys, numpy as np, superman_amd as S\n"
            "a = np.load(sys.argv[1])\n"
            "r = S.prepare(a, 'dense', jit=1)\n"
            "print(r['kind'], hex(S.plan_key(a, 'dense', jit=1)))\n")
    rng = np.random.default_rng(38)
    a = np.where(rng.random((38, 38)) < 0.5, rng.random((38, 38)) * 5, 0.0)
    a[np.arange(38), rng.permutation(38)] = 1.0
    np.save(tmp_path / "a.npy", a)
    out, objs = [], []
    for procs in ("0", "8"):
        cache = tmp_path / f"cache{procs}"
        env = dict(os.environ, SUP_JIT_CACHE_DIR=str(cache), AMD_COMGR_CACHE_DIR=str(cache / "comgr"),
                   SUP_RTC_PROCS=procs, PYTHONPATH=ROOT, OMP_NUM_THREADS="8")
        r = subprocess.run([sys.executable, "-c", code, str(tmp_path / "a.npy")], capture_output=True, text=True,
                           env=env, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        out.append(r.stdout.split())
        objs.append({p.name: p.read_bytes() for p in cache.glob("seg_*.co")})
    assert out[0][0] == "seg" and out[0] == out[1]
    assert len(objs[1]) > len(objs[0]) >= 2  # the helpers compiled ahead; the serial run only what it visited
    for name, data in objs[0].items():
        assert objs[1][name] == data, name
