#!/usr/bin/env python3
"""bench.py — Gray-code subset-steps/s of the exact Ryser permanent on MI355X.

Workload (BASELINE.json configs[3], the metric's config): the reference corpus
matrix double/40_0.50_0 (n = 40, d = 0.5), dense walk (-p4/-p6 path), all
2^39 Gray steps per "step".  With N ranks (one process per GPU, launched by
torch.distributed.run) the 2^h wave-chunks are split into N contiguous
power-of-two-aligned shards; each rank walks its shard through the C ABI
(sup_perman_shard) and one RCCL all-reduce (torch.distributed, backend nccl)
of a one-slot-per-rank vector, folded pairwise, sums the fp64 partials — the
only data-path collective; the result is bit-identical to the one-GPU walk.  Total work per
step is fixed (one permanent), so scaling is "strong".

The walk kernel is the segmented walk specialised for the matrix's pattern
(superman_amd/csrc/jit.cpp; --jit 1, the default here): it is compiled once
with hiprtc before the warmup (compile time reported as config.jit_compile_ms,
outside the timed region, like the plan), then every timed step walks all
2^39 Gray steps.  --jit -1 runs the ahead-of-time prefix-blocked kernel.

The north star also asks for density 0.2: the reference corpus matrix
double/40_0.20_0 (--also) is timed the same way (same shards, all-reduce and
clock) and reported under "densities"; `value` stays the d = 0.5 metric.
BASELINE configs 2, 3 and 5 are timed the same way under "configs"
(--configs 0 skips them).

Prints ONE JSON line on rank 0 (driver contract), including the roofline of
the walk kernel and a CPU baseline (oracle/ port of the reference's
parallel_perman64 chunk loop, timed on a bounded sample of the same workload
on this host's cores; beside it the reference's own compiled CPU code on
config 1).  Roofline: `achieved` = the walk's fp64 flops per Gray step
measured by rocprofv3 --pmc (SQ_INSTS_VALU_{ADD,MUL,FMA}_F64, FMA = 2 flops;
a child run of this script under rocprofv3, --pmc 1, N = 1) x the Gray steps
of a launch / the launch's mean duration (hipEvents on the walk's stream,
inside the library); `traffic` = HBM bytes per launch from the committed
FETCH_SIZE / WRITE_SIZE passes of the same plan (profiles/r3, tools/pmc_r3.py).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Gray-code subset-steps/sec (dense n=40, d=0.5) at 1/2/4/8 MI355X; rel-err vs CPU"
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 (vector = matrix), MI355X_MICROARCH.md / SURVEY §8(d)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU). Without WORLD_SIZE in the environment and N > 1, this process "
                         "starts torch.distributed.run with N ranks as a child and forwards its output")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--matrix", default=os.path.join(ROOT, "tests", "fixtures", "double__40_0.50_0"))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample budget (0 = skip)")
    ap.add_argument("--kernel", default="dense", choices=["dense", "dense_plain", "dense_lds", "sparse", "skip", "seg"],
                    help="dense = -p4/-p6 (engine picks the cheapest walk); sparse/skip = -s paths")
    ap.add_argument("--jit", type=int, default=1, choices=[-1, 0, 1],
                    help="segmented walk specialised for the pattern: 1 when cheaper, 0 auto, -1 never")
    ap.add_argument("--rehearse", action="store_true",
                    help="all ranks on device 0 over gloo: rehearse the N-rank path on a one-GPU box")
    ap.add_argument("--prep", type=int, default=0, choices=[0, 1, 2], help="-r: 1 SortOrder, 2 SkipOrder")
    ap.add_argument("--configs", type=int, default=1, help="also time BASELINE configs 2, 3 and 5 (0 = skip)")
    ap.add_argument("--also", default=",".join(os.path.join(ROOT, "tests", "fixtures", f)
                                                for f in ("double__40_0.20_0", "double__40_0.90_0")),
                    help="comma-separated companion matrices timed the same way (north star: densities "
                         "0.2 and 0.5 at every N; 0.9: a near-dense point); '' = none")
    ap.add_argument("--pmc", type=int, default=1,
                    help="1: measure the walk kernel's fp64 flops with rocprofv3 --pmc in a child run "
                         "(N = 1, rank 0; falls back to the committed profile); 0: committed profile only")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cold", type=int, default=1, help="time the CLI end to end with an empty / warm cache (N = 1)")
    ap.add_argument("--pg", action="store_true",
                    help="create the process group (RCCL, device_id = this rank's GPU) and run every collective "
                         "even at world 1: executes the N-GPU code path on a one-GPU box")
    return ap.parse_args()


def shard_chunks(n: int, rank: int, world: int) -> tuple[int, int]:
    """Wave-chunk range [c0, c1) of this rank's shard (sup_perman_shard): a
    contiguous run of the 2^h wave-chunks, power-of-two aligned when world is
    a power of two (then the shards are subtrees of the fixed reduction)."""
    import superman_amd as S
    L, m, h = S.layout(n)
    C = 1 << h
    return C * rank // world, C * (rank + 1) // world


def pairwise(parts):
    """Pairwise fold in index order (zero-padded to even length at each level):
    the engine's reduction tree, so power-of-two aligned shards combine to the
    single-device sum bit for bit."""
    parts = list(parts)
    while len(parts) > 1:
        if len(parts) & 1:
            parts.append(0.0)
        parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
    return parts[0]


def combine(part: float, rank: int, world: int, device) -> float:
    """Sum of every rank's shard partial with one all-reduce (RCCL over xGMI on
    the GPU ranks): a vector with one slot per rank, each rank filling its own,
    so every slot has a single nonzero addend and the all-reduce is exact in any
    ring order; then the pairwise fold.  The N-GPU permanent is therefore
    bit-identical to the one-GPU walk (the scalar all-reduce's own summation
    order differed from it in the last bits)."""
    import torch
    import torch.distributed as dist
    v = torch.zeros(world, dtype=torch.float64, device=device)
    v[rank] = part
    dist.all_reduce(v)  # the single data-path collective
    return pairwise(v.cpu().tolist())


def check_plans_agree(key: int, rank: int, world: int, device) -> list:
    """Every rank plans on its own (plan + compile before the warmup); the
    shards add up to the permanent only if all ranks walk the same plan.
    All-gather each rank's plan fingerprint (sup_plan_key: walk kind, layout,
    column map, tables, kernel source) and abort on any mismatch."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return [key]
    t = torch.tensor([key - (1 << 64) if key >= (1 << 63) else key], dtype=torch.int64, device=device)
    got = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(got, t)
    keys = [int(x.item()) & ((1 << 64) - 1) for x in got]
    if len(set(keys)) != 1:
        raise RuntimeError(f"rank {rank}: ranks planned different walks, their shards would not sum to one "
                           f"permanent: plan keys {[hex(k) for k in keys]}")
    return keys


# fp64 instruction counters (gfx950, rocprofv3 counter_defs.yaml: per-wave
# instructions, summed over SEs); flops = 64 lanes x (ADD + MUL + 2 FMA), the
# same expression as rocprofv3's derived FP64 FLOPS counter.  One pass: 6 SQ
# + 2 GRBM counters (the hardware allows 8 SQ, 2 GRBM per pass).
PMC_COUNTERS = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU",
                "SQ_WAVES", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]


def auto_decision(S, a, kernel: str, rank: int, world: int, dev: int, device) -> int:
    """Auto mode (jit = 0) decides from the disk cache's state: whether this
    matrix's plan choices are recorded, what this host's last cold plan cost.
    Ranks sharing a cache see it at different moments (one rank's plan writes
    what the next one reads), so they could decide differently.  Rank 0
    decides; every rank then walks that choice explicitly (jit = 1: the
    segmented walk, -1: the ahead-of-time kernel), the same plan auto mode
    chose."""
    import torch
    import torch.distributed as dist
    v = 0
    if rank == 0:
        v = 1 if S.plan_info(a, kernel, jit=0, gpu_num=world, device_id=dev)["kind"] == "seg" else -1
    t = torch.tensor([v], dtype=torch.int64, device=device)
    dist.broadcast(t, 0)
    return int(t.item())


def pmc_child(args) -> None:
    """--pmc-child: one launch of the walk the parent times (same plan: same
    matrix, kernel request, jit, one shard), run under rocprofv3 by the parent."""
    import superman_amd as S
    a = S.read_matrix(args.matrix)[0]
    if args.prep == 1:
        a = S.sort_order(a)[0]
    elif args.prep == 2:
        a = S.skip_order(a)[0]
    S.prepare(a, args.kernel, jit=args.jit, gpu_num=1)
    _, st = S.perman_shard(a, 0, 1, kernel=args.kernel, jit=args.jit, return_stats=True)
    print(json.dumps({"gray_steps": st["gray_steps"], "visited_steps": st["visited_steps"],
                      "walk_kind": st["walk_kind"]}), flush=True)


def kernel_matches(walk: str, name: str) -> bool:
    """rocprofv3's kernel name against a walk kernel's: `sup::walk_skip<44>`
    also matches the launched form `sup::walk_skip<44, 3>` (walk_skip.hip)."""
    return walk in name or (walk.endswith(">") and walk[:-1] + "," in name)


def pmc_live(matrix: str, kernel: str, jit: int, prep: int, walk: str):
    """Measured fp64 work of one launch of `walk`: runs this script's
    --pmc-child under `rocprofv3 --pmc` (a child process, --kernel-trace only)
    and reads the counters of the walk kernel's dispatch.  None if rocprofv3
    is absent or the pass fails (the caller falls back to the committed
    profile)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    out = tempfile.mkdtemp(prefix="sup_pmc_")
    cmd = [prof, "--pmc", *PMC_COUNTERS, "--kernel-trace", "-d", out, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-child", "--matrix", matrix, "--kernel", kernel,
           "--jit", str(jit), "--prep", str(prep)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
        child = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
        vals, ns = {}, []
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if kernel_matches(walk, row["Kernel_Name"]):
                    vals[row["Counter_Name"]] = vals.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                    ns.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        if r.returncode != 0 or not child or "SQ_INSTS_VALU_FMA_F64" not in vals:
            return None
    except (subprocess.SubprocessError, OSError, ValueError):
        return None
    finally:
        shutil.rmtree(out, ignore_errors=True)
    steps = child[-1]["gray_steps"]
    flops = 64.0 * (vals["SQ_INSTS_VALU_ADD_F64"] + vals["SQ_INSTS_VALU_MUL_F64"] + 2.0 * vals["SQ_INSTS_VALU_FMA_F64"])
    fp64_insts = vals["SQ_INSTS_VALU_ADD_F64"] + vals["SQ_INSTS_VALU_MUL_F64"] + vals["SQ_INSTS_VALU_FMA_F64"]
    wave_steps = steps / 64.0
    return {"flops_per_gray_step": flops / steps,
            "fp64_insts_per_lane_step": fp64_insts / wave_steps,
            "fma_share": vals["SQ_INSTS_VALU_FMA_F64"] / fp64_insts,
            "valu_insts_per_lane_step": vals.get("SQ_INSTS_VALU", 0.0) / wave_steps,
            "kernel_ns_under_pmc": max(ns) if ns else None,
            "counters": {k: vals[k] for k in PMC_COUNTERS if k in vals},
            "source": "rocprofv3 --pmc " + " ".join(PMC_COUNTERS) + " --kernel-trace, one launch of this walk "
                      "(bench.py --pmc-child, same plan), measured in this run"}


def pmc_committed(n: int, walk: str, key: str):
    """The committed F64-counter profile of this walk (profiles/*/pmc_f64_*.json,
    tools/pmc_summary.py f64) when it was taken on the same plan (plan key)."""
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_f64_*.json"), recursive=True), reverse=True):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("n") == n and walk in d.get("kernel", "") and d.get("plan_key") == key:
            d["source"] = f"committed profile {os.path.relpath(p, ROOT)} (same plan key)"
            return d
    return None


def pmc_record(n: int, kernel: str, key: str):
    """The committed rocprofv3 HBM profile (FETCH_SIZE + WRITE_SIZE per launch,
    tools/pmc_r3.py hbm) of this walk kernel taken on the same plan (plan
    key); None if there is none."""
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc*.json"), recursive=True), reverse=True):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if (d.get("n") == n and "hbm_bytes_per_launch" in d and kernel.split("::")[-1] in d.get("kernel", "")
                and d.get("plan_key") == key):
            d["_path"] = os.path.relpath(p, ROOT)
            return d
    return None


def hbm_traffic(pmc):
    """HBM bytes per launch from a committed FETCH_SIZE / WRITE_SIZE profile:
    FETCH_SIZE doubled (on gfx950 it reports half the bytes of a wide
    coalesced read, MI355X_MICROARCH.md's HBM / rocprofv3 section) unless the
    profile applied that already; None without a profile."""
    if not pmc:
        return None
    if pmc.get("fetch_size_doubled") or "fetch_bytes" not in pmc or "write_bytes" not in pmc:
        return pmc.get("hbm_bytes_per_launch")
    return 2.0 * pmc["fetch_bytes"] + pmc["write_bytes"]


def cpu_baseline(a, n: int, budget_s: float, gpu_sup, kernel: str):
    """Reference algorithm (oracle port of cpu_perman64, gpu_exact_dense.cu:6-69)
    on an aligned sample [2^(n-2), 2^(n-2)+S) of the same workload, all host
    threads; also the GPU (same walk family as the bench) on the same sample
    for the relative error."""
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    s0 = 1 << (n - 2)
    probe = 1 << 24
    t = time.perf_counter()
    oracle.ref_dense_partial(a, s0, s0 + probe, threads)
    dt = max(time.perf_counter() - t, 1e-3)
    rate = probe / dt
    k = max(20, min(n - 2, int((rate * budget_s)).bit_length() - 1))
    size = 1 << k
    t = time.perf_counter()
    cpu = oracle.ref_dense_partial(a, s0, s0 + size, threads)
    dt = time.perf_counter() - t
    gpu = gpu_sup.partial(a, s0, s0 + size, kernel=kernel)
    err = abs(gpu - cpu) / max(abs(cpu), 1e-300)
    return {"value": size / dt, "unit": "gray-steps/s", "cores": threads, "kind": "port",
            "sample": f"reference Gray indices [2^{n-2}, 2^{n-2}+2^{k}) of {os.path.basename(args.matrix)} "
                      f"({dt:.1f} s, oracle/oracle.c orc_ref_dense_partial = cpu_perman64 restated)"}, err


def cold_start(matrix: str) -> dict:
    """End-to-end wall time of the drop-in CLI (`perman -f <matrix> -g -p4`,
    a fresh process: HIP init, read, plan, compile, walk, print).  "Cold" is
    an empty plan cache AND an empty comgr cache (hiprtc's compiles are cached
    by comgr under ~/.cache/comgr, so a plan after another process compiled
    the same kernels would not be cold):
      cold_default  jit = 0 (auto: on a host of the modelled speed the n = 40
                    matrix specialises — its ~0.5 s saving per run repays the
                    ~1.6 s plan within 4 runs, and the decision is recorded),
      cold_jit1     --jit 1, its own empty caches (search + compile + walk),
      cold_aot      --jit -1, its own empty caches (the ahead-of-time walk:
                    what a one-shot run would cost without specialising),
      warm_default  jit = 0 again in cold_default's caches: the recorded
                    decision, plan choices and kernel are on disk."""
    import shutil
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "superman_amd", "bin", "perman")
    out = {"command": f"superman_amd/bin/perman -f {os.path.relpath(matrix, ROOT)} -g -p4 [--jit 1|-1]",
           "cache": "empty SUP_JIT_CACHE_DIR and AMD_COMGR_CACHE_DIR per cold run; warm_default reuses "
                    "cold_default's"}
    dirs = {k: tempfile.mkdtemp(prefix=f"sup_{k}_") for k in ("default", "jit1", "aot")}
    try:
        for label, extra, d in (("cold_default", [], "default"), ("cold_jit1", ["--jit", "1"], "jit1"),
                                ("cold_aot", ["--jit", "-1"], "aot"), ("warm_default", [], "default")):
            env = dict(os.environ, SUP_JIT_CACHE_DIR=os.path.join(dirs[d], "plans"),
                       AMD_COMGR_CACHE_DIR=os.path.join(dirs[d], "comgr"))
            t = time.perf_counter()
            r = subprocess.run([exe, "-f", matrix, "-g", "-p4", "-v", *extra], capture_output=True, text=True,
                               env=env, timeout=300)
            wall = time.perf_counter() - t
            perm = [ln.split()[1] for ln in r.stdout.splitlines() if ln.startswith("Permanent:")]
            kinds = {"0": "dense", "1": "prefix-blocked", "2": "skipper", "3": "segmented"}
            walk = [kinds.get(ln.split("walk_kind")[1].split()[0]) for ln in r.stdout.splitlines()
                    if ln.startswith("Stats:") and "walk_kind" in ln]
            out[label] = {"wall_s": wall, "rc": r.returncode, "permanent": float(perm[0]) if perm else None,
                          "walk": walk[0] if walk else None}
    except (subprocess.SubprocessError, OSError, ValueError) as e:
        out["error"] = repr(e)
    finally:
        for d in dirs.values():
            shutil.rmtree(d, ignore_errors=True)
    return out


def cpu_reference_config1(S, threads: int):
    """The reference's own CPU code (parallel_perman64, rev/cpu_algos.hpp:761,
    compiled unmodified from the reference sources into oracle/_ref/ref_v2 by
    oracle/Makefile) on BASELINE config 1 (double/30_0.50_0, all 2^29 Gray
    steps), next to the oracle port on the same input: shows the port that
    `cpu_baseline` times at n = 40 runs at the reference's speed."""
    import subprocess
    import oracle
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_v2")
    mat = os.path.join(ROOT, "tests", "fixtures", "double__30_0.50_0")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, mat, "dense", str(threads)], capture_output=True, text=True, timeout=120,
                             check=True).stdout.split()
        ref_perm, ref_s = float(out[0]), float(out[1])
    except (subprocess.SubprocessError, OSError, ValueError, IndexError):
        return None
    a = S.read_matrix(mat)[0]
    t = time.perf_counter()
    port_perm = oracle.ref_dense(a, threads)
    port_s = time.perf_counter() - t
    steps = 1 << 29
    return {"value": steps / ref_s, "unit": "gray-steps/s", "cores": threads, "kind": "reference",
            "sample": "oracle/_ref/ref_v2 (reference parallel_perman64<double,double>, compiled from the reference "
                      f"sources) on double/30_0.50_0, all 2^29 steps, {ref_s:.2f} s (its own timer)",
            "port_value": steps / port_s,
            # the reference adds its thread partials in omp-critical completion order
            "port_rel_diff": abs(port_perm - ref_perm) / abs(ref_perm)}


def reference_metric_run(matrix: str):
    """The reference's own CPU code on the whole metric workload — committed,
    not re-run here: oracle/_ref/ref_v2 (parallel_perman64<double,double>,
    rev/cpu_algos.hpp:761-873, compiled from the reference sources) walked all
    2^(n-1) steps of this file once in the build container (8 cores;
    tests/golden/make_golden.py), ~68 min at n = 40.  Its result beside the
    exact permanent shows the reference's own fp64 error at this size."""
    name = os.path.basename(matrix)
    try:
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
        ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
    except (OSError, ValueError):
        return None
    key = f"{name}|dense|r0|b0|t8"
    if key not in gold or key + "|seconds" not in gold:
        return None
    n = int(open(matrix).readline().split()[0])
    sec = gold[key + "|seconds"]
    out = {"value": float(1 << (n - 1)) / sec, "unit": "gray-steps/s", "cores": 8, "kind": "reference",
           "seconds": sec, "permanent": gold[key],
           "sample": f"all 2^{n - 1} steps of {name}, once, in the build container (8 cores, niced beside builds; "
                     "committed in tests/golden/golden.json, not timed on this box)"}
    if name in ex:
        out["rel_err_vs_exact"] = abs(gold[key] - ex[name]) / abs(ex[name])
    return out


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """`bench.py --gpus N` started by hand (no WORLD_SIZE): start N ranks, one
    process per GPU, with torch.distributed.run as a CHILD process and return
    its exit code.  Nothing here touches the GPU (torch.cuda.device_count()
    does not initialise it on this image; `superman_amd` is not imported), so
    the ranks own their devices; no exec.  Rank 0's JSON line reaches our
    stdout unchanged (inherited file descriptors)."""
    import subprocess
    if not args.rehearse:
        import torch
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} asks for {n} ranks, one per GPU, but this node has {have} GPU(s); "
                  f"use --rehearse to put all ranks on device 0", file=sys.stderr, flush=True)
            return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or n) // n)))
    return subprocess.run(cmd, env=env).returncode


def main():
    global args
    args = parse()
    if args.pmc_child:
        return pmc_child(args)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: the launcher and the flag disagree",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if args.gpus is not None and args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr, flush=True)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # --rehearse: every rank on device 0 with gloo (multi-rank rehearsal on a
    # one-GPU box); the real N-GPU run uses one device per rank and RCCL.
    dev = 0 if args.rehearse else local
    tdev = "cpu" if args.rehearse else f"cuda:{dev}"
    # use_pg: the process group exists and every collective below runs (world
    # > 1, or --pg at world 1, which executes the RCCL branch on one GPU)
    use_pg = world > 1 or args.pg
    # the ranks plan at once: each compiles its budget ladder ahead with helper
    # processes (one per core up to 16); share the host's cores among them
    if world > 1 and "SUP_RTC_PROCS" not in os.environ:
        os.environ["SUP_RTC_PROCS"] = str(max(2, 16 // world))
    if use_pg:
        if env_world is None:  # --pg without a launcher: a one-rank group on this host
            os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        torch.cuda.set_device(dev)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    import superman_amd as S

    def load(path, prep=None):
        a = S.read_matrix(path)[0]
        prep = args.prep if prep is None else prep
        if prep == 1:
            a = S.sort_order(a)[0]
        elif prep == 2:
            a = S.skip_order(a)[0]
        return a

    def barrier():
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()

    plan_keys = []  # every timed walk's per-rank plan fingerprints (all equal, or check_plans_agree raised)

    def timed(a, kernel=None, jit=None, min_seconds=0.0):
        """W untimed + K timed steps of one whole permanent of `a`; returns
        (elapsed max over ranks, permanent, mean walk-kernel ms, stats, compile ms, K).
        K = --steps, or (min_seconds > 0: the short config lines) enough steps
        for ~min_seconds, so the barriers around the timed region do not
        dominate a sub-millisecond step (at most 4000, the same K on every rank)."""
        n = a.shape[0]
        kernel = args.kernel if kernel is None else kernel
        jit = args.jit if jit is None else jit
        if jit == 0 and use_pg:
            jit = auto_decision(S, a, kernel, rank, world, dev, tdev)
        # plan + (segmented walk) hiprtc compile, once, before the timed region;
        # gpu_num = world so that --jit 0 decides as the N-rank plan would
        prep = S.prepare(a, kernel, jit=jit, gpu_num=world, device_id=dev)
        keys = check_plans_agree(S.plan_key(a, kernel, jit=jit, gpu_num=world, device_id=dev), rank, world, tdev)
        plan_keys.append([hex(k) for k in keys])

        # the same C-ABI call every step (sup_perman_shard), its arguments built
        # once; its walk's HIP events are read after the timed steps
        # (sup_opts.timing = 0: a call returns when its result is there instead
        # of waiting for the end event too)
        call = S.ShardCall(a, rank, world, kernel=kernel, device_id=dev, jit=jit, timing=False)

        def step():
            part, k_ms = call()
            if use_pg:
                part = combine(part, rank, world, tdev)  # one RCCL all-reduce over xGMI
            return (4 * (n & 1) - 2) * part, k_ms

        one = None
        for _ in range(args.warmup):
            t1 = time.perf_counter()
            step()
            one = time.perf_counter() - t1
        steps = args.steps
        if min_seconds > 0:
            if one is None:
                t1 = time.perf_counter()
                step()
                one = time.perf_counter() - t1
            steps = max(args.steps, min(4000, int(min_seconds / max(one, 1e-6)) + 1))
            if use_pg:
                t = torch.tensor([steps], dtype=torch.float64, device=tdev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                steps = int(t.item())
        S.kernel_time(dev)  # (the warm-up walks' times: dropped)
        barrier()
        t0 = time.perf_counter()
        perm = None
        for _ in range(steps):
            perm, _ = step()
        barrier()
        elapsed = time.perf_counter() - t0
        k_total, k_n = S.kernel_time(dev)  # the timed walks' HIP-event times (walk stream)
        assert k_n == steps, (k_n, steps)
        st = call.stats()
        if use_pg:
            t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, perm, k_total / k_n, st, prep["compile_ms"], steps

    walk_names = {0: "dense", 1: "prefix-blocked", 2: "skipper", 3: "segmented (pattern-specialised)",
                  4: "dense, X in LDS"}

    def walk_kernel(st, n):
        return {0: f"sup::walk_dense<{n}>", 1: f"sup::walk_sparse<{n}>", 2: f"sup::walk_skip<{n}>",
                3: "sup_walk_seg", 4: f"sup::walk_lds<{n}>"}[st["walk_kind"]]

    def roofline(path, b, prep, kernel, jit, kms, st):
        """Roofline of the walk kernel for this rank's shard.  achieved = the
        walk's fp64 flops per Gray step MEASURED with rocprofv3 --pmc (FMA = 2
        flops; pmc_live, or the committed profile of the same plan) x this
        rank's Gray steps / its mean walk-kernel time (hipEvents on the walk's
        stream, inside the library).  Without a measurement the cost model
        stands in and `achieved_source` says so.  SURVEY 8(d)'s nominal 2n
        flops per Gray step (the plain walk's n adds + n muls) is kept as
        gray_step_equiv_*: the rate the plain algorithm would need."""
        nb = b.shape[0]
        steps = st["gray_steps"]  # this rank's shard
        walk = walk_kernel(st, nb)
        key = hex(S.plan_key(b, kernel, jit=jit, gpu_num=world, device_id=dev))
        meas = pmc_live(path, kernel, jit, prep, walk) if (args.pmc and world == 1 and rank == 0) else None
        meas = meas or pmc_committed(nb, walk, key)
        fps = meas["flops_per_gray_step"] if meas else st["est_ops_per_step"]
        achieved = fps * steps / (kms * 1e-3) / 1e12
        nominal = 2.0 * nb * steps / (kms * 1e-3) / 1e12
        r = {"bound": "valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
             "frac": achieved / FP64_PEAK_TFLOPS, "kernel": walk, "kernel_ms_avg": kms,
             "flops_per_gray_step": fps,
             "achieved_source": meas["source"] if meas else "cost model (no rocprofv3 measurement available)",
             "algorithmic_flops_per_launch": fps * steps,
             "flops_definition": "fp64 flops per Gray step executed by the walk kernel: 64 x (SQ_INSTS_VALU_ADD_F64 "
                                 "+ SQ_INSTS_VALU_MUL_F64 + 2 SQ_INSTS_VALU_FMA_F64) per launch / its Gray steps",
             "model_ops_per_gray_step": st["est_ops_per_step"],
             "gray_step_equiv_tflops": nominal, "gray_step_equiv_frac": nominal / FP64_PEAK_TFLOPS,
             "gray_step_equiv_definition": f"2n = {2 * nb} fp64 flops per Gray step (SURVEY 8(d), the plain walk's "
                                           "n adds + n muls); above 1 where the walk skips the operations "
                                           "structural zeros make redundant", "plan_key": key}
        if meas:
            r["fp64_insts_per_lane_step"] = meas.get("fp64_insts_per_lane_step")
            r["fma_share"] = meas.get("fma_share")
            r["valu_insts_per_lane_step"] = meas.get("valu_insts_per_lane_step")
            # fp64 VALU issue: one wave-instruction per 4 cycles per SIMD; an
            # fma is 2 flops in one issue, so the issue-bound peak is
            # peak x (1 + fma share) / 2
            share = meas.get("fma_share") or 0.0
            r["issue_frac"] = achieved / (FP64_PEAK_TFLOPS * (1.0 + share) / 2.0)
        return r

    a = load(args.matrix)
    n = a.shape[0]
    elapsed, perm, k_ms, st, compile_ms, _ = timed(a)

    # companion densities (north star: 0.2 and 0.5; 0.9 near-dense), same shards / all-reduce / clock
    also = []
    for path in [p for p in args.also.split(",") if p and os.path.abspath(p) != os.path.abspath(args.matrix)]:
        b = load(path)
        nb = b.shape[0]
        e2, perm2, kms2, st2, _, _ = timed(b)
        roof_b = roofline(path, b, args.prep, args.kernel, args.jit, kms2, st2)
        roof_b["traffic"] = hbm_traffic(pmc_record(nb, roof_b["kernel"], roof_b["plan_key"]))
        also.append({"matrix": os.path.basename(path).replace("__", "/"), "n": nb,
                     "density": round(float((b != 0).sum()) / (nb * nb), 4),
                     "value": args.steps * (1 << (nb - 1)) / e2, "unit": "gray-steps/s",
                     "ms_per_step": e2 / args.steps * 1e3, "kernel_ms_avg": kms2,
                     "walk": walk_names[st2["walk_kind"]],
                     "roofline": roof_b,
                     "permanent": perm2})

    # the other BASELINE configs (2, 3, 5), same shards / all-reduce / clock.
    # Configs 2 and 3 with --jit 1 (the compile is outside the timed steps, as
    # for the headline; the CLI's auto mode keeps the AOT walk there because a
    # single run would not repay the compile); config 5 both as the SkipPer
    # kernel itself and as the engine's choice for the -p8 request
    configs = []
    if args.configs:
        fx = os.path.join(ROOT, "tests", "fixtures")
        for label, fname, prep, kernel, jit in (
                ("config 2: -p4 --jit 1 (dense n=32 d=0.5)", "double__32_0.50_0", 0, "dense", 1),
                ("config 3: -p4 -s -r1 --jit 1 (SpaRyser + SortOrder, n=36 d=0.2)", "double__36_0.20_0", 1,
                 "sparse", 1),
                ("config 5: -p8 -s -r2 --jit -1 (the SkipPer kernel + SkipOrder, n=44 d=0.15 int)",
                 "synth44_0.15_int", 2, "skip", -1),
                ("config 5: -p8 -s -r2 (engine's choice after sampling SkipPer's visited fraction)",
                 "synth44_0.15_int", 2, "skip", 0)):
            b = load(os.path.join(fx, fname), prep)
            nb = b.shape[0]
            e2, perm2, kms2, st2, _, k2 = timed(b, kernel, jit, min_seconds=0.25)
            roof2 = roofline(os.path.join(fx, fname), b, prep, kernel, jit, kms2, st2)
            pmc2 = pmc_record(nb, roof2["kernel"], roof2["plan_key"])
            roof2["traffic"] = hbm_traffic(pmc2)
            visited = float(st2["visited_steps"])
            if use_pg:  # the shards' visited counts differ (SkipPer's jumps): sum them
                t = torch.tensor([visited], dtype=torch.float64, device=tdev)
                dist.all_reduce(t)
                visited = float(t.item())
            configs.append({"config": label, "matrix": fname.replace("__", "/"), "n": nb, "steps": k2,
                            "roofline": roof2,
                            "value": k2 * (1 << (nb - 1)) / e2, "unit": "gray-steps/s (nominal)",
                            "ms_per_step": e2 / k2 * 1e3, "kernel_ms_avg": kms2,
                            "walk": walk_names[st2["walk_kind"]],
                            # states evaluated / Gray steps (SkipPer's jumps and the segmented
                            # walk's chunk skip make it < 1); SURVEY 8(d): visited steps/s beside
                            # the nominal rate
                            "visited_frac": visited / float(1 << (nb - 1)),
                            "visited_steps_per_s": k2 * visited / e2,
                            "permanent": perm2})

    # every rank's walk-kernel time (strong-scaling diagnosis: the slowest rank sets the step)
    rank_kms = [k_ms]
    if use_pg:
        t = torch.tensor([k_ms], dtype=torch.float64, device=tdev)
        lst = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        rank_kms = [float(x.item()) for x in lst]

    total_steps = args.steps * (1 << (n - 1))
    value = total_steps / elapsed
    roof = roofline(args.matrix, a, args.prep, args.kernel, args.jit, k_ms, st)
    walk = roof["kernel"]
    pmc = pmc_record(n, walk, roof["plan_key"])
    roof["traffic"] = hbm_traffic(pmc)
    fname = os.path.basename(args.matrix).replace("__", "/")
    density = float((a != 0).sum()) / (n * n)
    rec = {
        "metric": METRIC,
        "value": value,
        "unit": "gray-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"reference corpus matrix {fname} (tests/fixtures/{os.path.basename(args.matrix)})",
        "config": {"workload": f"{args.kernel} Ryser/Gray-code exact permanent (-p4/-p6 path), n={n} "
                               f"d={density:.2f} ({fname}), 2^{n - 1} Gray steps per step",
                   "n": n, "density": round(density, 4), "gray_steps_per_step": 1 << (n - 1),
                   "kernel_request": args.kernel, "preprocessing": args.prep, "jit": args.jit,
                   "walk": walk_names[st["walk_kind"]],
                   "jit_compile_ms": compile_ms,
                   "parallelism": f"dp{world}: contiguous wave-chunk shards + one RCCL all-reduce"},
        "roofline": roof,
        "permanent": perm,
        "kernel_ms_per_rank": rank_kms,
        "plan_keys_per_rank": plan_keys[0],
        "process_group": dist.get_backend() if use_pg else None,
        "densities": also,
        "configs": configs,
    }
    if pmc:  # rocprofv3 HBM evidence for the dominant kernel (committed profile of the same plan)
        alg = pmc.get("algorithmic_bytes_per_launch")
        rec["roofline"].update({
            "traffic_source": pmc["_path"],
            "traffic_definition": "FETCH_SIZE x 2 + WRITE_SIZE per launch (gfx950's FETCH_SIZE counts half the "
                                  "bytes of wide reads: MI355X_MICROARCH.md, HBM / rocprofv3)",
            "algorithmic_bytes_per_launch": alg,
            "traffic_over_algorithmic": roof["traffic"] / alg if alg and roof["traffic"] else None})
    # true error: the corpus files hold 6-digit decimals, whose exact permanent the
    # exact integer path computed once (tests/golden/exact_corpus.json)
    try:
        ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exact_corpus.json")))
        key = os.path.basename(args.matrix)
        if key in ex and args.prep == 0:
            rec["rel_err_vs_exact"] = abs(perm - ex[key]) / abs(ex[key])
            rec["exact_source"] = (
                "tests/golden/exact_corpus.json: this engine's exact integer path (sup_perman_exact: residue walks "
                "+ CRT with a divisibility self-check) on the file's 6-digit decimals; that path matches the "
                "reference's __float128 goldens wherever they exist (n <= 30, tests/test_gpu_exact.py), and at "
                "n = 40 the double-double walk, a different arithmetic, lands within 1 ulp of it "
                "(tests/test_gpu_quad.py::test_gpu_quad_bench_matrix)")
        for d in also:
            k2 = d["matrix"].replace("/", "__")
            if k2 in ex:
                d["rel_err_vs_exact"] = abs(d["permanent"] - ex[k2]) / abs(ex[k2])
        for d in configs:
            k2 = d["matrix"].replace("/", "__")
            if k2 in ex:
                d["rel_err_vs_exact"] = abs(d["permanent"] - ex[k2]) / abs(ex[k2])
    except (OSError, ValueError):
        pass
    # the reference's own fp64 result on the metric matrix (its parallel_perman64,
    # compiled from its sources and run once in the build container): this
    # walk's distance from it, beside both distances from the exact value
    ref_run = reference_metric_run(args.matrix) if args.prep == 0 else None
    if ref_run:
        rec["rel_err_vs_reference_cpu"] = abs(perm - ref_run["permanent"]) / abs(ref_run["permanent"])
        rec["rel_err_reference_cpu_vs_exact"] = ref_run.get("rel_err_vs_exact")
        rec["rel_err_note"] = ("the north star asks for 1e-6 of the CPU reference; at n = 40 the reference's own "
                               "fp64 sum is the inaccurate side (rel_err_reference_cpu_vs_exact), so the walk is "
                               "held to the exact permanent (rel_err_vs_exact) and to within 4x the reference's own "
                               "error of its result (tests/test_gpu_pinned.py)")
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cb_rec, err = cpu_baseline(a, n, args.cpu_seconds, S,
                                   "seg" if st["walk_kind"] == 3 else args.kernel)
        rec["cpu_baseline"] = cb_rec
        rec["rel_err_vs_cpu"] = err
        rec["cpu_baseline_reference_config1"] = cpu_reference_config1(S, cb_rec["cores"])
        rec["cpu_reference_metric_matrix"] = reference_metric_run(args.matrix)
    else:
        rec["cpu_baseline"] = None
    if rank == 0 and world == 1 and args.cold:
        rec["cold_start"] = cold_start(args.matrix)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
