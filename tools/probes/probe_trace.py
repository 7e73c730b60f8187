"""Where a segmented walk's launch spends its time, from per-wave stamps
(SUP_JIT_TRACE: entry / exit in realtime (100 MHz) and shader-clock ticks,
chunks walked, shader cycles of the chunk starts).

Per matrix: kernel time untraced and traced (the stamps cost a few
instructions per chunk), then for the traced launch:
  ramp   = last wave entry - first wave entry
  tail   = last wave exit - median wave exit
  idle   = 1 - mean(wave exit - wave entry) / launch span  (wave slots empty)
  start  = chunk-start cycles / wave cycles                (start states, copies, trees)

    python3 tools/probes/probe_trace.py [matrix[:prep[:kernel]] ...] [--walk-log2 m ...]
"""
import argparse
import os
import statistics
import sys
import tempfile

import torch  # noqa: F401  (torch's hiprtc, as bench.py)

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402


def load(spec):
    name, prep, kernel = (spec.split(":") + ["0", "dense"])[:3]
    a = S.read_matrix(os.path.join(ROOT, "tests", "fixtures", name))[0]
    if prep == "1":
        a = S.sort_order(a)[0]
    elif prep == "2":
        a = S.skip_order(a)[0]
    return name, a, kernel


def kernel_ms(a, kernel, wl, reps=7):
    S.perman_shard(a, 0, 1, kernel=kernel, jit=1, walk_log2=wl)
    ks, v = [], None
    for _ in range(reps):
        v, st = S.perman_shard(a, 0, 1, kernel=kernel, jit=1, walk_log2=wl, return_stats=True)
        ks.append(st["kernel_ms"])
    return statistics.median(ks), v, st


def parse(path):
    launches, cur = [], None
    for ln in open(path):
        if ln.startswith("#"):
            kv = ln.split()[2:]
            cur = {"meta": {kv[i]: kv[i + 1] for i in range(0, len(kv) - 1, 2)}, "w": []}
            launches.append(cur)
        elif ln.strip():
            f = [int(x) for x in ln.split()]
            if f[1] or f[2]:
                cur["w"].append(f[1:])
    return launches


def summarise(L):
    w = L["w"]
    r0 = min(x[0] for x in w)
    ent = sorted(x[0] - r0 for x in w)
    ext = sorted(x[1] - r0 for x in w)
    span = ext[-1]
    busy = sum(x[1] - x[0] for x in w) / len(w)
    cyc = sum(x[3] - x[2] for x in w)
    start = sum(x[5] for x in w)
    ch = [x[4] for x in w]
    ghz = cyc / sum(x[1] - x[0] for x in w) / 10.0  # shader ticks per 10 ns
    return (f"waves {len(w)} span {span / 100:.1f} us  ramp {ent[-1] / 100:.1f} us (median entry "
            f"{ent[len(ent) // 2] / 100:.1f})  tail {(ext[-1] - ext[len(ext) // 2]) / 100:.1f} us (first exit "
            f"{ext[0] / 100:.1f}, median {ext[len(ext) // 2] / 100:.1f})  idle {1 - busy / span:.3f}  "
            f"start {start / cyc:.3f}  chunks/wave {min(ch)}-{max(ch)} (mean {statistics.mean(ch):.2f})  "
            f"clock {ghz:.2f} GHz  [{L['meta']}]")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=["double__32_0.50_0", "double__36_0.20_0:1:sparse",
                                                 "double__40_0.50_0"])
    ap.add_argument("--walk-log2", type=int, nargs="*", default=[0])
    args = ap.parse_args()
    for spec in args.cases:
        name, a, kernel = load(spec)
        for wl in args.walk_log2:
            os.environ.pop("SUP_JIT_TRACE", None)
            info = S.plan_info(a, kernel, jit=1, walk_log2=wl)
            k0, v0, st = kernel_ms(a, kernel, wl)
            path = tempfile.mktemp(prefix="sup_trace_")
            os.environ["SUP_JIT_TRACE"] = path
            k1, v1, _ = kernel_ms(a, kernel, wl, reps=3)
            os.environ.pop("SUP_JIT_TRACE")
            launches = parse(path)
            os.unlink(path)
            print(f"== {name} {kernel} m={info['m']} cc={info.get('cached')} b={info.get('pair_bits')} "
                  f"ops {info['est_ops_per_step']:.2f}: kernel {k0:.4f} ms untraced, {k1:.4f} traced; "
                  f"same sum {v0 == v1}; grid {st['grid']}", flush=True)
            for L in launches[-2:]:
                print("   " + summarise(L), flush=True)


if __name__ == "__main__":
    main()
