"""Summarise round-3 rocprofv3 --pmc passes of the walk kernel into
profiles/r3/*.json, keyed by the plan they measured (sup_plan_key, computed
here for the same request: the box and this container run the same image, so
planning and the hiprtc build give the same plan and kernel).

    python tools/pmc_r3.py f64 <pmc dir> <out.json> <matrix> [kernel jit prep]
    python tools/pmc_r3.py hbm <fetch dir> <write dir> <out.json> <matrix> [kernel jit prep]

f64: fp64 flops per Gray step = 64 x (ADD_F64 + MUL_F64 + 2 FMA_F64) per
     launch / 2^(n-1) (rocprofv3's own FP64 FLOPS expression), fp64 and all
     VALU wave-instructions per lane-step, clock and VALU issue share.
hbm: FETCH_SIZE + WRITE_SIZE (KB) per launch of the walk, against its
     algorithmic bytes: one fp64 partial per wave-chunk (2^h of them for the
     plan's layout) + the tables it reads (signed columns, x0).  No gfx950 x2
     FETCH correction: MI355X_MICROARCH.md calibrates it for 16-B/lane
     streaming loads; this kernel reads its tables with scalar loads.
"""
import csv
import glob
import json
import os
import sys

import torch  # noqa: F401,E402  (first, as in bench.py: the kernels and the plan key come from torch's hiprtc)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

WALK = "sup_walk_seg"


def counters(d, walk=WALK):
    vals, ns, calls = {}, [], 0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if walk in r["Kernel_Name"]:
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                ns.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                calls += 1
    return vals, ns


def plan(matrix, kernel, jit, prep):
    a = S.read_matrix(matrix)[0]
    if prep == 1:
        a = S.sort_order(a)[0]
    elif prep == 2:
        a = S.skip_order(a)[0]
    info = S.plan_info(a, kernel, jit=jit)
    return a, info, hex(S.plan_key(a, kernel, jit=jit))


def main():
    mode = sys.argv[1]
    if mode == "f64":
        src, dst, matrix = sys.argv[2:5]
        rest = sys.argv[5:]
    else:
        src, wsrc, dst, matrix = sys.argv[2:6]
        rest = sys.argv[6:]
    kernel = rest[0] if rest else "dense"
    jit = int(rest[1]) if len(rest) > 1 else 1
    prep = int(rest[2]) if len(rest) > 2 else 0
    a, info, key = plan(matrix, kernel, jit, prep)
    n = a.shape[0]
    steps = 1 << (n - 1)
    rec = {"n": n, "kernel": WALK, "matrix": os.path.relpath(matrix, ROOT), "request": {"kernel": kernel, "jit": jit,
                                                                                      "prep": prep},
           "plan_key": key, "plan": {k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in info.items()}}
    if mode == "f64":
        v, ns = counters(src)
        flops = 64.0 * (v["SQ_INSTS_VALU_ADD_F64"] + v["SQ_INSTS_VALU_MUL_F64"] + 2.0 * v["SQ_INSTS_VALU_FMA_F64"])
        f64 = v["SQ_INSTS_VALU_ADD_F64"] + v["SQ_INSTS_VALU_MUL_F64"] + v["SQ_INSTS_VALU_FMA_F64"]
        t = max(ns) * 1e-9
        cyc = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # per XCD
        rec.update({
            "source": f"{os.path.relpath(src, ROOT)}: rocprofv3 --pmc {' '.join(sorted(v))} --kernel-trace, one "
                      "launch of the whole walk (bench.py --steps 1 --warmup 0)",
            "counters": v, "kernel_ns": max(ns),
            "flops_per_gray_step": flops / steps,
            "fp64_insts_per_lane_step": f64 / (steps / 64.0),
            "fma_share": v["SQ_INSTS_VALU_FMA_F64"] / f64,
            "valu_insts_per_lane_step": v.get("SQ_INSTS_VALU", 0.0) / (steps / 64.0),
            "achieved_tflops": flops / t / 1e12,
            "clock_ghz_est": cyc / t / 1e9 if cyc else None,
            # fp64 VALU: one wave-instruction issues per 4 cycles per SIMD
            "fp64_issue_busy_frac": f64 * 4.0 / 1024.0 / cyc if cyc else None,
            "valu_issue_busy_frac": v.get("SQ_INSTS_VALU", 0.0) * 4.0 / 1024.0 / cyc if cyc else None,
        })
    else:
        fv, fns = counters(src)
        wv, _ = counters(wsrc)
        L, m = info["L"], info["m"]
        chunks = 1 << (n - 1 - L - m)
        np8 = (n + 7) // 8 * 8
        algo = chunks * 8 + 2 * (n - 1) * np8 * 8 + np8 * 8
        hbm = (fv["FETCH_SIZE"] + wv["WRITE_SIZE"]) * 1024.0
        rec.update({
            "source": f"{os.path.relpath(src, ROOT)}, {os.path.relpath(wsrc, ROOT)}: rocprofv3 --pmc FETCH_SIZE / "
                      "WRITE_SIZE in separate passes, --kernel-trace, one launch of the whole walk",
            "fetch_size_kb": fv["FETCH_SIZE"], "write_size_kb": wv["WRITE_SIZE"],
            "hbm_bytes_per_launch": int(round(hbm)),
            "algorithmic_bytes_per_launch": algo,
            "hbm_over_algorithmic": hbm / algo,
            "algorithmic_definition": f"2^{n - 1 - L - m} wave-chunk partials x 8 B + signed column table "
                                      f"2(n-1) x {np8} x 8 B + x0",
        })
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(rec, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k not in ("plan",)}, indent=1))


if __name__ == "__main__":
    main()
