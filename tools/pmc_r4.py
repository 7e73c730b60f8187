"""Summarise a round-4 rocprofv3 --pmc pass of the walk kernel into a JSON
file under profiles/r4/, keyed by the plan it measured (sup_plan_key for the
same request, computed here with torch's hiprtc as bench.py plans it).

    python tools/pmc_r4.py <out.json> <matrix> <pmc dir> [<pmc dir> ...] [--kernel K --jit J --prep P --walk NAME]
    (default request: dense, jit 1, no prep, kernel sup_walk_seg)

Every counter of the walk kernel's dispatch is kept (summed over the
dispatches of the pass, which is one launch: bench.py --pmc-child), with
these derived figures where their counters are present:
  waves_per_simd   achieved occupancy = 4 SQ_WAVE_CYCLES (quad-cycles -> cycles,
                   summed over every wave) / (cycles the kernel ran x 1024 SIMDs);
                   cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs;
                   MI355X_MICROARCH.md, DVFS give-back)
  lds_bank_conflict_per_lds_inst   SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS
  sqc_dcache_hit   SQC_DCACHE_HITS / SQC_DCACHE_REQ (scalar data cache)
"""
import csv
import glob
import json
import os
import sys

import torch  # noqa: F401  (first, as in bench.py: the kernels and the plan key come from torch's hiprtc)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import superman_amd as S  # noqa: E402

WALK = "sup_walk_seg"


def counters(d, walk=WALK):
    vals, ns = {}, []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            if walk in r["Kernel_Name"] or (walk.endswith(">") and walk[:-1] + "," in r["Kernel_Name"]):
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                k = (r.get("Dispatch_Id"), r["Start_Timestamp"])
                if k not in seen:
                    seen.add(k)
                    ns.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, ns


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("dst")
    ap.add_argument("matrix")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="dense")
    ap.add_argument("--jit", type=int, default=1)
    ap.add_argument("--prep", type=int, default=0)
    ap.add_argument("--walk", default=WALK, help="kernel name filter (sup_walk_seg, sup::walk_skip<44>, ...)")
    ap.add_argument("--visited", action="store_true", help="the walk also stores a visited count per wave-chunk")
    args = ap.parse_args()
    dst, matrix, dirs = args.dst, args.matrix, args.dirs
    kernel, jit, prep, walk = args.kernel, args.jit, args.prep, args.walk
    a = S.read_matrix(matrix)[0]
    if prep == 1:
        a = S.sort_order(a)[0]
    elif prep == 2:
        a = S.skip_order(a)[0]
    info = S.plan_info(a, kernel, jit=jit)
    vals, ns = {}, []
    for d in dirs:  # one pass per directory (counters that cannot share a pass)
        v, t = counters(d, walk)
        vals.update(v)
        ns += t
    if not vals:
        sys.exit(f"no counters of {walk} under {dirs}")
    out = {"n": int(a.shape[0]), "matrix": os.path.basename(matrix), "kernel": walk, "request": kernel, "jit": jit,
           "prep": prep, "plan_key": hex(S.plan_key(a, kernel, jit=jit)), "walk": info["kind"],
           "cached": info["cached"], "pair_bits": info["pair_bits"], "model_ops_per_gray_step": info["est_ops_per_step"],
           "kernel_ns_per_pass": ns, "counters": vals,
           "source": "rocprofv3 --pmc <counters> --kernel-trace, one launch per pass (bench.py --pmc-child): "
                     + ", ".join(os.path.relpath(d) for d in dirs)}
    if "SQ_WAVE_CYCLES" in vals and vals.get("GRBM_GUI_ACTIVE"):
        cycles = vals["GRBM_GUI_ACTIVE"] / 8.0
        out["waves_per_simd"] = 4.0 * vals["SQ_WAVE_CYCLES"] / (cycles * 1024.0)
    if "MeanOccupancyPerCU" in vals:
        out["mean_occupancy_waves_per_cu"] = vals["MeanOccupancyPerCU"]
    if "SQ_LDS_BANK_CONFLICT" in vals:
        out["lds_bank_conflict_per_lds_inst"] = vals["SQ_LDS_BANK_CONFLICT"] / max(vals.get("SQ_INSTS_LDS", 0.0), 1.0)
    if vals.get("SQC_DCACHE_REQ"):
        out["sqc_dcache_hit"] = vals.get("SQC_DCACHE_HITS", 0.0) / vals["SQC_DCACHE_REQ"]
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        # KB per launch; one fp64 partial per wave-chunk + the tables it reads
        chunks = 1 << (a.shape[0] - 1 - info["L"] - info["m"])
        np_ = (a.shape[0] + 7) // 8 * 8
        alg = chunks * 8 + 2 * (a.shape[0] - 1) * np_ * 8 + np_ * 8
        if args.visited:  # SkipPer / the chunk skip: one 4-byte visited count per wave-chunk
            alg += chunks * 4
        # gfx950's FETCH_SIZE counts half the bytes of a wide coalesced read
        # (MI355X_MICROARCH.md, HBM / rocprofv3): doubled here (round 5 on)
        hbm = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
        out.update({"hbm_bytes_per_launch": hbm, "fetch_bytes": vals["FETCH_SIZE"] * 1024.0,
                    "write_bytes": vals["WRITE_SIZE"] * 1024.0, "algorithmic_bytes_per_launch": alg,
                    "hbm_over_algorithmic": hbm / alg, "fetch_size_doubled": True})
    if all(k in vals for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")):
        steps = float(1 << (a.shape[0] - 1))
        f64 = vals["SQ_INSTS_VALU_ADD_F64"] + vals["SQ_INSTS_VALU_MUL_F64"] + vals["SQ_INSTS_VALU_FMA_F64"]
        out.update({"flops_per_gray_step": 64.0 * (f64 + vals["SQ_INSTS_VALU_FMA_F64"]) / steps,
                    "fp64_insts_per_lane_step": f64 / (steps / 64.0),
                    "fma_share": vals["SQ_INSTS_VALU_FMA_F64"] / f64})
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in out.items() if k not in ("counters", "kernel_ns_per_pass")}))


if __name__ == "__main__":
    main()
