"""Summarise a round-4 rocprofv3 --pmc pass of the walk kernel into a JSON
file under profiles/r4/, keyed by the plan it measured (sup_plan_key for the
same request, computed here with torch's hiprtc as bench.py plans it).

    python tools/pmc_r4.py <pmc dir> <out.json> <matrix> [kernel jit prep]

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
            if walk in r["Kernel_Name"]:
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                k = (r.get("Dispatch_Id"), r["Start_Timestamp"])
                if k not in seen:
                    seen.add(k)
                    ns.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, ns


def main():
    src, dst, matrix = sys.argv[1:4]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "dense"
    jit = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    prep = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    a = S.read_matrix(matrix)[0]
    if prep == 1:
        a = S.sort_order(a)[0]
    elif prep == 2:
        a = S.skip_order(a)[0]
    info = S.plan_info(a, kernel, jit=jit)
    vals, ns = counters(src)
    if not vals:
        sys.exit(f"no counters of {WALK} under {src}")
    out = {"n": int(a.shape[0]), "matrix": os.path.basename(matrix), "kernel": WALK, "request": kernel, "jit": jit,
           "prep": prep, "plan_key": hex(S.plan_key(a, kernel, jit=jit)), "walk": info["kind"],
           "cached": info["cached"], "pair_bits": info["pair_bits"], "model_ops_per_gray_step": info["est_ops_per_step"],
           "kernel_ns": max(ns) if ns else None, "counters": vals,
           "source": f"rocprofv3 --pmc {' '.join(sorted(vals))} --kernel-trace, one launch (bench.py --pmc-child)"}
    if "SQ_WAVE_CYCLES" in vals and vals.get("GRBM_GUI_ACTIVE"):
        cycles = vals["GRBM_GUI_ACTIVE"] / 8.0
        out["waves_per_simd"] = 4.0 * vals["SQ_WAVE_CYCLES"] / (cycles * 1024.0)
        out["clock_ghz"] = cycles / max(ns) if ns else None
    if "SQ_LDS_BANK_CONFLICT" in vals:
        out["lds_bank_conflict_per_lds_inst"] = vals["SQ_LDS_BANK_CONFLICT"] / max(vals.get("SQ_INSTS_LDS", 0.0), 1.0)
    if vals.get("SQC_DCACHE_REQ"):
        out["sqc_dcache_hit"] = vals.get("SQC_DCACHE_HITS", 0.0) / vals["SQC_DCACHE_REQ"]
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in out.items() if k != "counters"}))


if __name__ == "__main__":
    main()
