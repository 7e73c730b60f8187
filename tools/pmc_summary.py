"""Summarise a gpu_session.sh 'pmc' + 'prof' run into profiles/<round>/pmc_n<n>.json.

    python tools/pmc_summary.py gpurun_out/<tag> profiles/r1/pmc_n40.json [n]

Reads the four separate rocprofv3 --pmc passes (pmc_fetch, pmc_write, pmc_sq,
pmc_lds; each --kernel-trace only, bench.py --steps 1) and the --stats pass
(prof), keeps the walk kernel's rows, and derives:
  * HBM bytes per launch = (FETCH_SIZE + WRITE_SIZE) KB x 1024.  No gfx950
    x2 correction: MI355X_MICROARCH.md calibrates it for 16-B/lane streaming
    global loads; this kernel reads its 25.6 KB table with scalar loads and
    writes 8-B partials;
  * VALU wave-instructions per lane-step = SQ_INSTS_VALU / (2^(n-1) / 64);
  * clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time; VALU busy = fp64 VALU
    issue cycles (4 per wave-instruction) per SIMD / active cycles;
  * achieved occupancy = resident waves per SIMD averaged over the kernel =
    4 x SQ_WAVE_CYCLES (quad-cycles) / 1024 SIMDs / cycles, and its share of
    the 8 wave slots of a gfx950 SIMD.
"""
import csv
import glob
import json
import os
import sys


def rows(path, kernel_sub="walk_"):
    out = {}
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel_sub in r["Kernel_Name"]:
                out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                out.setdefault("_kernel", [r["Kernel_Name"]])
                out.setdefault("_ns", []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    fetch, write = rows(os.path.join(src, "pmc_fetch")), rows(os.path.join(src, "pmc_write"))
    sq, lds = rows(os.path.join(src, "pmc_sq")), rows(os.path.join(src, "pmc_lds"))
    stats = {}
    for f in glob.glob(os.path.join(src, "prof", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if "walk_" in r["Name"]:
                stats = {"kernel": r["Name"], "calls": int(r["Calls"]), "average_ns": float(r["AverageNs"])}
    first = lambda d, k: d[k][0] if k in d else None  # noqa: E731
    fk, wk = first(fetch, "FETCH_SIZE"), first(write, "WRITE_SIZE")
    chunks = 1 << (n - 1 - 6 - min(max(min(n - 7, 10), n - 7 - 20), 31))
    rec = {
        "n": n,
        "kernel": (fetch.get("_kernel") or [stats.get("kernel")])[0],
        "source": f"{src}: rocprofv3 --pmc in separate passes (FETCH_SIZE; WRITE_SIZE; SQ_*; LDS), --kernel-trace, "
                  "bench.py --steps 1 --warmup 0; --kernel-trace --stats pass for durations",
        "fetch_size_kb": fk, "write_size_kb": wk,
        "hbm_bytes_per_launch": int(round((fk + wk) * 1024)) if fk is not None and wk is not None else None,
        "algorithmic_bytes_per_launch": chunks * 8 + 2 * (n - 1) * ((n + 7) // 8 * 8) * 8,
        "kernel_stats": stats,
    }
    sqd = {k: first(sq, k) for k in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES",
                                     "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT")}
    sqd.update({k: first(lds, k) for k in ("SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU",
                                           "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY")})
    if sqd.get("SQ_INSTS_VALU") and sq.get("_ns"):
        wave_steps = (1 << (n - 1)) / 64.0
        sqd["valu_insts_per_lane_step"] = round(sqd["SQ_INSTS_VALU"] / wave_steps, 2)
        t = sq["_ns"][0] * 1e-9
        if sqd.get("GRBM_GUI_ACTIVE"):
            cyc = sqd["GRBM_GUI_ACTIVE"] / 8.0
            sqd["clock_ghz_est"] = round(cyc / t / 1e9, 3)
            sqd["valu_busy_frac_est"] = round(sqd["SQ_INSTS_VALU"] * 4.0 / 1024.0 / cyc, 3)
            if sqd.get("SQ_WAVE_CYCLES"):
                # achieved occupancy: SQ_WAVE_CYCLES counts quad-cycles of resident waves
                # (MI355X_MICROARCH.md), over 1024 SIMDs x the kernel's cycles
                occ = sqd["SQ_WAVE_CYCLES"] * 4.0 / 1024.0 / cyc
                sqd["achieved_waves_per_simd"] = round(occ, 3)
                sqd["achieved_occupancy_frac"] = round(occ / 8.0, 4)  # of the 8 wave slots per SIMD
    rec["sq"] = sqd
    rec["notes"] = ("FETCH/WRITE_SIZE in KB per dispatch, no gfx950 x2 correction (scalar-load table, 8-B partial "
                    "stores). Algorithmic bytes = wave-chunk partials x 8 B + the signed column table. The walk is "
                    "fp64-VALU-bound; HBM traffic is negligible.")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(rec, open(dst, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
