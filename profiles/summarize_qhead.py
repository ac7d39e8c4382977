#!/usr/bin/env python3
"""Per-kernel MFMA summary of profiles/pmc_qhead.sh's outputs -> profiles/<tag>_qhead_mfma.json.

For every kernel of the act / update runs: calls, rocprofv3 average duration, MFMA FLOPs per
launch (SQ_INSTS_VALU_MFMA_MOPS_{BF16,F32} x 512, the derived MfmaFlops* of rocprofiler-sdk),
the rate they imply over the kernel-trace average, and MfmaUtil (rocprofiler-sdk
derived_counters.xml, gfx94x formula — ROCm 7.2 has no gfx950 section — with GRBM_GUI_ACTIVE per
XCD). Peaks: bf16 2.5 PFLOP/s, f32 matrix 157.3 TFLOP/s dense
(MI355X_MICROARCH.md).
  python profiles/summarize_qhead.py <tag> <outdir>"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PEAK = {"bf16": 2500.0, "f32": 157.3}
XCDS = 8


def main(tag, d):
    # the kernel-trace run and the counter run issue the same dispatch sequence: pair the i-th
    # dispatch of each (kernel, grid) of one with the i-th of the other
    tr = glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True)[0]
    seq = collections.defaultdict(list)
    for r in csv.DictReader(open(tr)):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        seq[(r["Kernel_Name"], g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    f = glob.glob(os.path.join(d, "mfma", "**", "*counter_collection.csv"), recursive=True)[0]
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        per[int(r["Dispatch_Id"])]["k"] = (r["Kernel_Name"], int(r["Grid_Size"]))
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    idx = collections.Counter()
    acc = collections.defaultdict(list)
    for did in sorted(per):
        c = per[did]
        k = c["k"]
        i = idx[k]
        idx[k] += 1
        if i >= len(seq.get(k, [])):
            continue
        bf = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) * 512
        f32 = c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0) * 512
        if bf + f32 == 0:
            continue
        acc[(k[0], k[1], round(bf + f32))].append(
            (seq[k][i], bf, f32, c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), c.get("GRBM_GUI_ACTIVE", 1)))
    rows = []
    for (name, grid, _), v in acc.items():
        ns = statistics.mean(x[0] for x in v)
        bf = statistics.mean(x[1] for x in v)
        f32 = statistics.mean(x[2] for x in v)
        busy = statistics.mean(x[3] for x in v)
        gui = statistics.mean(x[4] for x in v) / XCDS
        dt = "bf16" if bf >= f32 else "f32"
        fl = bf + f32
        rows.append({"kernel": name[:160], "grid": grid, "calls": len(v), "avg_us": round(ns / 1e3, 2),
                     "mfma_dtype": dt, "mfma_gflop_per_launch": round(fl / 1e9, 3),
                     "tflops": round(fl / ns / 1e3, 1),
                     "frac_of_dense_peak": round(fl / ns / 1e3 / PEAK[dt], 3),
                     "MfmaUtil_pct": round(100 * busy / (gui * 256 * 4), 1),
                     "clock_ghz_under_pmc": round(gui / ns, 2)})
    rows.sort(key=lambda r: -r["calls"] * r["avg_us"])
    out = {"source": "profiles/pmc_qhead.sh (exp_qhead.py act + update)",
           "note": "MfmaUtil = 100 x SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 "
                   "SIMDs): GRBM_GUI_ACTIVE sums the 8 XCDs (it reads 8 x duration x clock); the "
                   "busy cycles are emulated from the MOPS count at the dtype's peak rate, so "
                   "MfmaUtil is the fraction of dense peak at the clock the kernel ran at",
           "kernels": rows}
    with open(os.path.join(HERE, f"{tag}_qhead_mfma.json"), "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
