#!/usr/bin/env python3
"""Per-kernel PMC summary of a profiles/r0x_qact_pmc.sh run (exp_qact.py prof: the acting forward
at 65,536 rows with dropout, kernels one dispatch at a time under counter collection):
  python profiles/summarize_qact_pmc.py <outdir>     -> JSON on stdout
Per kernel and rows-list variant (grid size): mean counter values per dispatch, the kernel-trace
average duration, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs)
(the round-3 formula), VALU instructions per MFMA, and HBM bytes
(2 x FETCH_SIZE + WRITE_SIZE) x 1024 (MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def main(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("a", "b", "fetch", "write"):
        for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            dur[(short(r["Kernel_Name"]), g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, cs in sorted(vals.items()):
        if not k[0].startswith("k_q"):
            continue
        m = {c: statistics.mean(v) for c, v in cs.items()}
        rec = {"grid": k[1], "counters": {c: round(v, 1) for c, v in m.items()}}
        if k in dur:
            rec["kernel_trace_avg_us"] = round(statistics.mean(dur[k]) / 1e3, 2)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            rec["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
        if "SQ_INSTS_VALU" in m and m.get("SQ_INSTS_MFMA"):
            rec["valu_per_mfma"] = round(m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"], 2)
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            rec["hbm_mb"] = round((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 / 1e6, 1)
        out[f"{k[0]} grid {k[1]}"] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
