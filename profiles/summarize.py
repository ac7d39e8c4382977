#!/usr/bin/env python3
"""Turn rocprofv3 outputs under gpurun_out/ into the committed summaries under profiles/.

  python profiles/summarize.py <round_tag> <kernel-trace dir> <FETCH_SIZE dir> <WRITE_SIZE dir> \
      --envs 65536 --dim 81 --mode window|bits

Writes profiles/<tag>_kernel_stats.csv (copy of rocprofv3 --stats) and the <mode> record of
profiles/pmc_k_step.json (stamped with the hash of k_step's sources: bench.py uses a record only
while the sources are unchanged):
per-launch HBM bytes of k_step = (2 x FETCH_SIZE + WRITE_SIZE) x 1024, the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE tallies 64 B per L2-miss request, and every request is a
128-B line: calibrated for k_step's own read shapes — u32 gathers, 64-B coalesced state loads,
15-row window gathers — in profiles/r06x/fetch_calibration.json, so the doubled figure is the
line traffic of k_step's reads).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def counter(d, name, kernel_sub):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if r["Counter_Name"] == name and kernel_sub in r["Kernel_Name"]]
    return statistics.mean(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("kt")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=81)
    ap.add_argument("--kernel", default="k_step<16, false, true, true, true>")
    ap.add_argument("--mode", default="window", choices=["window", "bits"])
    a = ap.parse_args()
    from bench import kstep_source_sha
    stats = glob.glob(os.path.join(a.kt, "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(HERE, f"{a.tag}_kernel_stats.csv"))
    avg_ns = [float(r["AverageNs"]) for r in csv.DictReader(open(stats)) if a.kernel in r["Name"]][0]
    fetch_kb, nf = counter(a.fetch, "FETCH_SIZE", a.kernel)
    write_kb, nw = counter(a.write, "WRITE_SIZE", a.kernel)
    out = {
        "kernel": a.kernel, "envs": a.envs, "dim": a.dim, "mode": a.mode, "tag": a.tag,
        "source_sha": kstep_source_sha(),
        "rocprof_avg_ns": avg_ns,
        "FETCH_SIZE_kb_per_launch": fetch_kb, "WRITE_SIZE_kb_per_launch": write_kb,
        "launches_sampled": [nf, nw],
        "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024,
        "hbm_bytes_per_launch_uncorrected": (fetch_kb + write_kb) * 1024,
        "note": "traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md §HBM; "
                "separate --pmc passes for FETCH_SIZE and WRITE_SIZE",
    }
    path = os.path.join(HERE, "pmc_k_step.json")
    allrec = {}
    if os.path.exists(path):
        with open(path) as f:
            allrec = json.load(f)
        if "kernel" in allrec:  # the round-2 single-record layout
            allrec = {}
    allrec[a.mode] = out
    with open(path, "w") as f:
        json.dump(allrec, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
