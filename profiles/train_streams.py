#!/usr/bin/env python3
"""Per-stream breakdown of the training loop from a rocprofv3 kernel trace
(profiles/train_trace.sh): over the steady-state window of the DDQN training leg (vector steps
`--skip` .. end, delimited by the training k_step launches), each stream's busy time per vector
step (union of its kernels' intervals), and the kernels that make it up.

  python profiles/train_streams.py gpurun_out/trace/kt/run_kernel_trace.csv [--skip 50]
"""
import argparse
import collections
import csv
import json


def union(iv):
    tot, end = 0, None
    for s, e in sorted(iv):
        if end is None or s > end:
            tot += e - s
            end = e
        elif e > end:
            tot += e - end
            end = e
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=50)
    ap.add_argument("--step-kernel", default="k_step<16, false, true, true, false>")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    steps = sorted(int(r["Start_Timestamp"]) for r in rows if a.step_kernel in r["Kernel_Name"])
    if len(steps) <= a.skip + 1:
        raise SystemExit("not enough training steps in the trace")
    t0, t1 = steps[a.skip], steps[-1]
    n = len(steps) - 1 - a.skip
    by_stream = collections.defaultdict(list)
    kern = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 or s >= t1:
            continue
        sid = r["Stream_Id"]
        by_stream[sid].append((s, e))
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if name.startswith("void "):
            name = name[5:]
        name = name.split("(")[0] if "(" in name else name
        kern[sid][name[:80]] += (e - s)
    out = {"vector_steps": n, "us_per_vector_step": (t1 - t0) / n / 1e3,
           "all_streams_busy_us_per_step": union([x for v in by_stream.values() for x in v]) / n / 1e3,
           "streams": {}}
    for sid, iv in sorted(by_stream.items(), key=lambda kv: -union(kv[1])):
        top = sorted(kern[sid].items(), key=lambda kv: -kv[1])[:a.top]
        out["streams"][sid] = {"busy_us_per_step": union(iv) / n / 1e3, "launches_per_step": len(iv) / n,
                               "top_kernels_us_per_step": {k: round(v / n / 1e3, 2) for k, v in top}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
