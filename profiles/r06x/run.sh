#!/bin/bash
# round 6: FETCH_SIZE calibration for k_step's read shapes (profiles/ubench_fetch.hip)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 120 ./profiles/_bin/ubench_fetch > $O/plain.log 2>&1 || { cat $O/plain.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- ./profiles/_bin/ubench_fetch > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -f csv -d $O/rdreq -o run -- ./profiles/_bin/ubench_fetch > $O/rdreq.log 2>&1 || { tail -5 $O/rdreq.log; exit 1; }
cat $O/plain.log
python3 - <<'PY'
import csv, glob, collections, re, json
O = "gpurun_out/r06x"
for d in ("fetch", "rdreq"):
    f = glob.glob(f"{O}/{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if m:
            acc[(m.group(1), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(json.dumps({"kernel": k, "counter": c, "mean": sum(v) / len(v), "n": len(v)}))
PY
