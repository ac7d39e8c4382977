#!/usr/bin/env python3
"""Per-dispatch SQ counter sums of k_build / k_mcclendon from a rocprofv3 --pmc csv directory:
one JSON line per dispatch (kernel, grid, counters)."""
import csv
import glob
import json
import sys
from collections import OrderedDict

rows = OrderedDict()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "k_build" not in k and "k_mcclendon" not in k:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        e = rows.setdefault(d, {"kernel": "k_build" if "k_build" in k else "k_mcclendon",
                                "grid": r.get("Grid_Size"), "lds": r.get("LDS_Block_Size",
                                                                        r.get("Lds_Block_Size"))})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for d, e in rows.items():
    e["dispatch"] = d
    print(json.dumps(e))
