"""Per-dispatch counter values of one kernel from rocprofv3 --pmc output, in dispatch order.

usage: python scripts/pmc_dispatches.py <pmc_dir> <kernel-name-substring> [counter ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root, sub = sys.argv[1], sys.argv[2]
want = set(sys.argv[3:])
rows = defaultdict(dict)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if sub not in r.get("Kernel_Name", ""):
                continue
            c = r["Counter_Name"]
            if want and c not in want:
                continue
            did = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
            rows[did][c] = rows[did].get(c, 0.0) + float(r["Counter_Value"])
for i, (did, cs) in enumerate(sorted(rows.items())):
    print(i, did, " ".join(f"{c}={v:.6g}" for c, v in sorted(cs.items())))
