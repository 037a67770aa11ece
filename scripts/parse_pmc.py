"""Summarise rocprofv3 --pmc CSVs per kernel: mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            short = name.split("(")[0].replace("void ", "")[:60]
            vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
