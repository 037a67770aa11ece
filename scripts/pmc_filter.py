"""Aggregate one rocprofv3 counter-collection pass on the box (gpurun_out stays small): the rows
of kernels matching REGEX, averaged per (kernel, grid, workgroup, LDS, counter), into one small
CSV with a count column N (scripts/parse_pmc.py weights by it).
python3 scripts/pmc_filter.py <pass_dir> REGEX <out.csv>"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root, pat, out = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3]
agg = defaultdict(lambda: [0.0, 0])
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            if not pat.search(name):
                continue
            key = (name, row["Grid_Size"], row["Workgroup_Size"], row["LDS_Block_Size"], row["Counter_Name"])
            a = agg[key]
            a[0] += float(row["Counter_Value"])
            a[1] += 1
with open(out, "w", newline="") as fo:
    w = csv.writer(fo)
    w.writerow(["Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Counter_Name",
                "Counter_Value", "N"])
    for (name, gsz, wg, lds, c), (s, n) in sorted(agg.items()):
        w.writerow([name, gsz, wg, lds, c, s / n, n])
