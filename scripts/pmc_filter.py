"""Keep only the rows of kernels matching REGEX from a rocprofv3 counter-collection CSV tree
(one pass), into one small CSV: python3 scripts/pmc_filter.py <pass_dir> REGEX <out.csv>"""
import csv
import glob
import os
import re
import sys

root, pat, out = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3]
w = None
with open(out, "w", newline="") as fo:
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            r = csv.DictReader(fh)
            for row in r:
                if not pat.search(row.get("Kernel_Name", "")):
                    continue
                if w is None:
                    w = csv.DictWriter(fo, fieldnames=r.fieldnames)
                    w.writeheader()
                w.writerow(row)
