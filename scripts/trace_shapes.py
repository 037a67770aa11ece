"""Per launch shape durations from a rocprofv3 --kernel-trace CSV: kernels matching REGEX grouped
by (name, grid, workgroup, LDS) with dispatch count, mean / min duration (us) and total ms.
python3 scripts/trace_shapes.py <trace_dir> REGEX"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root, pat = sys.argv[1], re.compile(sys.argv[2])
d = defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"]
            if not pat.search(name):
                continue
            key = (name.split("(")[0].replace("void ", "")[:90], int(row["Grid_Size_X"]) * int(row.get("Grid_Size_Y", 1) or 1),
                   int(row["Workgroup_Size_X"]), int(row.get("LDS_Block_Size", row.get("Lds_Size", 0)) or 0))
            d[key].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
tot = 0.0
for key, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"{key[0]} grid={key[1]} wg={key[2]} lds={key[3]} n={len(v)} mean_us={sum(v) / len(v):.2f} "
          f"min_us={min(v):.2f} total_ms={sum(v) / 1e3:.3f}")
print(f"# total {tot / 1e3:.3f} ms")
