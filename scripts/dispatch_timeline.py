"""Timeline of consecutive kernel dispatches from a rocprofv3 --kernel-trace CSV: for a window of
dispatches, each kernel's duration and the gap since the previous dispatch ended — where a
launch-bound sequence (one off-policy learn() iteration) spends its time.

usage: python scripts/dispatch_timeline.py <trace_dir> <anchor-substring> <occurrence> <before> <count>
  the window starts `before` dispatches ahead of the occurrence-th dispatch whose name contains
  the anchor (e.g. "ddpg_td_kernel" 10 4 40: one DDPG learn() after warm-up)"""
import csv
import glob
import os
import sys

root, anchor, occ, before, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
rows = []
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
hits = [i for i, r in enumerate(rows) if anchor in r[2]]
if len(hits) <= occ:
    sys.exit(f"only {len(hits)} dispatches match {anchor!r}")
first = max(hits[occ] - before, 0)
win = rows[first:first + count]
tot_k = tot_g = 0
prev_end = None
for s, e, name in win:
    gap = 0 if prev_end is None else s - prev_end
    tot_k += e - s
    tot_g += max(gap, 0)
    print(f"{(e - s) / 1e3:9.2f} us  gap {gap / 1e3:7.2f} us  {name[:100]}")
    prev_end = e
if win:
    span = win[-1][1] - win[0][0]
    print(f"{len(win)} dispatches: kernels {tot_k / 1e3:.1f} us, gaps {tot_g / 1e3:.1f} us, "
          f"span {span / 1e3:.1f} us")
