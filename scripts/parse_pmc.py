"""Summarise rocprofv3 --pmc CSVs per kernel: mean counter value per dispatch.

python3 scripts/parse_pmc.py <dir> [--by-grid REGEX]
  --by-grid REGEX   also list the kernels whose name matches REGEX per (template, grid size,
                    workgroup size, LDS) shape — e.g. the dense GEMM's SOI and UGV-OA launches —
                    with derived ratios (MFMA busy per SIMD-cycle, VALU:MFMA, LDS conflict share)
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
by_grid = None
if "--by-grid" in sys.argv:
    by_grid = re.compile(sys.argv[sys.argv.index("--by-grid") + 1])
vals = defaultdict(lambda: defaultdict(list))
shapes = defaultdict(lambda: defaultdict(list))
files = glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)
files += glob.glob(os.path.join(root, "p*_filtered.csv"))   # scripts/pmc_filter.py output
for f in files:
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            short = name.split("(")[0].replace("void ", "")[:60]
            v = float(row["Counter_Value"])
            reps = int(row.get("N") or 1)   # aggregated rows (scripts/pmc_filter.py): mean x N
            vals[short][row["Counter_Name"]].extend([v] * reps)
            if by_grid and by_grid.search(name):
                key = (name.split("(")[0].replace("void ", "")[:90], int(row["Grid_Size"]),
                       int(row["Workgroup_Size"]), int(row["LDS_Block_Size"]))
                shapes[key][row["Counter_Name"]].extend([v] * reps)
for k, cs in sorted(vals.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")


def mean(cs, c):
    v = cs.get(c)
    return sum(v) / len(v) if v else None


if by_grid:
    print("\n# per launch shape (name, grid threads, workgroup, LDS bytes); ratios: mfma_busy = "
          "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), valu_per_mfma = "
          "SQ_INSTS_VALU / SQ_INSTS_MFMA, lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, "
          "hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (kB, gfx950 FETCH_SIZE halving)")
    for key, cs in sorted(shapes.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        n = max(len(v) for v in cs.values())
        busy, gui = mean(cs, "SQ_VALU_MFMA_BUSY_CYCLES"), mean(cs, "GRBM_GUI_ACTIVE")
        valu, mfma = mean(cs, "SQ_INSTS_VALU"), mean(cs, "SQ_INSTS_MFMA")
        conf, idx = mean(cs, "SQ_LDS_BANK_CONFLICT"), mean(cs, "SQ_LDS_IDX_ACTIVE")
        fs, ws = mean(cs, "FETCH_SIZE"), mean(cs, "WRITE_SIZE")
        out = [f"{key[0]} grid={key[1]} wg={key[2]} lds={key[3]} dispatches/pass~{n}"]
        if busy is not None and gui:
            out.append(f"mfma_busy={busy / (gui / 8 * 1024):.3f}")
        if valu is not None and mfma:
            out.append(f"valu_per_mfma={valu / mfma:.2f} mfma_insts={mfma:.4g}")
        if conf is not None and idx:
            out.append(f"lds_conflict={conf / idx:.3f}")
        if fs is not None and ws is not None:
            out.append(f"hbm_kB={(2 * fs + ws):.6g}")
        if gui:
            out.append(f"gui_active={gui:.4g}")
        print("  " + " ".join(out))
