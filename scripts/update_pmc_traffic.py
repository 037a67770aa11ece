"""Fold a scripts/gpu_pmc.sh run into profiles/pmc_traffic.json (the `traffic` bench.py reports).

Reads gpurun_out/<TAG>/p*/**/*counter_collection.csv, averages FETCH_SIZE and WRITE_SIZE per
dispatch of each rollout kernel and stores hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) *
1024 (gfx950: FETCH_SIZE counts half of a wide coalesced read stream, MI355X_MICROARCH.md §HBM).
Usage: python scripts/update_pmc_traffic.py gpurun_out/<TAG> profiles/<round>/<summary>.txt [out.json]
(out.json: write the updated file there instead of profiles/pmc_traffic.json, e.g. on the GPU box)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {  # workload -> (kernel name prefix, envs per GPU, T, algorithmic bytes per launch)
    "cartpole_ppo2_rollout": ("rlp::rollout_sp_kernel<1, 256, 2, 8, 2>", 65536, 128,
                              65536 * 128 * 55 + 65536 * (2 * 5 * 8 + 2)),
    "uav_ppo2_rollout": ("rlp::rollout_sp_kernel<6, 256, 2, 4, 1>", 32768, 64,
                         # obs / obs_next 2 x 6 f32 + action / logp 2 x 3 f32 + reward, value,
                         # value_next + done / success / flag per transition; f64 state 22 x 8 r+w
                         32768 * 64 * (48 + 24 + 12 + 3) + 32768 * (2 * 22 * 8 + 2)),
}


# bench.py hbm_legs kernels -> the kernel-name prefixes whose FETCH / WRITE add up to one launch
# (round 6: the learn side's launches; bench.py checks these prefixes against its labels)
HBM_KERNELS = {
    "gae": ["rlp::gae_kernel<1>"],
    "reward_norm": ["rlp::reward_stats_kernel", "rlp::reward_merge_kernel"],
    "adv_normalize": ["rlp::adv_stats_merge_kernel", "rlp::adv_norm_kernel"],
    "reward_norm_stored": ["rlp::reward_stats_kernel", "rlp::reward_merge_kernel",
                           "rlp::reward_apply_kernel"],
    "env_step_soi": ["rlp::env_step_kernel<3>"],
    "env_step_ugv": ["rlp::env_step_kernel<4>"],
    "env_step_uav": ["rlp::env_step_kernel<6>"],
}


def main(run_dir, profile, out_path=None):
    # per kernel name, the dispatches of its largest grid only (the bench's hbm_legs shapes; the
    # same kernel also runs at smaller shapes in other legs, which must not be averaged in)
    vals = defaultdict(lambda: defaultdict(list))
    grid = {}
    rows = []
    for f in glob.glob(os.path.join(run_dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "").replace("void ", "")
                g = int(row.get("Grid_Size", 0) or 0)
                grid[name] = max(grid.get(name, 0), g)
                rows.append((name, g, row["Counter_Name"], float(row["Counter_Value"])))
    for name, g, c, v in rows:
        if g == grid[name]:
            vals[name][c].append(v)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(path) as f:
        d = json.load(f)
    for wl, (prefix, n, T, alg) in WORKLOADS.items():
        hit = [k for k in vals if k.startswith(prefix)]
        if not hit or "FETCH_SIZE" not in vals[hit[0]] or "WRITE_SIZE" not in vals[hit[0]]:
            print(f"{wl}: no FETCH_SIZE/WRITE_SIZE for {prefix}")
            continue
        c = vals[hit[0]]
        fetch = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        e = d.get(wl, {})
        e.update({"envs_per_gpu": n, "T": T, "FETCH_SIZE_KB": round(fetch, 1),
                  "WRITE_SIZE_KB": round(write, 1),
                  "hbm_bytes_per_launch": int((2 * fetch + write) * 1024),
                  "algorithmic_bytes_per_launch": alg, "profile": profile, "kernel": prefix})
        d[wl] = e
        print(f"{wl}: {e['hbm_bytes_per_launch'] / 1e6:.1f} MB per launch vs {alg / 1e6:.1f} MB algorithmic")
    hk = d.setdefault("hbm_kernels", {})
    for leg, prefixes in HBM_KERNELS.items():
        fetch = write = 0.0
        found = True
        for pre in prefixes:
            hit = [k for k in vals if k.startswith(pre) and "FETCH_SIZE" in vals[k] and "WRITE_SIZE" in vals[k]]
            if not hit:
                found = False
                break
            c = vals[hit[0]]
            fetch += sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
            write += sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        if not found:
            print(f"{leg}: no FETCH_SIZE/WRITE_SIZE")
            continue
        # FETCH_SIZE doubled as for the rollout (128-B requests tallied at 64 B,
        # MI355X_MICROARCH.md §HBM)
        hk[leg] = {"kernels": prefixes, "FETCH_SIZE_KB": round(fetch, 1), "WRITE_SIZE_KB": round(write, 1),
                   "hbm_bytes_per_launch": int((2 * fetch + write) * 1024), "profile": profile}
        print(f"{leg}: {hk[leg]['hbm_bytes_per_launch'] / 1e6:.1f} MB per launch")
    with open(out_path or path, "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
