"""Recompute bench.py's roofline fractions from a rocprofv3 kernel trace of the SAME run.

usage: python scripts/trace_check.py <trace_dir> <bench_log> [--warmup W --steps K] > summary.txt

The bench times its K rollout launches with HIP events after W warm-up iterations; the CartPole
rollout kernel's dispatches [W, W+K) in the trace are exactly those launches (the exact-f32 leg
and the UAV leg launch other template instances; the e2e leg's rollouts come after them). The
UAV leg runs 2 warm-up + 5 timed launches. For every kernel the bench prices, this prints the
trace's mean duration over the timed dispatches, the bench's HIP-event mean of the same run, the
two fractions and their ratio; plus per-kernel stats of the update kernels (all dispatches).
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KINDS = {"cartpole": 1, "uav": 6}


def targs(name):
    return [a.strip() for a in name[name.find("<") + 1:name.find(">")].split(",")]


def matches(trace_name, bench_kernel, kind):
    base = bench_kernel.split("<")[0]
    trace_name = trace_name.replace("void ", "", 1) if trace_name.startswith("void ") else trace_name
    if not trace_name.startswith(base + "<"):
        return False
    want = [str(kind) if a == "KIND" else a for a in targs(bench_kernel)]
    have = targs(trace_name)
    return all(w == h for w, h in zip(want, have) if w.isdigit())


def load_trace(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def bench_line(path):
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                return json.loads(line)
    raise SystemExit(f"no bench JSON line in {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("bench_log")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    args = ap.parse_args()
    rows = load_trace(args.trace_dir)
    b = bench_line(args.bench_log)
    W = args.warmup if args.warmup is not None else b["warmup"]
    K = args.steps if args.steps is not None else b["steps"]
    out = {"bench_cmd_steps": K, "bench_cmd_warmup": W, "dispatches": len(rows), "legs": {}}

    def leg(name, roof, kind, w, k):
        ds = [(e - s) * 1e-6 for s, e, n in rows if matches(n, roof["kernel"], kind)]
        timed = ds[w:w + k]
        if len(timed) < k:
            out["legs"][name] = {"error": f"{len(ds)} dispatches of {roof['kernel']}"}
            return
        ms = sum(timed) / len(timed)
        ach = roof["flop_per_launch"] / (ms * 1e-3) / 1e12
        out["legs"][name] = {
            "kernel": roof["kernel"], "trace_dispatches": len(ds), "timed_dispatches": f"[{w}, {w + k})",
            "trace_timed_mean_ms": ms, "trace_timed_min_ms": min(timed), "trace_timed_max_ms": max(timed),
            "trace_all_mean_ms": sum(ds) / len(ds),
            "bench_hip_event_ms": roof["avg_launch_ms"], "ratio_trace_over_bench": ms / roof["avg_launch_ms"],
            "frac_bench": roof["frac"], "frac_trace": ach / roof["peak"]}

    leg("cartpole_rollout", b["roofline"], KINDS["cartpole"], W, K)
    if "uav_ppo2_rollout" in b:
        leg("uav_rollout", b["uav_ppo2_rollout"]["roofline"], KINDS["uav"], 2, 5)
    out["ms_per_step"] = b["ms_per_step"]
    stats = defaultdict(list)
    for s, e, n in rows:
        stats[n.split("(")[0].replace("void ", "")].append((e - s) * 1e-6)
    top = sorted(stats.items(), key=lambda kv: -sum(kv[1]))[:25]
    out["top_kernels_total_ms"] = [{"kernel": k, "calls": len(v), "mean_ms": sum(v) / len(v),
                                    "total_ms": sum(v)} for k, v in top]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.exit(main())
