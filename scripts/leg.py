"""Run one bench.py leg by name on cuda:0 and print its JSON (A/B and profiling helper; not the
bench contract). Usage: python scripts/leg.py ugvoa_ppo2_leg [key=value ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    kw = {}
    for a in sys.argv[2:]:
        k, v = a.split("=", 1)
        kw[k] = int(v) if v.lstrip("-").isdigit() else v
    out = getattr(bench, sys.argv[1])(0, **kw)
    print(json.dumps(out, default=str), flush=True)
