"""Profiling driver for the native DDPG update: N rlp_ddpg_update calls at the bench shape
(SOI DDPG nets, batch 4096). usage: python scripts/ddpg_prof.py [iters] [batch]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_replay_ddpg import _batch, make_agent  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
for native in (True, False):
    torch.manual_seed(0)
    agent = make_agent(batch=B, native=native)
    batch = _batch(B, 0)
    for _ in range(3):
        agent.update(*batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        agent._update_core(*batch)
    torch.cuda.synchronize()
    print(f"native={native} B={B}: {(time.perf_counter() - t0) / iters * 1e3:.3f} ms per update (eager)")
