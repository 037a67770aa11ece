"""Profiling driver for the native off-policy updates: N eager rlp_ddpg_update / rlp_sac_update
calls at the bench shapes (SOI DDPG nets, UGV-OA SAC demo nets; batch 4096) next to the torch path.
usage: python scripts/ddpg_prof.py [iters] [batch] [ddpg|sac|both]"""
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_replay_ddpg as td  # noqa: E402
import test_gpu_sac as ts  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
which = sys.argv[3] if len(sys.argv) > 3 else "both"
for name, mk, bt in (("ddpg", td.make_agent, td._batch), ("sac", ts.make_agent, ts._sac_batch)):
    if which not in (name, "both"):
        continue
    for native in (True, False):
        torch.manual_seed(0)
        agent = mk(batch=B, native=native)
        batch = bt(B, 0)
        for _ in range(3):
            agent.update(*batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            agent.update(*batch)
        torch.cuda.synchronize()
        print(f"{name} native={native} B={B}: {(time.perf_counter() - t0) / iters * 1e3:.3f} ms per "
              f"update (eager)")
