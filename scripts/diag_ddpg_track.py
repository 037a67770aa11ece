"""Where the native DDPG update and the torch one part over tests/test_gpu_replay_ddpg.py's five
updates: per iteration and net, max |native - torch| of the parameters, the count of elements
outside the test's tolerance, and for the critic's worst element its gradient on both paths
(an Adam step moves an element by ~lr whatever its gradient's size, so a near-zero gradient whose
sign differs between two f32 summation orders moves the two copies 2 lr apart).

usage: python scripts/diag_ddpg_track.py [B]  (RLP_LIBRARY selects the library)"""
import copy
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("tddpg", os.path.join(ROOT, "tests", "test_gpu_replay_ddpg.py"))
T = importlib.util.module_from_spec(spec)
spec.loader.exec_module(T)

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
torch.manual_seed(3)
t_agent, n_agent = T.make_agent(native=False), T.make_agent(native=True)
for k in ("actor", "target_actor", "critic", "target_critic"):
    getattr(n_agent, k).load_state_dict(getattr(t_agent, k).state_dict())
for it in range(5):
    batch = T._batch(B, it)
    t_agent.update(*batch)
    n_agent.update(*batch)
    gt = torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros_like(p).reshape(-1)
                    for p in t_agent.critic.parameters()])
    gn = n_agent._native.grad["critic"]
    for k in ("actor", "critic"):
        a, b = T._flat(getattr(n_agent, k)), T._flat(getattr(t_agent, k))
        d = (a - b).abs()
        bad = d > 2e-6 + 1e-4 * b.abs()
        i = int(d.argmax())
        line = f"it {it} {k:7s} max|d| {float(d.max()):.3e} outside {int(bad.sum())}"
        if k == "critic":
            line += f"  worst #{i}: grad native {float(gn[i]):.3e} torch {float(gt[i]):.3e} max|g| {float(gt.abs().max()):.3e}"
        print(line, flush=True)
