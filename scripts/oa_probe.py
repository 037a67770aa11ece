"""Host-side timing probe of the UGVForwardObstacleAvoidance step / reset launches (GPU box)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from reinforcementlearningplatform_amd import kernels as K
from reinforcementlearningplatform_amd.environment.UGVForwardObstacleAvoidance import \
    UGVForwardObstacleAvoidance

for n in (16384, 131072):
    env = UGVForwardObstacleAvoidance(n_envs=n, seed=1)
    kind, p = env.KIND, env.params
    a = torch.rand(n, 2, device="cuda")
    d = torch.zeros(n, dtype=torch.uint8, device="cuda")

    def t(f, it=50):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / it * 1e3

    ms_step = t(lambda: K.env_step(kind, p, env.state, a, want_obs_cur=False))
    ms_reset = t(lambda: K.env_reset(kind, p, env.state, mask=d, seed=1, counter=1))
    ms_obs = t(lambda: K.env_observe(kind, p, env.state))
    ms_sum = t(lambda: d.sum())
    print(f"n={n}: step {ms_step:.3f} ms, reset(mask none set) {ms_reset:.3f} ms, "
          f"observe {ms_obs:.3f} ms, d.sum {ms_sum:.3f} ms", flush=True)
