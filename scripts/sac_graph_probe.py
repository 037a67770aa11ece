"""Stage-by-stage probe of the SAC HIP-graph learn path (GPU box)."""
import faulthandler
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.enable()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from reinforcementlearningplatform_amd.algorithm.actor_critic.Soft_Actor_Critic import SAC  # noqa
from reinforcementlearningplatform_amd.utils.classes import SACActor, SACCritic  # noqa: E402

S, A = 41, 2
LO, HI = np.array([-3., -2 * np.pi]), np.array([3., 2 * np.pi])
msg = {'state_dim': S, 'action_dim': A, 'action_range': np.stack([LO, HI], 1), 'name': 'OA'}
agent = SAC(msg, 0.99, 0.005, 4096, 256, SACActor(S, A, LO, HI, std_min=0.05, std_scale=1.),
            SACCritic(S, A), SACCritic(S, A), 1e-4, 1e-4, 1e-4, True, device="cuda", seed=1,
            graph=True)
rng = np.random.default_rng(0)
n = 3000
agent.memory.store_transition(rng.uniform(-1, 1, (n, S)), rng.uniform(LO, HI, (n, A)),
                              rng.normal(size=n), rng.uniform(-1, 1, (n, S)),
                              (rng.uniform(size=n) < 0.1).astype(np.float32))
print("stored", flush=True)
s = agent.memory.sample_buffer(False)
print("eager sample ok", flush=True)
out = agent.learn(iter=1)
torch.cuda.synchronize()
print("graphed learn 1 ok", [float(x) for x in out], flush=True)
for _ in range(10):
    agent.learn(iter=2)
torch.cuda.synchronize()
print("graphed learn x20 ok", float(agent.log_alpha), flush=True)
del agent
torch.cuda.synchronize()
print("teardown ok", flush=True)
