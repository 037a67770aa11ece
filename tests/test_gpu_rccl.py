"""RCCL on the MI355X: the data-parallel PPO2 path (VecPPO2 -> NativePPO2Learner with an explicit
process group, Distributed_PPO2's Worker) on an `init_process_group("nccl")` group of world size 1,
so the RCCL code path — device_id binding, the parameter broadcast, one flat gradient all-reduce
per optimiser step — executes on the GPU. World size 1 makes the all-reduce an identity, so the
update must equal the non-distributed learner's bit for bit.

Reference: demonstration/DPPO2/DPPO2-4-CartPole/train.py:136-210 (the worker processes this
replaces), Distributed_PPO2.py:76-103 (Worker.learn)."""
import socket

import numpy as np
import pytest
import torch

from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import VecPPO2
from reinforcementlearningplatform_amd.environment.CartPole.CartPole import CartPole
from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic

pytestmark = pytest.mark.gpu

N, T = 4096, 32


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _vec(pg, rule):
    torch.manual_seed(0)
    env = CartPole(n_envs=N, seed=5, env_id0=0)
    actor = PPOActor_Gaussian(4, 1, np.array([-8.]), np.array([8.]), init_std=2.0)
    msg = {'K_epochs': 3, 'update_rule': rule, 'use_grad_clip': rule == 'dppo2'}
    return VecPPO2(env, actor, PPOCritic(4), msg, T=T, seed=11, process_group=pg, learner="native")


def _flat(v):
    return torch.cat([p.detach().reshape(-1) for p in v.learner.params()]).cpu().numpy()


def test_rccl_world1_update_equals_local():
    import torch.distributed as dist
    assert not dist.is_initialized()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        for rule in ("ppo2", "dppo2"):
            out = []
            for pg in (dist.group.WORLD, None):
                v = _vec(pg, rule)
                assert v.learner.distributed == (pg is not None) and v.world == 1
                v.iteration(learn=True)
                v.iteration(learn=True)
                torch.cuda.synchronize()
                out.append((_flat(v), v.bufs["action"].cpu().numpy()))
            np.testing.assert_array_equal(out[0][1], out[1][1], err_msg=rule)
            np.testing.assert_array_equal(out[0][0], out[1][0], err_msg=rule)
        # an RCCL all-reduce of a gradient-sized buffer returns the rank's own values
        g = torch.randn(134658, device="cuda")
        r = g.clone()
        dist.all_reduce(r)
        torch.cuda.synchronize()
        assert torch.equal(r, g)
    finally:
        dist.destroy_process_group()
