"""The N > 1 path on CPU (gloo, world size 2), as SURVEY.md §4 tier 4 asks:
  * synchronous data-parallel PPO2 update == a single-rank update on the concatenated batch;
  * env sharding: the union of two ranks' env shards (global ids r*n + i) reproduces the
    single-device rollout exactly (checked on the CPU oracle, which keys Philox like the kernels).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import oracle
from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import (DEFAULT_PPO_MSG,
                                                                               PPO2Learner)
from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(N, seed=0):
    g = torch.Generator().manual_seed(seed)
    s = torch.rand(N, 4, generator=g) * 4 - 2
    a = torch.rand(N, 1, generator=g) * 16 - 8
    a_lp = torch.randn(N, 1, generator=g) - 2
    adv = torch.randn(N, 1, generator=g)
    vt = torch.randn(N, 1, generator=g) * 5
    return s, a, a_lp, adv, vt


def _nets(seed=1):
    torch.manual_seed(seed)
    actor = PPOActor_Gaussian(4, 1, np.array([-8.]), np.array([8.]), init_std=8 / 3, hidden=32)
    critic = PPOCritic(4, hidden=32)
    return actor, critic


MSGS = {"ppo2": dict(DEFAULT_PPO_MSG, K_epochs=3, use_grad_clip=True),
        # the DPPO2 Worker.learn rule (Distributed_PPO2's default): clip 0.2, SharedAdam betas
        "dppo2": dict(DEFAULT_PPO_MSG, K_epochs=6, use_grad_clip=True, update_rule='dppo2',
                      grad_clip_norm=0.2, adam_betas=(0.9, 0.99))}


def _worker(rank, world, port, N, out, rule="ppo2"):
    MSG = MSGS[rule]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    actor, critic = _nets(seed=100 + rank)         # different inits: rank 0's is broadcast
    learner = PPO2Learner(actor, critic, MSG, device="cpu")
    s, a, a_lp, adv, vt = _batch(N)
    sl = slice(rank * N // world, (rank + 1) * N // world)
    learner.update(s[sl], a[sl], a_lp[sl], adv[sl], vt[sl])
    flat = torch.cat([p.detach().reshape(-1) for p in learner.params()])
    out[rank] = flat.numpy().copy()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("rule", ["ppo2", "dppo2"])
def test_data_parallel_update_equals_single_rank(rule):
    MSG = MSGS[rule]
    N, world = 512, 2
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, N, out, rule), nprocs=world, start_method="spawn")
    r0, r1 = np.asarray(out[0]), np.asarray(out[1])
    np.testing.assert_array_equal(r0, r1)                         # replicas stay identical
    actor, critic = _nets(seed=100)
    single = PPO2Learner(actor, critic, MSG, device="cpu")
    single.update(*_batch(N))
    ref = torch.cat([p.detach().reshape(-1) for p in single.params()]).numpy()
    np.testing.assert_allclose(r0, ref, rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("kind", [A.RLP_ENV_CARTPOLE, A.RLP_ENV_UAV_HOVER_OUTER_LOOP])
def test_env_shards_reproduce_single_device(kind):
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind)
    rng = np.random.default_rng(0)
    ad = A.MLPDesc.make([S, 32, 32, Ad], [1, 1, 1])
    cd = A.MLPDesc.make([S, 32, 32, 1], [1, 1, 0])
    ap = (rng.normal(0, 0.3, ad.param_count())).astype(np.float32)
    cp = (rng.normal(0, 0.3, cd.param_count())).astype(np.float32)
    lo, hi = A.action_bounds(kind, p)
    n, T = 96, 10

    def run(n_loc, env_id0):
        import ctypes  # noqa: F401
        cfg = A.RolloutCfg()
        cfg.T, cfg.n, cfg.seed, cfg.step0, cfg.env_id0 = T, n_loc, 3407, 0, env_id0
        cfg.success_rule, cfg.success_flag = 0, A.timeout_flag(kind)
        for j in range(Ad):
            cfg.std[j], cfg.a_min[j], cfg.a_max[j] = (hi[j] - lo[j]) / 6, lo[j], hi[j]
        st = np.zeros((D, n_loc))
        need = np.ones(n_loc, np.uint8)
        b = oracle.rollout(kind, p, st, need, ad, ap, cd, cp, cfg)
        return b, st

    full, st_full = run(n, 0)
    shards = [run(n // 2, 0), run(n // 2, n // 2)]
    for key in ("obs", "action", "reward", "done", "flag", "value"):
        np.testing.assert_array_equal(np.concatenate([s[0][key] for s in shards], axis=1), full[key])
    np.testing.assert_array_equal(np.concatenate([s[1] for s in shards], axis=1), st_full)
