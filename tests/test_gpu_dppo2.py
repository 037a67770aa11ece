"""Distributed_PPO2 (the DPPO2 drop-in) at world size 2: two ranks on one GPU over gloo (the
N-GPU runs use RCCL with one GPU per rank; the arithmetic is the same).

Reference: demonstration/DPPO2/DPPO2-4-CartPole/train.py:136-210 (20 Worker processes) and
Distributed_PPO2.py:13-172. Here each rank is one Worker with n envs; rank r's envs have global
ids r*n .. r*n+n-1 and draw from the Philox stream keyed by those ids, so
  (1) the union of the ranks' rollout buffers equals a single rank's buffers on 2n envs, bit for
      bit, and
  (2) after the synchronous update (one gradient all-reduce, the Worker.learn() rule) the replicas
      are bit-identical, and stay so for the next iteration's rollout;
  (3) with the default global normalisation (ppo_msg norm_scope 'global', SURVEY §8e: reward
      chunk statistics and advantage partials gathered across ranks) the update equals the single
      rank's on 2n envs to f32 rounding of the gradient sums (1e-5), for CartPole (the DPPO2-CartPole
      copy) and the UavRobust hover outer loop (config 4's sharded PPO2).
"""
import os

import numpy as np
import pytest
import torch

from reinforcementlearningplatform_amd.algorithm.policy_base.Distributed_PPO2 import (
    DPPO2_COPY, Distributed_PPO2, dppo2_std_schedule)
from reinforcementlearningplatform_amd.environment.CartPole.CartPole import CartPole
from reinforcementlearningplatform_amd.environment.UavRobust.UavHoverOuterLoop import \
    uav_hover_outer_loop
from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic
from reinforcementlearningplatform_amd import _abi

pytestmark = pytest.mark.gpu

N, T = 2048, 64
KEYS = ("obs", "obs_next", "action", "logp", "reward", "value", "value_next", "done", "success",
        "flag")


def _agent(n, env_id0, env="cartpole", scope="global"):
    torch.manual_seed(0)   # the same initial nets on every rank (rank 0's are broadcast anyway)
    if env == "cartpole":
        e = CartPole(n_envs=n, seed=5, env_id0=env_id0, variant="dppo2")
    else:
        e = uav_hover_outer_loop(n_envs=n, seed=5, env_id0=env_id0)
        e.reset(random=True)
    ar = np.array(e.action_range, dtype=np.float64)
    actor = PPOActor_Gaussian(e.state_dim, e.action_dim, ar[:, 0], ar[:, 1], init_std=1.2)
    critic = PPOCritic(e.state_dim)
    P = 20   # train.py:136-140
    return Distributed_PPO2(e, actor_lr=1e-4 / min(P, 5), critic_lr=1e-3 / min(P, 5),
                            num_of_pro=P, ppo_msg={'k_epo': int(30 / min(P, 5)), 'gamma': 0.99,
                                                   'norm_scope': scope},
                            T=T, actor=actor, critic=critic, seed=3407)


def _flat(ag):
    return torch.cat([p.detach().reshape(-1) for p in
                      list(ag.global_actor.parameters()) + list(ag.global_critic.parameters())]
                     ).cpu().numpy()


def _run(ag):
    """Two iterations; per iteration the rollout buffers (+ the normalised rewards / advantages
    and value targets learn() consumes), then the params after learn() and the (all-reduced)
    gradient the learner stepped with."""
    rec = []
    for _ in range(2):
        w = ag.worker
        w.rollout()
        bufs = {k: w.bufs[k].cpu().numpy().copy() for k in KEYS}
        w.advantages()
        for k, t in (("rnorm", w.rnorm), ("adv", w.adv), ("v_target", w.v_target)):
            bufs[k] = t.cpu().numpy().copy()
        w.update()
        lr = w.learner
        grad = torch.cat([lr.net_a.grad, lr.net_c.grad]).cpu().numpy().copy()
        rec.append((bufs, _flat(ag), grad))
    return rec


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    for case in CASES:
        ag = _agent(N, rank * N, *case)
        assert ag.world == world and ag.worker.learner.distributed
        assert ag.worker.global_norm == (case[1] == "global")
        res[case] = _run(ag)
    out[rank] = res
    torch.distributed.destroy_process_group()


CASES = [("cartpole", "global"), ("uav", "global"), ("cartpole", "rank")]


def test_dppo2_two_ranks_union_and_replicas():
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_rank, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    for key in ("WORLD_SIZE", "RANK"):
        os.environ.pop(key, None)
    for case in CASES:
        r0, r1 = out[0][case], out[1][case]
        single = _run(_agent(2 * N, 0, *case))
        # (1) the first iteration's rollouts: the union is the 2n-env run, bit for bit
        b0, b1, bs = r0[0][0], r1[0][0], single[0][0]
        for k in KEYS:
            np.testing.assert_array_equal(np.concatenate([b0[k], b1[k]], axis=1), bs[k],
                                          err_msg=f"{case} {k}")
        assert bs["done"].any() or case[0] == "uav"
        # (2) replicas identical after each synchronous update, and the second rollout too
        for it in range(2):
            np.testing.assert_array_equal(r0[it][1], r1[it][1])
        err = np.abs(r0[0][1] - single[0][1]).max()
        gs = single[0][2]
        gerr = np.abs(r0[0][2] - gs).max() / np.abs(gs).max()
        print(f"{case}: max |param diff| {err:.3e}, gradient diff {gerr:.3e} of max|g|")
        if case[1] == "global":   # (3) the same learn() inputs and update as one rank on 2n envs
            for k in ("rnorm", "adv", "v_target"):
                u = np.concatenate([r0[0][0][k], r1[0][0][k]], axis=1)
                np.testing.assert_allclose(u, bs[k], rtol=1e-6, atol=1e-6, err_msg=f"{case} {k}")
            assert gerr <= 1e-5, (case, gerr)
            assert err <= 1e-5, (case, err)
        else:                     # per-rank normalisers: the same objective up to the statistics
            assert err < 1e-2, (case, err)
        for k in ("action", "value"):
            assert not np.array_equal(r0[1][0][k], r0[0][0][k])   # the second rollout used new nets


def test_dppo2_copy_semantics_selected():
    """Distributed_PPO2 picks the DPPO2-CartPole copy's Worker: success = (flag != 1) on every
    step, clip 0.2, SharedAdam betas, Worker.learn update rule, no lr decay."""
    ag = _agent(256, 0)
    w = ag.worker
    assert (w.rule, w.flag) == (_abi.RLP_SUCCESS_FLAG_NE, 1)
    lr = w.learner
    assert lr.rule == 'dppo2' and lr.max_norm == 0.2 and lr.betas == (0.9, 0.99)
    a_lr = lr.lr["a"]
    ag.msg['use_lr_decay'] = True
    ag.start_multi_process(iterations=1, eval_every=0, std_schedule=False)
    assert lr.lr["a"] == a_lr
    su = w.bufs["success"].cpu().numpy()
    fl = w.bufs["flag"].cpu().numpy()
    np.testing.assert_array_equal(su, (fl != 1).astype(np.uint8))


def test_dppo2_std_schedules():
    """Worker.run's exploration schedules (DPPO2-4-CartPole :160-165; the other copies :163-168)."""
    class A:
        std = torch.tensor(1.2)
    a = A()
    sch = dppo2_std_schedule(DPPO2_COPY[_abi.RLP_ENV_CARTPOLE], [[-8., 8.]])
    for t in range(501):
        sch(t, a)
    # t=250: 8/3 * 0.95; t=500: 8/3 * 0.9
    assert float(a.std.reshape(-1)[0]) == pytest.approx(8 / 3 * 0.9, rel=1e-6)
    b = A()
    sch = dppo2_std_schedule(DPPO2_COPY[_abi.RLP_ENV_UGV_FORWARD], [[-3., 3.], [-6.28, 6.28]])
    for t in range(2001):
        sch(t, b)
    assert float(b.std) == pytest.approx(1.2 * 0.95 * 0.9, rel=1e-6)
