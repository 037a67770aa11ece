"""GPU parity of the native PPO2 update (rlp_ppo2_grad + rlp_adam_step, NativePPO2Learner) against
the reference learn() arithmetic (Proximal_Policy_Optimization2.py:102-163) in torch autograd.

Truth is the same loss evaluated in float64; the native gradients must be within a small factor of
torch float32's own error (the reference computes in float32), and the full K-epoch update must
track the torch-autograd learner (vec_ppo2.PPO2Learner, torch.optim.Adam) step for step.
"""
import copy

import numpy as np
import pytest
import torch

from reinforcementlearningplatform_amd.algorithm.policy_base.native_ppo2 import NativePPO2Learner
from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import (DEFAULT_PPO_MSG,
                                                                               PPO2Learner)
from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic

pytestmark = pytest.mark.gpu


def make_case(S, A, N, seed):
    torch.manual_seed(seed)
    lo, hi = -8.0 * np.ones(A), 8.0 * np.ones(A)
    actor = PPOActor_Gaussian(S, A, lo, hi, init_std=8 / 3)
    critic = PPOCritic(S)
    with torch.no_grad():  # a last layer large enough for non-trivial tanh'(z3)
        torch.nn.init.orthogonal_(actor.mean_layer.weight, gain=1.0)
        for m in (actor.fc1, actor.fc2, actor.mean_layer, critic.fc1, critic.fc2, critic.fc3):
            m.bias.normal_(0, 0.1)
    g = torch.Generator().manual_seed(seed + 1)
    s = torch.rand(N, S, generator=g) * 4 - 2
    with torch.no_grad():
        mean = actor(s)
        a = torch.clamp(mean + actor.std * torch.randn(N, A, generator=g), -8, 8)
        lp = torch.distributions.Normal(mean, actor.std).log_prob(a)
        lp = lp + 0.3 * torch.randn(N, A, generator=g)   # ratios spread over the clip range
    adv = torch.randn(N, 1, generator=g)
    vt = 2 * torch.randn(N, 1, generator=g)
    return actor, critic, s, a, lp, adv, vt


def torch_grads(actor, critic, s, a, lp, adv, vt, msg, dtype):
    actor, critic = copy.deepcopy(actor).to(dtype), copy.deepcopy(critic).to(dtype)
    s, a, lp, adv, vt = (t.to(dtype) for t in (s, a, lp, adv, vt))
    dist = actor.get_dist(s)
    ent = dist.entropy().sum(1, keepdim=True)
    ratios = torch.exp(dist.log_prob(a).sum(1, keepdim=True) - lp.sum(1, keepdim=True))
    surr1 = ratios * adv
    surr2 = torch.clamp(ratios, 1 - msg['eps_clip'], 1 + msg['eps_clip']) * adv
    al = (-torch.min(surr1, surr2) - msg['entropy_coef'] * ent).mean()
    cl = torch.nn.functional.mse_loss(vt, critic(s))
    al.backward()
    cl.backward()
    ga = torch.cat([p.grad.reshape(-1) for p in actor.parameters()]).double()
    gc = torch.cat([p.grad.reshape(-1) for p in critic.parameters()]).double()
    return ga, gc, float(al.detach()), float(cl.detach())


def split(flat, module):
    out, off = [], 0
    for p in module.parameters():
        out.append(flat[off:off + p.numel()])
        off += p.numel()
    return out


@pytest.mark.parametrize("S,A,N", [(4, 1, 3037), (6, 3, 2113), (2, 2, 64), (4, 1, 1)])
def test_ppo2_grads_vs_torch(S, A, N):
    msg = dict(DEFAULT_PPO_MSG)
    actor, critic, s, a, lp, adv, vt = make_case(S, A, N, seed=S * 10 + A)
    ga64, gc64, al64, cl64 = torch_grads(actor, critic, s, a, lp, adv, vt, msg, torch.float64)
    ga32, gc32, al32, cl32 = torch_grads(actor, critic, s, a, lp, adv, vt, msg, torch.float32)
    ref_a, ref_c = copy.deepcopy(actor), copy.deepcopy(critic)
    nl = NativePPO2Learner(actor, critic, msg, device="cuda")
    dev = lambda t: t.cuda().contiguous()
    nl.grads(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
    gan, gcn = nl.net_a.grad.double().cpu(), nl.net_c.grad.double().cpu()
    for name, gn, g32, g64, mod in (("actor", gan, ga32, ga64, ref_a),
                                    ("critic", gcn, gc32, gc64, ref_c)):
        for i, (tn, t32, t64) in enumerate(zip(split(gn, mod), split(g32, mod), split(g64, mod))):
            scale = float(t64.abs().max()) + 1e-12
            en = float((tn - t64).abs().max())
            e32 = float((t32 - t64).abs().max())
            assert en <= 4 * e32 + 2e-6 * scale, (name, i, en, e32, scale)
    la, lc = (nl.loss / N).cpu().tolist()
    assert abs(la - al64) <= 1e-5 * (abs(al64) + 1) and abs(lc - cl64) <= 1e-5 * (abs(cl64) + 1)
    # run-to-run identical: gradients and the loss sums (per-wave partials, fixed-order reduce)
    g0, l0 = (nl.net_a.grad.clone(), nl.net_c.grad.clone()), nl.loss.clone()
    nl.grads(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
    assert torch.equal(g0[0], nl.net_a.grad) and torch.equal(g0[1], nl.net_c.grad)
    assert torch.equal(l0, nl.loss)


def test_ppo2_grads_minibatch_index():
    msg = dict(DEFAULT_PPO_MSG)
    actor, critic, s, a, lp, adv, vt = make_case(4, 1, 2000, seed=5)
    idx = torch.randperm(2000, generator=torch.Generator().manual_seed(1))[:517]
    ga64, gc64, _, _ = torch_grads(actor, critic, s[idx], a[idx], lp[idx], adv[idx], vt[idx], msg,
                                   torch.float64)
    ga32, gc32, _, _ = torch_grads(actor, critic, s[idx], a[idx], lp[idx], adv[idx], vt[idx], msg,
                                   torch.float32)
    nl = NativePPO2Learner(actor, critic, msg, device="cuda")
    dev = lambda t: t.cuda().contiguous()
    nl.grads(dev(s), dev(a), dev(lp), dev(adv), dev(vt), index=dev(idx))
    for gn, g32, g64 in ((nl.net_a.grad, ga32, ga64), (nl.net_c.grad, gc32, gc64)):
        en = float((gn.double().cpu() - g64).abs().max())
        e32 = float((g32 - g64).abs().max())
        assert en <= 4 * e32 + 2e-6 * float(g64.abs().max()), (en, e32)


@pytest.mark.parametrize("clip,mini", [(False, False), (True, False), (False, True)])
def test_native_update_tracks_torch_learner(clip, mini):
    msg = dict(DEFAULT_PPO_MSG, K_epochs=3, use_grad_clip=clip, using_mini_batch=mini,
               mini_batch_size=700)
    actor, critic, s, a, lp, adv, vt = make_case(4, 1, 2500, seed=9)
    ta, tc = copy.deepcopy(actor), copy.deepcopy(critic)
    tl = PPO2Learner(ta, tc, msg, device="cuda")
    nl = NativePPO2Learner(actor, critic, msg, device="cuda")
    dev = lambda t: t.cuda().contiguous()
    args = [dev(t) for t in (s, a, lp, adv, vt)]
    g1, g2 = (torch.Generator(device="cuda").manual_seed(3) for _ in range(2))
    lt = tl.update(*args, generator=g1)
    ln = nl.update(*args, generator=g2)
    for m_t, m_n in ((ta, actor), (tc, critic)):
        for pt, pn in zip(m_t.parameters(), m_n.parameters()):
            assert torch.allclose(pn, pt, rtol=1e-5, atol=2e-6), float((pn - pt).abs().max())
    assert abs(float(ln[0]) - float(lt[0])) <= 1e-4 * (abs(float(lt[0])) + 1)
    assert abs(float(ln[1]) - float(lt[1])) <= 1e-4 * (abs(float(lt[1])) + 1)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, out):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    # gloo on one card: both ranks share cuda:0 (the N-GPU runs use RCCL, one GPU per rank)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    msg = dict(DEFAULT_PPO_MSG, K_epochs=3, use_grad_clip=True)
    actor, critic, s, a, lp, adv, vt = make_case(4, 1, 2048, seed=21)
    if rank == 1:  # a different init: rank 0's replica is broadcast
        with torch.no_grad():
            for p in list(actor.parameters()) + list(critic.parameters()):
                p.add_(0.05)
    nl = NativePPO2Learner(actor, critic, msg, device="cuda")
    sl = slice(rank * 1024, (rank + 1) * 1024)
    dev = lambda t: t[sl].cuda().contiguous()
    nl.update(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
    out[rank] = torch.cat([nl.net_a.flat, nl.net_c.flat]).cpu().numpy().copy()
    torch.distributed.destroy_process_group()


def test_native_update_data_parallel_two_ranks():
    """Synchronous DP (one flat gradient all-reduce per step) of the native learner == a single
    learner on the concatenated batch (equal halves: mean of means == mean)."""
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_dp_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    r0, r1 = np.asarray(out[0]), np.asarray(out[1])
    np.testing.assert_allclose(r0, r1, rtol=0, atol=1e-7)
    msg = dict(DEFAULT_PPO_MSG, K_epochs=3, use_grad_clip=True)
    actor, critic, s, a, lp, adv, vt = make_case(4, 1, 2048, seed=21)
    nl = NativePPO2Learner(actor, critic, msg, device="cuda")
    dev = lambda t: t.cuda().contiguous()
    nl.update(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
    ref = torch.cat([nl.net_a.flat, nl.net_c.flat]).cpu().numpy()
    np.testing.assert_allclose(r0, ref, rtol=1e-5, atol=2e-6)


DUP_CASES = [("ppo2", False), ("ppo2", True), ("dppo2", False), ("dppo2", True)]


def _dup_msg(rule, clip):
    return dict(DEFAULT_PPO_MSG, K_epochs=3, use_grad_clip=clip, update_rule=rule,
                grad_clip_norm=0.2 if rule == "dppo2" else 0.5)


def _dp_dup_worker(rank, world, port, out):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    res = []
    for rule, clip in DUP_CASES:
        actor, critic, s, a, lp, adv, vt = make_case(4, 1, 1536, seed=33)
        nl = NativePPO2Learner(actor, critic, _dup_msg(rule, clip), device="cuda")
        dev = lambda t: t.cuda().contiguous()
        nl.update(dev(s), dev(a), dev(lp), dev(adv), dev(vt))   # the SAME batch on both ranks
        nl.update(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
        res.append(torch.cat([nl.net_a.flat, nl.net_c.flat]).cpu().numpy().copy())
    out[rank] = res
    torch.distributed.destroy_process_group()


def test_native_update_data_parallel_duplicated_batch_bit_exact():
    """with the same batch on both ranks the gradient average is the identity
    ((g + g) / 2 == g exactly in f32), so a missing or doubled `/ world` in the all-reduce, or an
    all-reduce applied at the wrong point of the update rule, shows as a bit difference against a
    single-rank learner. Both update rules, clipping off and on, two learn() calls."""
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_dp_dup_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    for i, (rule, clip) in enumerate(DUP_CASES):
        actor, critic, s, a, lp, adv, vt = make_case(4, 1, 1536, seed=33)
        nl = NativePPO2Learner(actor, critic, _dup_msg(rule, clip), device="cuda")
        dev = lambda t: t.cuda().contiguous()
        nl.update(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
        nl.update(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
        ref = torch.cat([nl.net_a.flat, nl.net_c.flat]).cpu().numpy()
        for r in (0, 1):
            np.testing.assert_array_equal(out[r][i], ref, err_msg=f"rank {r} {rule} clip={clip}")


# ---------------------------------------------------------------------------------------------
# Rows exactly at a clip kink (ratio = 1 -/+ eps_clip in float64). There the clipped surrogate's
# gradient jumps: torch.min / clamp give a row either its full term or none, and which one two
# correct float32 evaluations pick depends on the last ulp of their ratio. The native update must
# give one of the two (the rest of the batch unchanged), for both kinks and advantage signs.
# ---------------------------------------------------------------------------------------------
def _kink_candidates(actor, critic, s, a, lp64, adv, vt, msg, row):
    """float64 actor gradients with row `row`'s old log-prob 1e-6 to either side of the exact
    float64 kink lp64[row] (beyond the float32 errors of lp and of the ratio, ~3e-7): one candidate
    has the row inside the clip range, the other clipped."""
    out = []
    for delta in (-1e-6, 1e-6):
        lp2 = lp64.clone()
        lp2[row, 0] += delta
        ga, _, _, _ = torch_grads(actor, critic, s, a, lp2, adv, vt, msg, torch.float64)
        out.append(ga)
    return out


@pytest.mark.parametrize("kink,adv_sign", [(+1, +1), (+1, -1), (-1, +1), (-1, -1)])
def test_ppo2_grad_at_clip_kink(kink, adv_sign):
    msg = dict(DEFAULT_PPO_MSG)
    eps = msg['eps_clip']
    actor, critic, s, a, lp, adv, vt = make_case(4, 1, 257, seed=77)
    row = 100
    with torch.no_grad():   # the row's old log-prob puts its float64 ratio exactly on the kink
        a64 = copy.deepcopy(actor).double()
        lp_now = a64.get_dist(s.double()).log_prob(a.double())
        lp64 = lp.clone().double()
        lp64[row, 0] = lp_now[row, 0] - np.log(1 + kink * eps)
        lp = lp64.float()
        adv = adv.clone()
        adv[row, 0] = adv_sign * (abs(float(adv[row, 0])) + 0.5)
    cands = _kink_candidates(actor, critic, s, a, lp64, adv, vt, msg, row)
    ga32, _, _, _ = torch_grads(actor, critic, s, a, lp, adv, vt, msg, torch.float32)
    nl = NativePPO2Learner(copy.deepcopy(actor), copy.deepcopy(critic), msg, device="cuda")
    dev = lambda t: t.cuda().contiguous()
    nl.grads(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
    gn = nl.net_a.grad.double().cpu()
    errs = [float((gn - c).abs().max()) for c in cands]
    e32 = min(float((ga32 - c).abs().max()) for c in cands)
    floor = 2e-6 * float(max(c.abs().max() for c in cands))
    # the candidates differ by the row's whole term where the branches disagree (upper kink with
    # adv > 0, lower kink with adv < 0), else they agree; the native gradient is one of them
    assert min(errs) <= 4 * e32 + floor, (errs, e32, floor)
