"""Gradient-level pins of the native DDPG and SAC updates against the reference's own p.grad.

Fixtures (tests/golden/make_golden.py gen_ddpg_grad / gen_sac_grad, made by running the reference):
one DDPG.learn (algorithm/actor_critic/DDPG.py:72-109, the DDPG-SOI driver's nets) and one
SAC.learn (algorithm/actor_critic/Soft_Actor_Critic.py:70-124, the SAC-UGVForward demo's nets, its
Normal.rsample noise recorded) on 1000-row batches, with every optimizer's .grad recorded at its
step(). Adam's first step is about lr * sign(g), so after-weights alone would pass a gradient that
is off by a percent; these compare the gradient itself, the way tests/test_learn_golden.py pins
the PPO2 update:

  * CPU: the recorded gradients are the float32 gradients of the losses restated below (the
    fixture is what it says), and float64 evaluation of the same losses gives the truth;
  * GPU: librlp's gradient (rlp_ddpg_update / rlp_sac_update, f32 MFMA) against that float64
    truth within 4x the reference's own float32 error + 2e-7 of the tensor's max.

DDPG's actor gradient is taken through the critic after its Adam step (learn() steps the critic
first); each side is compared with the float64 gradient through the critic it actually used.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

S_D, A_D, H = 4, 2, 256          # DDPG-SOI: actor [4,256,256,2], critic [6,256,256,1] (+ action_value)
S_S, A_S = 41, 2                 # SAC-UGVForward demo: actor [41,128,64,2+2], twin critic [43,128,64,1]
LO_S, HI_S = np.array([-3., -2 * np.pi]), np.array([3., 2 * np.pi])


def _split(flat, shapes, dtype):
    out, off = [], 0
    t = torch.as_tensor(np.asarray(flat), dtype=torch.float32).to(dtype)
    for sh in shapes:
        n = int(np.prod(sh))
        out.append(t[off:off + n].view(*sh).clone())
        off += n
    assert off == t.numel()
    return out


DDPG_ACTOR = [(H, S_D), (H,), (H, H), (H,), (A_D, H), (A_D,)]
DDPG_CRITIC = [(H, S_D + A_D), (H,), (H, H), (H,), (H, A_D), (H,), (1, H), (1,)]   # fc1 fc2 action_value q


def _ddpg_actor(P, s):   # demonstration/DDPG/DDPG-4-SecondOrderIntegration/train.py:63-100
    h = F.relu(F.linear(F.relu(F.linear(s, P[0], P[1])), P[2], P[3]))
    return 3.0 * torch.tanh(F.linear(h, P[4], P[5]))          # gain 3, off 0 (action range +-3)


def _ddpg_critic(P, s, a):   # train.py:26-60 (action_value is never used by forward)
    h = F.relu(F.linear(F.relu(F.linear(torch.cat([s, a], 1), P[0], P[1])), P[2], P[3]))
    return F.linear(h, P[6], P[7])


def ddpg_grads(g, dtype, critic_after=None):
    """DDPG.learn's two gradients in `dtype`: the critic's at the before-weights, the actor's
    through `critic_after` (default: the reference's critic after its step)."""
    t = lambda k: torch.as_tensor(np.asarray(g[k]), dtype=torch.float32).to(dtype)
    s, a, r, s2, end = t("s"), t("a"), t("r"), t("s2"), t("end")
    Pa = _split(g["before_actor"], DDPG_ACTOR, dtype)
    Pc = _split(g["before_critic"], DDPG_CRITIC, dtype)
    with torch.no_grad():
        q_ = _ddpg_critic(_split(g["before_target_critic"], DDPG_CRITIC, dtype), s2,
                          _ddpg_actor(_split(g["before_target_actor"], DDPG_ACTOR, dtype), s2))
        target = r.unsqueeze(1) + 0.99 * end.unsqueeze(1) * q_
    for p in Pc:
        p.requires_grad_(True)
    F.mse_loss(target, _ddpg_critic(Pc, s, a)).backward()
    gc = torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros(p.numel(), dtype=dtype)
                    for p in Pc])
    Pc2 = _split(g["after_critic"] if critic_after is None else critic_after, DDPG_CRITIC, dtype)
    for p in Pa:
        p.requires_grad_(True)
    (-_ddpg_critic(Pc2, s, _ddpg_actor(Pa, s)).mean()).backward()
    ga = torch.cat([p.grad.reshape(-1) for p in Pa])
    return {"critic": gc.double().numpy(), "actor": ga.double().numpy()}


SAC_ACTOR = [(128, S_S), (128,), (64, 128), (64,), (A_S, 64), (A_S,), (A_S, 64), (A_S,)]
SAC_CRITIC = [(128, S_S + A_S), (128,), (64, 128), (64,), (1, 64), (1,)] * 2


def _sac_bounds(dtype):
    """SACActor's log_std clamp bounds as the demo computes them, in float32
    (demonstration/SAC/SAC-4-UGVForward/train.py:68-70: std_min 0.05, std_scale 1)."""
    lo, hi = torch.tensor(LO_S, dtype=torch.float), torch.tensor(HI_S, dtype=torch.float)
    return torch.log(0.05 * (hi - lo) / 2).to(dtype), ((hi - lo) / 2 / 1.0).to(dtype)


def _sac_actor(P, x, eps, dtype):   # train.py:63-87
    h = F.relu(F.linear(F.relu(F.linear(x, P[0], P[1])), P[2], P[3]))
    mean = F.linear(h, P[4], P[5])
    blo, bhi = _sac_bounds(dtype)
    ls = torch.clamp(F.linear(h, P[6], P[7]), blo, bhi)
    std = torch.exp(ls)
    u = mean + eps * std
    lp = torch.distributions.Normal(mean, std).log_prob(u).sum(1, keepdim=True)
    lp = lp - (2 * (np.log(2) - u - F.softplus(-2 * u))).sum(1, keepdim=True)
    hi = torch.tensor(HI_S, dtype=torch.float).to(dtype)
    return torch.tanh(u) * hi, lp                               # gain = a_max (off 0)


def _sac_critic(P, s, a):   # train.py:90-120
    sa = torch.cat([s, a], 1)
    q = [F.linear(F.relu(F.linear(F.relu(F.linear(sa, P[o], P[o + 1])), P[o + 2], P[o + 3])),
                  P[o + 4], P[o + 5]) for o in (0, 6)]
    return q[0], q[1]


def sac_grads(g, dtype):
    """SAC.learn's actor, critic and log_alpha gradients in `dtype` (all taken at the before-
    weights: learn() forms every loss before its first optimizer step)."""
    t = lambda k: torch.as_tensor(np.asarray(g[k]), dtype=torch.float32).to(dtype)
    s, a, r, s2, dw = t("s"), t("a"), t("r").unsqueeze(1), t("s2"), t("dw").unsqueeze(1)
    eps = t("eps")
    Pa = _split(g["before_actor"], SAC_ACTOR, dtype)
    Pc = _split(g["before_critic"], SAC_CRITIC, dtype)
    la = t("before_log_alpha").clone().requires_grad_(True)
    alpha = la.exp()
    with torch.no_grad():
        a_, lp_ = _sac_actor(Pa, s2, eps[0], dtype)
        q1, q2 = _sac_critic(_split(g["before_target_critic"], SAC_CRITIC, dtype), s2, a_)
        target = r + 0.99 * (1 - dw) * (torch.min(q1, q2) - alpha.detach() * lp_)
    for p in Pa + Pc:
        p.requires_grad_(True)
    an, lp = _sac_actor(Pa, s, eps[1], dtype)
    q1, q2 = _sac_critic(Pc, s, an)
    ga = torch.autograd.grad((alpha.detach() * lp - torch.min(q1, q2)).mean(), Pa)
    c1, c2 = _sac_critic(Pc, s, a)
    gc = torch.autograd.grad(F.mse_loss(c1, target) + F.mse_loss(c2, target), Pc)
    gl = torch.autograd.grad(-(la.exp() * (lp + (-A_S)).detach()).mean(), [la])
    cat = lambda gs: torch.cat([x.reshape(-1) for x in gs]).double().numpy()
    return {"actor": cat(ga), "critic": cat(gc), "log_alpha": cat(gl)}


def _check_fixture(g, g32, g64, names):
    for k in names:
        ref = g[f"grad_{k}"].astype(np.float64)
        scale = np.abs(g64[k]).max()
        assert scale > 0, k
        assert np.abs(ref - g32[k]).max() <= 1e-6 * scale, (k, np.abs(ref - g32[k]).max() / scale)
        assert np.abs(ref - g64[k]).max() <= 1e-4 * scale, (k, np.abs(ref - g64[k]).max() / scale)


def test_ddpg_reference_grads_cpu(golden):
    g = golden("ddpg_soi_grad")
    _check_fixture(g, ddpg_grads(g, torch.float32), ddpg_grads(g, torch.float64), ("critic", "actor"))
    # the critic's action_value layer gets no gradient (forward never reaches it)
    off = H * (S_D + A_D) + H + H * H + H
    assert not g["grad_critic"][off:off + H * A_D + H].any()


def test_sac_reference_grads_cpu(golden):
    g = golden("sac_grad")
    _check_fixture(g, sac_grads(g, torch.float32), sac_grads(g, torch.float64),
                   ("actor", "critic", "log_alpha"))
    # both log_std clamp bounds are active in the fixture's s-draw rows (the clamp's zero gradient)
    with torch.no_grad():
        P = _split(g["before_actor"], SAC_ACTOR, torch.float64)
        x = torch.as_tensor(g["s"])
        h = F.relu(F.linear(F.relu(F.linear(x, P[0], P[1])), P[2], P[3]))
        ls = F.linear(h, P[6], P[7])
        blo, bhi = _sac_bounds(torch.float64)
        assert (ls < blo).any() and (ls > bhi).any() and ((ls > blo) & (ls < bhi)).any()


def _bound(name, native, ref, truth_n, truth_r, floor_rel=2e-7):
    """|native - truth| <= 4 |reference - truth| + floor (each against the float64 gradient of the
    inputs it used)."""
    e32 = np.abs(ref - truth_r).max()
    floor = floor_rel * np.abs(truth_n).max()
    en = np.abs(native - truth_n).max()
    print(f"{name}: native err {en:.3e}, reference f32 err {e32:.3e}, floor {floor:.3e}")
    assert en <= 4 * e32 + floor, (name, en, e32, floor)


@pytest.mark.gpu
def test_native_ddpg_grads_match_reference(golden):
    from test_gpu_replay_ddpg import make_agent
    g = golden("ddpg_soi_grad")
    agent = make_agent(g, native=True, batch=1000)
    dev = lambda k: torch.as_tensor(np.asarray(g[k]), dtype=torch.float32, device="cuda")
    agent.update(dev("s"), dev("a"), dev("r"), dev("s2"), dev("end"))
    torch.cuda.synchronize()
    gn = {k: agent._native.grad[k].double().cpu().numpy() for k in ("critic", "actor")}
    crit_n = torch.cat([p.detach().reshape(-1) for p in agent.critic.parameters()]).cpu().numpy()
    t_ref = ddpg_grads(g, torch.float64)
    t_nat = ddpg_grads(g, torch.float64, critic_after=crit_n)
    _bound("critic", gn["critic"], g["grad_critic"].astype(np.float64), t_ref["critic"], t_ref["critic"])
    _bound("actor", gn["actor"], g["grad_actor"].astype(np.float64), t_nat["actor"], t_ref["actor"])
    # after-weights of the four nets (the soft updates included)
    for k, m in (("actor", agent.actor), ("target_actor", agent.target_actor),
                 ("critic", agent.critic), ("target_critic", agent.target_critic)):
        got = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        np.testing.assert_allclose(got, g[f"after_{k}"], rtol=1e-5, atol=1e-7, err_msg=k)


@pytest.mark.gpu
def test_native_sac_grads_match_reference(golden):
    from test_gpu_sac import load_flat, make_agent
    g = golden("sac_grad")
    agent = make_agent(native=True, batch=1000)
    for k, m in (("before_actor", agent.actor), ("before_critic", agent.critic),
                 ("before_target_critic", agent.target_critic)):
        load_flat(m, g[k])
    dev = lambda k: torch.as_tensor(np.asarray(g[k]), dtype=torch.float32, device="cuda")
    agent.update(dev("s"), dev("a"), dev("r"), dev("s2"), dev("dw"), noise=dev("eps"))
    torch.cuda.synchronize()
    nat = agent._native
    gn = {"actor": nat.grad["actor"].double().cpu().numpy(),
          "critic": nat.grad["critic"].double().cpu().numpy(),
          "log_alpha": nat.alpha_grad.double().cpu().numpy()}
    t64 = sac_grads(g, torch.float64)
    for k in ("actor", "critic", "log_alpha"):
        _bound(k, gn[k], g[f"grad_{k}"].astype(np.float64), t64[k], t64[k])
    for k, m in (("actor", agent.actor), ("critic", agent.critic),
                 ("target_critic", agent.target_critic)):
        got = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        np.testing.assert_allclose(got, g[f"after_{k}"], rtol=1e-5, atol=1e-7, err_msg=k)
    np.testing.assert_allclose(agent.log_alpha.detach().cpu().numpy(), g["after_log_alpha"],
                               rtol=1e-5, atol=1e-8)
