"""Nets the fused f16x3 kernels do not take, on librlp (the four PPO2 drivers):

  * the PPO2-SecondOrderIntegration demo's actor 4 -> 128 -> 64 -> 32 -> 2 and critic
    4 -> 64 -> 64 -> 1 (demonstration/PPO2/PPO2-4-SecondOrderIntegration/train.py:37-125, K = 30),
  * the obstacle-avoidance demos' 41 -> 256 -> 256 -> 2 / -> 1 nets (demonstration/PPO2/
    PPO2-4-UGVForwardObstacleAvoidance/train.py:48-50,95-97, K = 25).

(1) rlp_ppo2_dense_grad (exact f32 MFMA GEMMs) against the same loss in torch float64: within 4x
    torch float32's own error + 2e-6 of the tensor's max, at 1 000 rows and across two 2^18-row
    chunks; bit-identical on a second run.
(2) NativePPO2Learner on the SOI demo nets against the reference's own learn() (tests/golden/
    ppo2_soi_learn.npz, made by running the reference): first-step p.grad and after-weights.
(3) rlp_rollout's plain-layout path (cfg net_layout 1) with the SOI demo nets, teacher-forced
    against the oracle: physics exact / 1e-9, the oracle's double-accumulated policy and critic on
    the kernel's observations; VecPPO2 runs whole iterations on them.
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn
from torch.distributions import Normal

from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd import kernels as K
from reinforcementlearningplatform_amd.algorithm.policy_base.native_ppo2 import (NativePPO2Learner,
                                                                                 dense_fits)
from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import DEFAULT_PPO_MSG, VecPPO2

pytestmark = pytest.mark.gpu


class SoiActor(nn.Module):   # demonstration/PPO2/PPO2-4-SecondOrderIntegration/train.py:37-88
    """PPOActor_Gaussian of the demo drivers with any hidden widths (the SOI demo's (128, 64, 32);
    the lidar demos' (256, 256)): tanh hidden layers, tanh(mean_layer) * gain + off."""

    def __init__(self, a_min=(-3., -3.), a_max=(3., 3.), init_std=1.0, S=4, widths=(128, 64, 32)):
        super().__init__()
        dims = (S,) + tuple(widths)
        self.hidden = nn.ModuleList([nn.Linear(dims[i], dims[i + 1]) for i in range(len(widths))])
        self.mean_layer = nn.Linear(dims[-1], len(a_min))
        self.a_min, self.a_max = torch.tensor(a_min, dtype=torch.float), torch.tensor(a_max, dtype=torch.float)
        self.off = (self.a_min + self.a_max) / 2.0
        self.gain = self.a_max - self.off
        self.std = torch.tensor(init_std, dtype=torch.float)
        for l in self.hidden:
            nn.init.orthogonal_(l.weight)
            nn.init.constant_(l.bias, 0)
        nn.init.orthogonal_(self.mean_layer.weight, gain=0.01)
        nn.init.constant_(self.mean_layer.bias, 0)

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)
        self.a_min, self.a_max, self.off, self.gain = (fn(t) for t in (self.a_min, self.a_max,
                                                                       self.off, self.gain))
        self.std = fn(self.std)
        return self

    def forward(self, s):
        for l in self.hidden:
            s = torch.tanh(l(s))
        return torch.tanh(self.mean_layer(s)) * self.gain + self.off

    def get_dist(self, s):
        mean = self.forward(s)
        return Normal(mean, self.std.expand_as(mean))


class SoiCritic(nn.Module):  # train.py:91-125 (fc3 is the output layer)
    def __init__(self, S=4, widths=(64, 64)):
        super().__init__()
        self.fc1, self.fc2 = nn.Linear(S, widths[0]), nn.Linear(widths[0], widths[1])
        self.fc3 = nn.Linear(widths[1], 1)
        for l in (self.fc1, self.fc2, self.fc3):
            nn.init.orthogonal_(l.weight)
            nn.init.constant_(l.bias, 0)

    def forward(self, s):
        return self.fc3(torch.tanh(self.fc2(torch.tanh(self.fc1(s)))))


def _load(m, flat):
    off = 0
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.as_tensor(np.asarray(flat[off:off + p.numel()])).view_as(p))
            off += p.numel()


def _loss_grads(actor, critic, s, a, lp, adv, vt, eps_clip=0.2, ent=0.01):
    """Proximal_Policy_Optimization2.py:133-159's two losses and their gradients (any dtype)."""
    dist = actor.get_dist(s)
    e = dist.entropy().sum(1, keepdim=True)
    ratios = torch.exp(dist.log_prob(a).sum(1, keepdim=True) - lp.sum(1, keepdim=True))
    surr1 = ratios * adv
    surr2 = torch.clamp(ratios, 1 - eps_clip, 1 + eps_clip) * adv
    la = (-torch.min(surr1, surr2) - ent * e).mean()
    lc = torch.nn.functional.mse_loss(vt, critic(s))
    ga = torch.autograd.grad(la, list(actor.parameters()))
    gc = torch.autograd.grad(lc, list(critic.parameters()))
    cat = lambda g: torch.cat([t.reshape(-1) for t in g]).double().cpu().numpy()
    return cat(ga), cat(gc)


def _as(m, dtype, device):
    import copy
    return copy.deepcopy(m).to(device=device, dtype=dtype)


def _f32_class(name, native, t32, t64, floor_rel=2e-6):
    e32 = np.abs(t32 - t64).max()
    en = np.abs(native - t64).max()
    floor = floor_rel * np.abs(t64).max()
    print(f"{name}: native err {en:.3e}, torch f32 err {e32:.3e}, floor {floor:.3e}")
    assert en <= 4 * e32 + floor, (name, en, e32, floor)


def _off_kinks(actor, s, a, lp, eps_clip=0.2, margin=1e-4):
    """The clipped surrogate's gradient jumps where the ratio crosses 1 -/+ eps_clip (torch.min /
    clamp): a row whose ratio lies within f32 rounding of a kink takes either side's gradient in
    two correct f32 evaluations, a whole row's term apart (at 3e5 rows a few such rows are
    expected). Rows within `margin` of a kink (in float64) get their old log-prob moved by 0.01,
    so every evaluation differentiates the same branch."""
    with torch.no_grad():
        d = _as(actor, torch.float64, "cuda").get_dist(s.double())
        r = torch.exp(d.log_prob(a.double()).sum(1) - lp.double().sum(1))
        near = ((r - (1 - eps_clip)).abs() < margin) | ((r - (1 + eps_clip)).abs() < margin)
        lp = lp.clone()
        lp[near, 0] += 0.01
    return lp


NETS = {"soi": (lambda: SoiActor(), lambda: SoiCritic(), 4, 2),
        "lidar": (lambda: SoiActor(a_min=(-3., -2 * np.pi), a_max=(3., 2 * np.pi), S=41,
                                   widths=(256, 256)),
                  lambda: SoiCritic(S=41, widths=(256, 256)), 41, 2)}


@pytest.mark.parametrize("rows", [1, 33, 1000, 300_000])
@pytest.mark.parametrize("net,kernels", [("lidar", "auto"), ("lidar", "dense"), ("soi", "auto")])
def test_dense_grad_vs_float64(net, kernels, rows):
    """rlp_ppo2_dense_grad (kernels 'dense', and the SOI nets' 'auto') and, for the lidar nets'
    'auto', rlp_ppo2_grad's f16x3 FD / wgrad kernels with layer 1 on the exact-f32 GEMM."""
    mk_a, mk_c, S, Ad = NETS[net]
    torch.manual_seed(7)
    actor, critic = mk_a(), mk_c()
    with torch.no_grad():
        nn.init.orthogonal_(actor.mean_layer.weight, gain=1.0)
    assert dense_fits(actor, True) and dense_fits(critic, False)
    g = torch.Generator(device="cuda").manual_seed(rows)
    s = torch.rand(rows, S, device="cuda", generator=g) * 4 - 2
    with torch.no_grad():
        mean = _as(actor, torch.float32, "cuda")(s)
    a = (mean + 0.7 * torch.randn(rows, Ad, device="cuda", generator=g)).clamp(-3, 3)
    lp = Normal(mean, 1.0).log_prob(a) + 0.3 * torch.randn(rows, Ad, device="cuda", generator=g)
    adv = torch.randn(rows, 1, device="cuda", generator=g)
    vt = torch.randn(rows, 1, device="cuda", generator=g)
    lp = _off_kinks(actor, s, a, lp)
    lrn = NativePPO2Learner(_as(actor, torch.float32, "cuda"), _as(critic, torch.float32, "cuda"),
                            dict(DEFAULT_PPO_MSG, update_kernels=kernels), device="cuda")
    f16x3 = net == "lidar" and kernels == "auto"
    assert lrn.net_a.dense != f16x3 and lrn.net_c.dense != f16x3
    assert lrn.net_a.ext == f16x3 and lrn.net_c.ext == f16x3
    assert lrn.net_a.fused == (net == "soi") and lrn.net_c.fused == (net == "soi")  # fg_grad_kernel
    lrn.grads(s, a, lp, adv, vt)
    gn = [lrn.net_a.grad.double().cpu().numpy(), lrn.net_c.grad.double().cpu().numpy()]
    g2 = [lrn.net_a.grad.clone(), lrn.net_c.grad.clone()]
    loss1 = lrn.loss.clone()
    lrn.grads(s, a, lp, adv, vt)
    assert torch.equal(g2[0], lrn.net_a.grad) and torch.equal(g2[1], lrn.net_c.grad)  # fixed order
    assert torch.equal(loss1, lrn.loss)   # the loss sums too (per-block partials, fixed order)
    t64 = _loss_grads(_as(actor, torch.float64, "cuda"), _as(critic, torch.float64, "cuda"),
                      *(x.double() for x in (s, a, lp, adv, vt)))
    t32 = _loss_grads(_as(actor, torch.float32, "cuda"), _as(critic, torch.float32, "cuda"),
                      s, a, lp, adv, vt)
    for i, name in enumerate(("actor", "critic")):
        _f32_class(f"{net} {kernels} {rows} {name}", gn[i], t32[i], t64[i])


@pytest.mark.parametrize("kink,adv_sign", [(+1, +1), (-1, -1)])
def test_soi_grad_at_clip_kink(kink, adv_sign):
    """A row whose float64 ratio lies exactly on a clip kink, where the two branches of torch.min /
    clamp give the row its whole term or none (upper kink with adv > 0, lower kink with adv < 0):
    the fused SOI-net gradient is one of the two float64 candidates (the row's old log-prob 1e-6
    inside / outside the kink), within 4x torch float32's error of it."""
    mk_a, mk_c, S, Ad = NETS["soi"]
    torch.manual_seed(11)
    actor, critic = mk_a(), mk_c()
    with torch.no_grad():
        nn.init.orthogonal_(actor.mean_layer.weight, gain=1.0)
    rows, row = 777, 300
    g = torch.Generator(device="cuda").manual_seed(5)
    s = torch.rand(rows, S, device="cuda", generator=g) * 4 - 2
    with torch.no_grad():
        mean = _as(actor, torch.float32, "cuda")(s)
    a = (mean + 0.7 * torch.randn(rows, Ad, device="cuda", generator=g)).clamp(-3, 3)
    lp = Normal(mean, 1.0).log_prob(a) + 0.3 * torch.randn(rows, Ad, device="cuda", generator=g)
    adv = torch.randn(rows, 1, device="cuda", generator=g)
    vt = torch.randn(rows, 1, device="cuda", generator=g)
    lp = _off_kinks(actor, s, a, lp)
    with torch.no_grad():
        d = _as(actor, torch.float64, "cuda").get_dist(s.double())
        lp_now = d.log_prob(a.double()).sum(1)
        lp64 = lp.double().clone()
        # the row's summed old log-prob on the kink: shift its first component
        lp64[row, 0] += (lp_now[row] - np.log(1 + kink * 0.2)) - lp64[row].sum()
        adv[row, 0] = adv_sign * (abs(float(adv[row, 0])) + 0.5)
    lp = lp64.float()
    a64, c64 = _as(actor, torch.float64, "cuda"), _as(critic, torch.float64, "cuda")
    cands = []
    for delta in (-1e-6, 1e-6):
        l2 = lp64.clone()
        l2[row, 0] += delta
        cands.append(_loss_grads(a64, c64, s.double(), a.double(), l2, adv.double(), vt.double())[0])
    t32 = _loss_grads(_as(actor, torch.float32, "cuda"), _as(critic, torch.float32, "cuda"),
                      s, a, lp, adv, vt)[0]
    lrn = NativePPO2Learner(_as(actor, torch.float32, "cuda"), _as(critic, torch.float32, "cuda"),
                            dict(DEFAULT_PPO_MSG), device="cuda")
    lrn.grads(s, a, lp, adv, vt)
    gn = lrn.net_a.grad.double().cpu().numpy()
    errs = [np.abs(gn - c).max() for c in cands]
    e32 = min(np.abs(t32 - c).max() for c in cands)
    floor = 2e-6 * max(np.abs(c).max() for c in cands)
    assert np.abs(cands[0] - cands[1]).max() > 10 * floor   # the branches do differ here
    assert min(errs) <= 4 * e32 + floor, (errs, e32, floor)


def test_dense_learner_matches_reference_soi_learn(golden):
    """The PPO2-SOI demo's nets: NativePPO2Learner (dense path) from the reference's
    before-weights on its buffer (normalised advantages and v_target as learn() computed them):
    first-step gradients against the reference's own p.grad, and the after-weights of K = 3
    full-batch epochs."""
    g = golden("ppo2_soi_learn")

    def nets(device):
        actor, critic = SoiActor(init_std=float(g["std"])), SoiCritic()
        _load(actor, g["before_actor"])
        _load(critic, g["before_critic"])
        return actor.to(device), critic.to(device)
    t = lambda k, w=1: torch.as_tensor(g[k], dtype=torch.float32, device="cuda").reshape(-1, w)
    s, a, lp, adv, vt = t("s", 4), t("a", 2), t("a_lp", 2), t("adv_norm"), t("v_target")
    msg = dict(DEFAULT_PPO_MSG, K_epochs=3, gamma=0.99)
    actor, critic = nets("cuda")
    lrn = NativePPO2Learner(actor, critic, msg, device="cuda")
    assert lrn.net_a.dense and lrn.net_c.dense
    lrn.grads(s, a, lp, adv, vt)
    a64, c64 = (_as(m, torch.float64, "cpu") for m in nets("cpu"))
    t64 = _loss_grads(a64, c64, *(x.double().cpu() for x in (s, a, lp, adv, vt)))
    for name, net, truth in (("actor", lrn.net_a, t64[0]), ("critic", lrn.net_c, t64[1])):
        ref = g[f"grad_{name}"].astype(np.float64)
        e32 = np.abs(ref - truth).max()
        en = np.abs(net.grad.double().cpu().numpy() - truth).max()
        floor = 2e-6 * np.abs(truth).max()
        assert en <= 4 * e32 + floor, (name, en, e32)
    actor, critic = nets("cuda")
    lrn = NativePPO2Learner(actor, critic, msg, device="cuda")
    lrn.update(s, a, lp, adv, vt)
    torch.cuda.synchronize()
    for name, m in (("actor", actor), ("critic", critic)):
        got = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        np.testing.assert_allclose(got, g[f"after_{name}"], rtol=1e-5, atol=2e-6, err_msg=name)


def test_learner_matches_reference_ugvoa_learn(golden):
    """The PPO2-UGVForwardObstacleAvoidance demo's 41 -> 256 -> 256 nets with the demo's K = 25
    (tests/golden/ppo2_ugvoa_learn.npz, made by running the reference's learn()): first-step
    gradients within 4x the reference's own f32 error of float64, and the after-weights of the 25
    full-batch epochs (rtol 1e-5 / atol 2e-6 per 3 Adam steps, growing with sqrt(steps) as in
    tests/test_learn_golden.py)."""
    g = golden("ppo2_ugvoa_learn")
    K = int(g["K"])
    lo, hi = tuple(float(x) for x in g["a_min"]), tuple(float(x) for x in g["a_max"])

    def nets(device):
        actor = SoiActor(a_min=lo, a_max=hi, init_std=g["std"], S=41, widths=(256, 256))
        critic = SoiCritic(S=41, widths=(256, 256))
        _load(actor, g["before_actor"])
        _load(critic, g["before_critic"])
        return actor.to(device), critic.to(device)
    t = lambda k, w=1: torch.as_tensor(g[k], dtype=torch.float32, device="cuda").reshape(-1, w)
    s, a, lp, adv, vt = t("s", 41), t("a", 2), t("a_lp", 2), t("adv_norm"), t("v_target")
    msg = dict(DEFAULT_PPO_MSG, K_epochs=K, gamma=0.99, a_lr=1e-4, c_lr=1e-3)
    actor, critic = nets("cuda")
    lrn = NativePPO2Learner(actor, critic, msg, device="cuda")
    lrn.grads(s, a, lp, adv, vt)
    a64, c64 = (_as(m, torch.float64, "cpu") for m in nets("cpu"))
    t64 = _loss_grads(a64, c64, *(x.double().cpu() for x in (s, a, lp, adv, vt)))
    for name, net, truth in (("actor", lrn.net_a, t64[0]), ("critic", lrn.net_c, t64[1])):
        ref = g[f"grad_{name}"].astype(np.float64)
        e32 = np.abs(ref - truth).max()
        en = np.abs(net.grad.double().cpu().numpy() - truth).max()
        floor = 2e-6 * np.abs(truth).max()
        print(f"ugvoa {name}: native {en:.3e} reference f32 {e32:.3e} floor {floor:.3e}")
        assert en <= 4 * e32 + floor, (name, en, e32)
    actor, critic = nets("cuda")
    lrn = NativePPO2Learner(actor, critic, msg, device="cuda")
    lrn.update(s, a, lp, adv, vt)
    torch.cuda.synchronize()
    atol = 2e-6 * np.sqrt(K / 3)
    for name, m in (("actor", actor), ("critic", critic)):
        got = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        np.testing.assert_allclose(got, g[f"after_{name}"], rtol=1e-5, atol=atol, err_msg=name)


# ---------------------------------------------------------------------------------------------
# (3) plain-layout rollout
# ---------------------------------------------------------------------------------------------
def _flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()]).float().contiguous()


@pytest.mark.parametrize("variant", ["env", "dppo2"])
def test_plain_rollout_soi_demo_nets_teacher_forced(variant):
    from test_gpu_rollout_parity import (_check_physics, _oracle_forced, bound, bound_rows, host,
                                         policy_bounds)
    kind = A.RLP_ENV_SOI
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind, variant)
    torch.manual_seed(3)
    actor, critic = SoiActor(), SoiCritic()
    with torch.no_grad():
        nn.init.orthogonal_(actor.mean_layer.weight, gain=1.0)
    ad = A.MLPDesc.make([4, 128, 64, 32, 2], [1, 1, 1, 1])
    cd = A.MLPDesc.make([4, 64, 64, 1], [1, 1, 0])
    ap, cp = _flat(actor), _flat(critic)
    lo, hi = A.action_bounds(kind, p)
    std = [(h_ - l_) / 6 for l_, h_ in zip(lo, hi)]
    n, T = 4096 + 37, 64
    cfg = K.make_rollout_cfg(T, n, 3407, 0, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE,
                             A.timeout_flag(kind), plain=True)
    st = K.new_state(kind, n)
    need = torch.ones(n, dtype=torch.uint8, device="cuda")
    g = []
    for seg in range(2):
        cfg.step0 = seg * T
        bufs = K.rollout_buffers(kind, T, n)
        K.rollout(kind, p, st, need, ad, ap.cuda(), cd, cp.cuda(), cfg, bufs)
        g.append({k: host(v) for k, v in bufs.items()})
    torch.cuda.synchronize()
    gst, gneed = host(st), host(need)
    assert g[0]["done"].any() or g[1]["done"].any()
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g, ad, ap.numpy(), cd, cp.numpy())
    _check_physics(kind, g, o, gst, ost, gneed, oneed, f"SOI {variant} plain nets")
    for gb, ob in zip(g, o):
        a_tol, lp_tol = policy_bounds(ad, ap.numpy(), gb["obs"], ob["action"], lo, hi, std)
        bound_rows(gb["action"], ob["action"], 1e-5, a_tol, "action")
        bound_rows(gb["logp"], ob["logp"], 1e-5, lp_tol, "log-prob")
        bound(gb["value"], ob["value"], 1e-5, 2e-6, "V(s)")
        nd = gb["done"] == 0
        bound(gb["value_next"][nd], ob["value_next"][nd], 1e-5, 2e-6, "V(s')")


def test_vec_ppo2_soi_demo_nets():
    """VecPPO2 on the PPO2-SOI demo's nets: the plain-layout rollout, the value fix-up through
    the generic forward, GAE and K epochs of the dense native update; the rollout's nets follow
    the learner (the second segment's actions differ)."""
    from reinforcementlearningplatform_amd.environment.SecondOrderIntegration.SecondOrderIntegration \
        import SecondOrderIntegration
    env = SecondOrderIntegration(n_envs=2048, seed=4)
    env.reset(random=True)
    torch.manual_seed(1)
    agent = VecPPO2(env, SoiActor(), SoiCritic(), {'K_epochs': 3, 'gamma': 0.99}, T=64)
    assert agent.plain and type(agent.learner).__name__ == "NativePPO2Learner"
    assert agent.learner.net_a.dense and agent.learner.net_c.dense
    a0 = None
    checked = 0
    for it in range(4):   # 4 x 64 steps: the envs still running at 250 steps (time_max 5 s) time out
        agent.rollout()
        agent.advantages()
        # V(s') of the done && !success rows (time-outs) comes from the masked generic forward:
        # the critic on obs_next, against a float64 torch forward of the same critic
        b = agent.bufs
        assert torch.isfinite(b["value_next"]).all()
        m = (b["done"].bool() & ~b["success"].bool()).view(-1)
        if m.any():
            x = b["obs_next"].view(-1, env.state_dim)[m].double()
            ref = copy.deepcopy(agent.critic).double()(x).view(-1)
            got = b["value_next"].view(-1)[m].double()
            torch.testing.assert_close(got, ref, rtol=1e-5, atol=2e-6)
            checked += int(m.sum())
        al, cl = agent.update()
        assert torch.isfinite(al) and torch.isfinite(cl)
        if it == 0:
            a0 = agent.bufs["action"].clone()
    assert checked > 0
    assert not torch.equal(a0, agent.bufs["action"])
