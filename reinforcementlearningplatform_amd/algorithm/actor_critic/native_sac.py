"""Native SAC update: one learn() iteration (algorithm/actor_critic/Soft_Actor_Critic.py:70-129)
as ONE librlp call, rlp_sac_update (csrc/rlp_dense.hip) — target, actor and critic passes on the
f32-MFMA dense GEMM with fused relu epilogues, the squashed-Gaussian head and its backward as
elementwise kernels, Adam for the actor, the twin critic and log_alpha, and the soft target
update — instead of torch autograd and three optimizers (~250 small kernels per iteration).

Applies to the SAC drivers' nets (SACActor: relu trunk, mean / log_std heads, log_std clamp,
tanh squash with gain / off; SACCritic: twin relu chains on cat(s, a)). The structure is read from
the order the modules' Linear layers run in on a probe batch and accepted only if that
composition reproduces the modules' own forward (actor: deterministic action and, with the
Gaussian noise pinned, the sampled action and log-prob; critic: both heads). Parameters become
views of flat fp32 buffers the kernels update in place. Exploration noise: Philox keyed by
(seed, device counter, row) — or, for replaying a recorded tape, the eps tensors passed in.
"""
import torch
import torch.nn as nn

from ... import _abi
from ... import kernels as K
from .native_ddpg import _FlatNet, _adam_hyper, _linear_chain


def _ls_bounds(actor, A, device):
    if hasattr(actor, "log_std_bounds"):
        lo, hi = actor.log_std_bounds()
    elif getattr(actor, "std_min", None) is not None:
        lo = torch.log(actor.std_min * (actor.a_max - actor.a_min) / 2)
        hi = (actor.a_max - actor.a_min) / 2 / actor.std_scale
    else:
        lo, hi = torch.full((A,), -20.0), torch.full((A,), 2.0)
    f = lambda t: torch.as_tensor(t, dtype=torch.float32).reshape(-1).expand(A).to(device).contiguous()
    return f(lo), f(hi)


class _PinnedNoise:
    def __init__(self, eps):
        self.eps, self.orig = eps, torch.distributions.Normal.rsample

    def __enter__(self):
        eps = self.eps
        torch.distributions.Normal.rsample = lambda d, sample_shape=torch.Size(): d.loc + eps * d.scale
        return self

    def __exit__(self, *a):
        torch.distributions.Normal.rsample = self.orig


def _actor_structure(actor, S, A, device):
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(64, S, generator=g) * 4 - 2).to(device)
    try:
        chain, _ = _linear_chain(actor, x)
    except Exception:
        return None
    if len(chain) < 3 or len(set(map(id, chain))) != len(chain):
        return None
    trunk, (hm, hl) = chain[:-2], chain[-2:]
    if len(trunk) > _abi.RLP_DENSE_MAX_LAYERS or any(l.bias is None for l in chain):
        return None
    dims = [trunk[0].in_features] + [l.out_features for l in trunk]
    if dims[0] != S or any(p.out_features != q.in_features for p, q in zip(trunk[:-1], trunk[1:])):
        return None
    H = dims[-1]
    if (hm.in_features, hm.out_features, hl.in_features, hl.out_features) != (H, A, H, A):
        return None
    if not all(torch.is_tensor(getattr(actor, k, None)) for k in ("gain", "off")):
        return None
    lo, hi = _ls_bounds(actor, A, device)
    gain, off = actor.gain.to(device), actor.off.to(device)
    eps = torch.randn(64, A, generator=g).to(device)
    with torch.no_grad():
        h = x
        for lin in trunk:
            h = torch.relu(lin(h))
        mean = hm(h)
        std = torch.exp(torch.clamp(hl(h), lo, hi))
        u = mean + eps * std
        dist = torch.distributions.Normal(mean, std)
        lp = dist.log_prob(u).sum(1, keepdim=True)
        lp = lp - (2 * (0.6931471805599453 - u - torch.nn.functional.softplus(-2 * u))).sum(1, keepdim=True)
        a_det = torch.tanh(mean) * gain + off
        a_smp = torch.tanh(u) * gain + off
        try:
            ref_det, _ = actor(x, True, False)
            with _PinnedNoise(eps):
                ref_smp, ref_lp = actor(x, False, True)
        except Exception:
            return None
    ok = (torch.allclose(a_det, ref_det, rtol=1e-5, atol=1e-6)
          and torch.allclose(a_smp, ref_smp, rtol=1e-5, atol=1e-6)
          and torch.allclose(lp, ref_lp.reshape(lp.shape), rtol=1e-5, atol=1e-5))
    return (trunk, dims, hm, hl, lo, hi) if ok else None


def _critic_structure(critic, S, A, device):
    g = torch.Generator().manual_seed(1)
    s = (torch.rand(64, S, generator=g) * 4 - 2).to(device)
    a = (torch.rand(64, A, generator=g) * 4 - 2).to(device)
    try:
        chain, out = _linear_chain(critic, s, a)
    except Exception:
        return None
    if not (isinstance(out, tuple) and len(out) == 2) or len(set(map(id, chain))) != len(chain):
        return None
    ends = [i for i, l in enumerate(chain) if l.out_features == 1]
    if len(ends) != 2 or ends[1] != len(chain) - 1:
        return None
    chains = [chain[:ends[0] + 1], chain[ends[0] + 1:]]
    x = torch.cat([s, a], 1)
    res = []
    for c, ref in zip(chains, out):
        if not c or len(c) > _abi.RLP_DENSE_MAX_LAYERS or any(l.bias is None for l in c):
            return None
        dims = [c[0].in_features] + [l.out_features for l in c]
        if dims[0] != S + A or any(p.out_features != q.in_features for p, q in zip(c[:-1], c[1:])):
            return None
        with torch.no_grad():
            h = x
            for i, lin in enumerate(c):
                h = lin(h)
                if i < len(c) - 1:
                    h = torch.relu(h)
        if not torch.allclose(h, ref, rtol=1e-5, atol=1e-6):
            return None
        res.append((c, dims))
    return res


class SACNativeUpdate:
    """rlp_sac_update for a SAC agent's actor / critic / target critic (module docstring)."""

    @staticmethod
    def fits(agent):
        S, A = agent.env_msg['state_dim'], agent.env_msg['action_dim']
        if not 1 <= A <= 4:
            return False
        dev = agent.device
        cs = _critic_structure(agent.critic, S, A, dev)
        ts = _critic_structure(agent.target_critic, S, A, dev)
        if _actor_structure(agent.actor, S, A, dev) is None or cs is None or ts is None:
            return False
        if [d for _, d in cs] != [d for _, d in ts]:
            return False
        opts = [agent.actor_optimizer, agent.critic_optimizer] + (
            [agent.alpha_optimizer] if agent.adaptive_alpha else [])
        return all(_adam_hyper(o) is not None for o in opts)

    def __init__(self, agent):
        S, A = agent.env_msg['state_dim'], agent.env_msg['action_dim']
        dev = agent.device
        self.agent, self.A = agent, A
        ast = _actor_structure(agent.actor, S, A, dev)
        cst = _critic_structure(agent.critic, S, A, dev)
        tst = _critic_structure(agent.target_critic, S, A, dev)
        if ast is None or cst is None or tst is None:
            raise ValueError("native SAC: actor / critic forward is not the structure this update implements")
        trunk, dims, hm, hl, self.ls_lo, self.ls_hi = ast
        self.fa = _FlatNet(agent.actor, trunk, dims, dev)
        off = {id(p): o for p, o in zip(self.fa.params, _offsets(self.fa.params))}
        self.mean_offset, self.log_std_offset = off[id(hm.weight)], off[id(hl.weight)]
        for lin, o in ((hm, self.mean_offset), (hl, self.log_std_offset)):
            if off[id(lin.bias)] != o + lin.weight.numel():
                raise ValueError("native SAC: a head's bias must follow its weight")
        self.fc = _FlatNet(agent.critic, None, None, dev, chains=cst)
        self.ft = _FlatNet(agent.target_critic, None, None, dev, chains=tst)
        if self.ft.chain_nets_offsets != self.fc.chain_nets_offsets or self.ft.flat.numel() != self.fc.flat.numel():
            raise ValueError("native SAC: the target critic must have the critic's parameter layout")
        self.opt = {"actor": _adam_hyper(agent.actor_optimizer),
                    "critic": _adam_hyper(agent.critic_optimizer),
                    "alpha": _adam_hyper(agent.alpha_optimizer) if agent.adaptive_alpha else None}
        if self.opt["actor"] is None or self.opt["critic"] is None or (
                agent.adaptive_alpha and self.opt["alpha"] is None):
            raise ValueError("native SAC: plain torch.optim.Adam optimizers expected")
        z = torch.zeros_like
        self.grad = {"actor": z(self.fa.flat), "critic": z(self.fc.flat)}
        self.m = {"actor": z(self.fa.flat), "critic": z(self.fc.flat)}
        self.v = {"actor": z(self.fa.flat), "critic": z(self.fc.flat)}
        f32 = dict(dtype=torch.float32, device=dev)
        if agent.adaptive_alpha:
            self.log_alpha = agent.log_alpha   # the agent's own leaf tensor, updated in place
        else:
            self.log_alpha = torch.zeros(1, **f32)
        self.alpha_grad, self.alpha_m, self.alpha_v = (torch.zeros(1, **f32) for _ in range(3))
        self.steps = torch.zeros(3, dtype=torch.int32, device=dev)
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self._import_adam_state()
        self.gain = agent.actor.gain.to(dev, torch.float32).contiguous()
        self.off = agent.actor.off.to(dev, torch.float32).contiguous()
        n = _abi.SACNets()
        n.actor = self.fa.net
        n.mean_offset, n.log_std_offset, n.action_dim = self.mean_offset, self.log_std_offset, A
        n.q1, n.q2 = self.fc.chain_nets
        n.target_critic = self.ft.flat.data_ptr()
        for k in ("actor", "critic"):
            setattr(n, f"{k}_grad", self.grad[k].data_ptr())
            setattr(n, f"{k}_m", self.m[k].data_ptr())
            setattr(n, f"{k}_v", self.v[k].data_ptr())
        n.log_alpha, n.alpha_grad = self.log_alpha.data_ptr(), self.alpha_grad.data_ptr()
        n.alpha_m, n.alpha_v = self.alpha_m.data_ptr(), self.alpha_v.data_ptr()
        n.steps, n.counter = self.steps.data_ptr(), self.counter.data_ptr()
        n.gain, n.off = self.gain.data_ptr(), self.off.data_ptr()
        n.ls_lo, n.ls_hi = self.ls_lo.data_ptr(), self.ls_hi.data_ptr()
        self.c_nets = n
        self.losses = torch.zeros(2, **f32)
        self.work, self.batch = None, None

    def _import_adam_state(self):
        ag = self.agent
        pairs = [("actor", ag.actor_optimizer, self.fa.params), ("critic", ag.critic_optimizer, self.fc.params)]
        for i, (k, opt, params) in enumerate(pairs):
            steps, off = set(), 0
            for p in params:
                st = opt.state.get(p, {})
                if st:
                    self.m[k][off:off + p.numel()].copy_(st["exp_avg"].reshape(-1))
                    self.v[k][off:off + p.numel()].copy_(st["exp_avg_sq"].reshape(-1))
                    steps.add(int(st["step"]))
                off += p.numel()
            if len(steps) > 1:
                raise ValueError(f"native SAC: {k} optimizer states disagree on the step count")
            if steps:
                self.steps[i] = steps.pop()
        if ag.adaptive_alpha:
            st = ag.alpha_optimizer.state.get(ag.log_alpha, {})
            if st:
                self.alpha_m.copy_(st["exp_avg"].reshape(-1))
                self.alpha_v.copy_(st["exp_avg_sq"].reshape(-1))
                self.steps[2] = int(st["step"])

    def state_tensors(self):
        """Device state a graph warm-up must restore."""
        return [self.m["actor"], self.v["actor"], self.m["critic"], self.v["critic"], self.alpha_m,
                self.alpha_v, self.steps, self.counter]

    def _cfg(self, B):
        ag = self.agent
        c = _abi.SACCfg()
        c.batch, c.adaptive_alpha = int(B), int(bool(ag.adaptive_alpha))
        c.gamma, c.tau = float(ag.gamma), float(ag.tau)
        c.target_entropy = float(getattr(ag, "target_entropy", 0.0))
        c.alpha = 0.0 if ag.adaptive_alpha else float(ag.alpha)
        c.seed = int(ag.seed)
        for k, dst in (("actor", c.actor_adam), ("critic", c.critic_adam), ("alpha", c.alpha_adam)):
            g = self.opt[k]
            if g is not None:
                dst.lr, dst.beta1, dst.beta2, dst.eps = g["lr"], g["betas"][0], g["betas"][1], g["eps"]
        return c

    def update(self, s, a, r, s_, dw, noise=None, out=None):
        """noise: None (Philox) or [2][B][A] eps (s' draw, then s draw). out: a float32 [2]
        device tensor to receive (critic loss, actor loss) (no copies); else fresh tensors."""
        B = int(s.shape[0])
        if self.work is None or self.batch != B:
            self.work = K.sac_workspace(self.c_nets, B, s.device)
            self.batch = B
        f = lambda t: t.to(torch.float32).contiguous()
        s, a, r, s_, dw = f(s), f(a), f(r).reshape(-1), f(s_), f(dw).reshape(-1)
        nz = None if noise is None else f(noise)
        with torch.no_grad():
            K.sac_update(self.c_nets, self._cfg(B), s, a, r, s_, dw, nz, self.work,
                         out if out is not None else self.losses)
        if out is not None:
            return out[0], out[1]
        out = self.losses.clone()   # fresh tensors: self.losses is rewritten by the next call
        return out[0], out[1]


def _offsets(params):
    out, off = [], 0
    for p in params:
        out.append(off)
        off += p.numel()
    return out
