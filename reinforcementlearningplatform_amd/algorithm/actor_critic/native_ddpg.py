"""Native DDPG update: one learn() iteration (algorithm/actor_critic/DDPG.py:83-109 and the soft
update :111-118) as ONE librlp call, rlp_ddpg_update (csrc/rlp_dense.hip): the target, critic
and actor passes on v_mfma_f32_16x16x4_f32 GEMMs with fused bias / relu / tanh epilogues, the
weight gradients reduced in a fixed order, torch.optim.Adam's arithmetic and the soft target
updates — instead of torch autograd + two Adam optimizers (~100 small kernels).

Applies to the drivers' nets (demonstration/DDPG/DDPG-4-*/train.py:26-100): an actor whose forward
is relu(Linear) ... then gain * tanh(Linear) + off, a critic whose forward is relu(Linear(cat(s, a)))
... then Linear. The chain is found by recording the order the module's Linear layers run in on a
probe batch, and accepted only if that composition reproduces the module's own forward on the probe
(`DDPGNativeUpdate.fits`). The modules' parameters become views of flat fp32 buffers the kernels
update in place, so `state_dict()`, `save_ac` and the torch forward see every step. Parameters the
forward does not reach (the drivers' critic.action_value) keep a zero gradient: Adam leaves them
unchanged, as torch skips parameters without .grad, and the soft update still blends them.
"""
import torch
import torch.nn as nn
import torch.nn.functional as func

from ... import _abi
from ... import kernels as K


def _linear_chain(module, *args):
    """(Linear layers in the order the forward runs them, output) on a probe input."""
    seen = []
    hooks = [m.register_forward_hook(lambda m, i, o: seen.append(m))
             for m in module.modules() if isinstance(m, nn.Linear)]
    try:
        with torch.no_grad():
            out = module(*args)
    finally:
        for h in hooks:
            h.remove()
    return seen, out


def _compose(chain, x, head):
    with torch.no_grad():
        for l, lin in enumerate(chain):
            x = lin(x)
            if l < len(chain) - 1:
                x = func.relu(x)
        return head(x)


def _chain_of(module, is_actor, S, A, device):
    """The Linear chain of a driver net if its forward is the composition this update implements,
    else None."""
    g = torch.Generator().manual_seed(0)
    s = (torch.rand(64, S, generator=g) * 4 - 2).to(device)
    a = (torch.rand(64, A, generator=g) * 4 - 2).to(device)
    try:
        chain, ref = _linear_chain(module, s) if is_actor else _linear_chain(module, s, a)
    except Exception:
        return None
    if not chain or len(chain) > _abi.RLP_DENSE_MAX_LAYERS or len(set(map(id, chain))) != len(chain):
        return None
    dims = [chain[0].in_features] + [l.out_features for l in chain]
    if any(l.bias is None for l in chain) or any(
            p.out_features != q.in_features for p, q in zip(chain[:-1], chain[1:])):
        return None
    if is_actor:
        if dims[0] != S or dims[-1] != A or not all(
                torch.is_tensor(getattr(module, k, None)) for k in ("gain", "off")):
            return None
        gain, off = module.gain.to(device), module.off.to(device)
        got = _compose(chain, s, lambda z: gain * torch.tanh(z) + off)
    else:
        if dims[0] != S + A or dims[-1] != 1:
            return None
        got = _compose(chain, torch.cat([s, a], 1), lambda z: z)
    if got.shape != ref.shape or not torch.allclose(got, ref.float(), rtol=1e-5, atol=1e-6):
        return None
    return chain, dims


class _FlatNet:
    """A module's parameters as views of one flat fp32 buffer + the rlp_dense_net of its Linear
    chain (or, with `chains`, one rlp_dense_net per chain: e.g. a twin critic)."""

    def __init__(self, module, chain, dims, device, chains=None):
        params = list(module.parameters())
        self.flat = torch.cat([p.detach().reshape(-1).to(device, torch.float32)
                               for p in params]).contiguous()
        offset, off = {}, 0
        for p in params:
            offset[id(p)] = off
            p.data = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.params = params

        def offs_of(ch):
            offs = []
            for lin in ch:
                w, b = offset[id(lin.weight)], offset[id(lin.bias)]
                if b != w + lin.weight.numel():
                    raise ValueError("native update: a Linear's bias must follow its weight in "
                                     "parameters()")
                offs.append(w)
            return offs

        if chains is None:
            self.offsets = offs_of(chain)
            self.net = K.dense_net(self.flat, dims, self.offsets)
        else:
            self.chain_nets_offsets = [offs_of(c) for c, _ in chains]
            self.chain_nets = [K.dense_net(self.flat, d, o)
                               for (_, d), o in zip(chains, self.chain_nets_offsets)]


def _adam_hyper(opt):
    """The single param group of a plain torch.optim.Adam (or AdamW with weight_decay 0: the same
    update), else None — any other optimizer (SGD, RMSprop, NAdam, RAdam, Adamax, ...) keeps the
    torch update path."""
    if type(opt) not in (torch.optim.Adam, torch.optim.AdamW) or len(opt.param_groups) != 1:
        return None
    g = opt.param_groups[0]
    if (g.get("weight_decay", 0) or g.get("amsgrad", False) or g.get("maximize", False)
            or g.get("differentiable", False) or torch.is_tensor(g.get("lr"))):
        return None
    return g


class DDPGNativeUpdate:
    """rlp_ddpg_update for a DDPG agent's four nets (see the module docstring)."""

    @staticmethod
    def fits(agent):
        S, A = agent.env_msg['state_dim'], agent.env_msg['action_dim']
        dev = agent.device
        ca = _chain_of(agent.actor, True, S, A, dev)
        cta = _chain_of(agent.target_actor, True, S, A, dev)
        cc = _chain_of(agent.critic, False, S, A, dev)
        ctc = _chain_of(agent.target_critic, False, S, A, dev)
        if None in (ca, cta, cc, ctc) or ca[1] != cta[1] or cc[1] != ctc[1]:
            return False
        oa, oc = (_adam_hyper(getattr(agent.actor, "optimizer", None)),
                  _adam_hyper(getattr(agent.critic, "optimizer", None)))
        return oa is not None and oc is not None

    def __init__(self, agent):
        S, A = agent.env_msg['state_dim'], agent.env_msg['action_dim']
        dev = agent.device
        self.agent = agent
        chains = {}
        for k, is_actor in (("actor", True), ("target_actor", True), ("critic", False),
                            ("target_critic", False)):
            c = _chain_of(getattr(agent, k), is_actor, S, A, dev)
            if c is None:
                raise ValueError(f"native DDPG: {k}'s forward is not a chain this update implements")
            chains[k] = c
        self.nets = {k: _FlatNet(getattr(agent, k), *chains[k], dev) for k in chains}
        for k, t in (("actor", "target_actor"), ("critic", "target_critic")):
            if (self.nets[k].offsets != self.nets[t].offsets
                    or self.nets[k].flat.numel() != self.nets[t].flat.numel()):
                raise ValueError(f"native DDPG: {t} must have {k}'s parameter layout")
        self.opt = {"actor": _adam_hyper(agent.actor.optimizer),
                    "critic": _adam_hyper(agent.critic.optimizer)}
        if None in self.opt.values():
            raise ValueError("native DDPG: plain torch.optim.Adam optimizers expected")
        f = self.nets["actor"].flat, self.nets["critic"].flat
        self.grad = {"actor": torch.zeros_like(f[0]), "critic": torch.zeros_like(f[1])}
        self.m = {"actor": torch.zeros_like(f[0]), "critic": torch.zeros_like(f[1])}
        self.v = {"actor": torch.zeros_like(f[0]), "critic": torch.zeros_like(f[1])}
        self.steps = torch.zeros(2, dtype=torch.int32, device=dev)
        self._import_adam_state()
        self.gain = agent.actor.gain.to(dev, torch.float32).contiguous()
        self.off = agent.actor.off.to(dev, torch.float32).contiguous()
        n = _abi.DDPGNets()
        n.actor, n.target_actor = self.nets["actor"].net, self.nets["target_actor"].net
        n.critic, n.target_critic = self.nets["critic"].net, self.nets["target_critic"].net
        for k in ("actor", "critic"):
            setattr(n, f"{k}_grad", self.grad[k].data_ptr())
            setattr(n, f"{k}_m", self.m[k].data_ptr())
            setattr(n, f"{k}_v", self.v[k].data_ptr())
        n.steps, n.gain, n.off = self.steps.data_ptr(), self.gain.data_ptr(), self.off.data_ptr()
        self.c_nets = n
        self.losses = torch.zeros(2, dtype=torch.float32, device=dev)
        self.work = None
        self.batch = None

    def _import_adam_state(self):
        """An optimizer that already stepped hands its moments and step count over."""
        for i, k in enumerate(("actor", "critic")):
            opt = getattr(self.agent, k).optimizer
            fn = self.nets[k]
            steps = set()
            off = 0
            for p in fn.params:
                st = opt.state.get(p, {})
                if st:
                    self.m[k][off:off + p.numel()].copy_(st["exp_avg"].reshape(-1))
                    self.v[k][off:off + p.numel()].copy_(st["exp_avg_sq"].reshape(-1))
                    steps.add(int(st["step"]))
                off += p.numel()
            if len(steps) > 1:
                raise ValueError(f"native DDPG: {k} optimizer states disagree on the step count")
            if steps:
                self.steps[i] = steps.pop()

    def state_tensors(self):
        """Device state a graph warm-up must restore (Adam moments and step counts)."""
        return [self.m["actor"], self.v["actor"], self.m["critic"], self.v["critic"], self.steps]

    def _cfg(self, B):
        c = _abi.DDPGCfg()
        c.batch, c.gamma = int(B), float(self.agent.gamma)
        c.actor_tau, c.critic_tau = float(self.agent.actor_tau), float(self.agent.critic_tau)
        for k, dst in (("actor", c.actor_adam), ("critic", c.critic_adam)):
            g = self.opt[k]
            dst.lr, dst.beta1, dst.beta2, dst.eps = g["lr"], g["betas"][0], g["betas"][1], g["eps"]
        return c

    def update(self, s, a, r, s_, end, out=None):
        """out: a float32 [2] device tensor to receive (critic loss, actor loss) — e.g. a
        captured graph's loss buffer (no copies); else fresh tensors."""
        B = int(s.shape[0])
        if self.work is None or self.batch != B:
            self.work = K.ddpg_workspace(self.c_nets, B, s.device)
            self.batch = B
        f = lambda t: t.to(torch.float32).contiguous()
        s, a, r, s_, end = f(s), f(a), f(r).reshape(-1), f(s_), f(end).reshape(-1)
        if out is not None:
            K.ddpg_update(self.c_nets, self._cfg(B), s, a, r, s_, end, self.work, out)
            return out[0], out[1]
        K.ddpg_update(self.c_nets, self._cfg(B), s, a, r, s_, end, self.work, self.losses)
        out = self.losses.clone()   # fresh tensors: self.losses is rewritten by the next call
        return out[0], out[1]
