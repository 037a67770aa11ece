"""NativePPO2Learner — the K-epoch PPO2 update (Proximal_Policy_Optimization2.learn,
algorithm/policy_base/Proximal_Policy_Optimization2.py:102-174) on librlp's HIP kernels.

Per optimiser step and net: rlp_mfma_pack (packed weights), rlp_ppo2_grad (forward + loss
gradient + backward + weight gradients on MFMA, include/rlp.h) — or, for nets those f16x3 kernels
do not take (the PPO2-SOI demo's 4-128-64-32 actor / 4-64-64 critic, the 41-input lidar nets),
rlp_ppo2_dense_grad on exact f32 MFMA GEMMs — optional RCCL all-reduce of the
actor+critic gradients (one flat buffer, as PPO2Learner), rlp_grad_sqnorm + rlp_adam_step
(clip_grad_norm_ and torch.optim.Adam, evaluated on the device). Same interface and semantics as
PPO2Learner (vec_ppo2.py), which stays as the torch-autograd reference the parity tests compare
against.

The modules' parameters become views of the learner's flat fp32 buffers, so `actor.state_dict()`
(save_ac), GPUNet.refresh and evaluation see every update without a copy.

msg keys beyond the reference's ppo_msg (all optional):
  update_rule     'ppo2' (Proximal_Policy_Optimization2.learn) or 'dppo2' (the DPPO2 Worker.learn,
                  demonstration/DPPO2/DPPO2-4-CartPole/Distributed_PPO2.py:54-103: the local nets
                  stay frozen for the k_epo epochs, so every epoch's gradient is the same one; it
                  is ADDED to the local .grad buffers, which are never zeroed — SharedAdam's
                  zero_grad() only drops the global nets' aliases — clipped in place, and the
                  global nets take one Adam step on the accumulated buffer per epoch; the buffer
                  carries over to the next learn())
  grad_clip_norm  clip_grad_norm_'s max_norm (PPO2 0.5, :150; DPPO2 CartPole/SOI copies 0.2)
  adam_betas      (0.9, 0.999) for torch.optim.Adam; SharedAdam's default is (0.9, 0.99)
                  (utils/classes.py:676-679), which every DPPO2 driver uses
  update_kernels  'auto' (f16x3 FD + wgrad kernels where they take the net: [S -> 256 -> 256 -> A],
                  S <= 8 or the lidar demos' 41; exact-f32 dense GEMMs otherwise) or 'dense' (the
                  dense GEMM path for every net: A/B and tests)
"""
import numpy as np
import torch
import torch.nn as nn

from ... import _abi
from ... import kernels as K


def _linears(module):
    lin = [m for m in module.modules() if isinstance(m, nn.Linear)]
    dims = [lin[0].in_features] + [l.out_features for l in lin] if lin else []
    return lin, dims


def native_fits(module, is_actor):
    """True when librlp's f16x3 update kernels (rlp_ppo2_grad) take the net: a
    [S -> 256 -> 256 -> A<=4] Linear stack, S <= 8 (the drivers' envs) or 41..44 (the lidar demos'
    4 + 37 inputs: layer 1 on the exact-f32 GEMM beside the f16x3 kernels), whose forward is what
    those kernels differentiate —
    tanh hidden layers, the actor's tanh(z) * gain + off head or the critic's linear head (the same
    probe-forward check as dense_fits: a ReLU 256-256 net has the shape but not the arithmetic)."""
    lin, dims = _linears(module)
    shape = (len(lin) == 3 and dims[1] == 256 and dims[2] == 256 and dims[3] <= 4
             and (dims[0] <= 8 or 41 <= dims[0] <= 44))
    return shape and dense_fits(module, is_actor)


def dense_fits(module, is_actor):
    """True when rlp_ppo2_dense_grad takes the net: Linear layers that chain, tanh after every
    hidden layer, the actor's output tanh(z) * gain + off (A <= 4), the critic's linear (one
    output), widths <= 1024 — checked against the module's own forward on a probe batch (the
    PPO2-SOI demo's 4-128-64-32-A actor / 4-64-64-1 critic, the 41-input lidar nets)."""
    lin, dims = _linears(module)
    if not lin or len(lin) > _abi.RLP_MLP_MAX_LAYERS or max(dims) > 1024:
        return False
    if any(a.out_features != b.in_features for a, b in zip(lin[:-1], lin[1:])):
        return False
    if (is_actor and dims[-1] > 4) or (not is_actor and dims[-1] != 1):
        return False
    dev = lin[0].weight.device
    x = torch.rand(64, dims[0], generator=torch.Generator().manual_seed(0)).to(dev) * 4 - 2
    with torch.no_grad():
        h = x
        for i, l in enumerate(lin):
            h = l(h)
            if i < len(lin) - 1:
                h = torch.tanh(h)
        if is_actor:
            gain, off = getattr(module, "gain", None), getattr(module, "off", None)
            if not (torch.is_tensor(gain) and torch.is_tensor(off)):
                return False
            h = torch.tanh(h) * gain.to(dev) + off.to(dev)
        try:
            ref = module(x)
        except Exception:
            return False
    return ref.shape == h.shape and bool(torch.allclose(ref, h, rtol=1e-5, atol=1e-6))


def _update_kind(module, is_actor, kernels="auto"):
    """'f16x3' (rlp_ppo2_grad) or 'dense' (rlp_ppo2_dense_grad); ValueError for any other net.
    kernels='dense' takes the dense GEMM path for nets both paths take (A/B, tests)."""
    if kernels not in ("auto", "dense"):
        raise ValueError(f"NativePPO2Learner: update_kernels {kernels!r} (auto | dense)")
    if kernels == "auto" and native_fits(module, is_actor):
        return "f16x3"
    if dense_fits(module, is_actor):
        return "dense"
    raise ValueError(f"NativePPO2Learner: needs a Linear/Tanh stack (got {_linears(module)[1]} or a "
                     f"forward that is not tanh hidden layers + "
                     f"{'tanh * gain + off' if is_actor else 'linear'} output)")


class _Net:
    def __init__(self, module, is_actor, device, kernels="auto"):
        lin, dims = _linears(module)
        # f16x3: rlp_ppo2_grad (FD + wgrad kernels); dense: rlp_ppo2_dense_grad (f32 MFMA GEMMs)
        self.dense = _update_kind(module, is_actor, kernels) == "dense"
        # the 41-input nets' f16x3 path takes contiguous rows (mini-batches gathered first)
        self.ext = not self.dense and dims[0] > 8
        # rlp_ppo2_dense_grad's fused per-row kernel takes the SOI demo's nets (rlp_dense.hip,
        # ppo2_fused_kind); other dense nets go through its chunked GEMMs
        self.fused = self.dense and dims[0] <= 8 and dims[-1] <= 4 and list(dims[1:-1]) in ([128, 64, 32], [64, 64])
        acts = [_abi.RLP_ACT_TANH] * (len(lin) - 1) + [
            _abi.RLP_ACT_TANH if is_actor else _abi.RLP_ACT_NONE]
        self.desc = _abi.MLPDesc.make(dims, acts)
        params = [p for l in lin for p in (l.weight, l.bias)]
        self.flat = torch.cat([p.detach().reshape(-1).to(device, torch.float32)
                               for p in params]).contiguous()
        off = 0
        for p in params:  # the module's parameters are views of the flat buffer from now on
            p.data = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.grad = torch.zeros_like(self.flat)
        self.acc = None        # the DPPO2 Worker's persistent local gradient buffer
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.packed = None if self.dense else K.mfma_pack(self.desc, self.flat)
        self.sqnorm = torch.zeros(1, dtype=torch.float64, device=device)
        self.step = 0


class NativePPO2Learner:
    """PPO2Learner on librlp's kernels; synchronous data parallelism under torch.distributed."""

    def __init__(self, actor, critic, msg, process_group=None, device=None):
        self.msg = msg
        self.device = torch.device(device) if device is not None else next(actor.parameters()).device
        self.actor, self.critic = actor.to(self.device), critic.to(self.device)
        for name in ("a_min", "a_max", "off", "gain", "std"):
            v = getattr(self.actor, name, None)
            if torch.is_tensor(v):
                setattr(self.actor, name, v.to(self.device))
        kernels = msg.get('update_kernels', 'auto')
        _update_kind(self.actor, True, kernels)    # both nets checked before any device work
        _update_kind(self.critic, False, kernels)
        self.net_a = _Net(self.actor, True, self.device, kernels)
        self.net_c = _Net(self.critic, False, self.device, kernels)
        self.pg = process_group
        self.distributed = process_group is not None or (
            torch.distributed.is_available() and torch.distributed.is_initialized()
            and torch.distributed.get_world_size() > 1)
        self.world = torch.distributed.get_world_size(process_group) if self.distributed else 1
        if self.distributed:
            self.broadcast_params()
        self.lr = {"a": msg['a_lr'], "c": msg['c_lr']}
        self.eps = 1e-5 if msg['set_adam_eps'] else 1e-8
        self.betas = tuple(msg.get('adam_betas', (0.9, 0.999)))
        self.max_norm = float(msg.get('grad_clip_norm', 0.5))
        self.rule = msg.get('update_rule', 'ppo2')
        if self.rule not in ('ppo2', 'dppo2'):
            raise ValueError(f"NativePPO2Learner: update_rule {self.rule!r} (ppo2 | dppo2)")
        self.loss = torch.zeros(2, dtype=torch.float64, device=self.device)
        self.ws = None
        self.total_steps = 0

    # same accessors as PPO2Learner
    def params(self):
        return list(self.actor.parameters()) + list(self.critic.parameters())

    def broadcast_params(self):
        src = 0 if self.pg is None else torch.distributed.get_global_rank(self.pg, 0)
        flat = torch.cat([self.net_a.flat, self.net_c.flat])
        torch.distributed.broadcast(flat, src=src, group=self.pg)
        na = self.net_a.flat.numel()
        self.net_a.flat.copy_(flat[:na])
        self.net_c.flat.copy_(flat[na:])

    def _actor_cfg(self):
        A = self.net_a.desc.dims[self.net_a.desc.n_layers]
        std = np.broadcast_to(torch.as_tensor(self.actor.std, dtype=torch.float32).reshape(-1)
                              .cpu().numpy(), (A,))
        lo = torch.as_tensor(self.actor.a_min, dtype=torch.float32).reshape(-1).cpu().numpy()
        hi = torch.as_tensor(self.actor.a_max, dtype=torch.float32).reshape(-1).cpu().numpy()
        lo, hi = np.broadcast_to(lo, (A,)), np.broadcast_to(hi, (A,))
        return K.ppo2_loss_cfg(_abi.RLP_LOSS_ACTOR, self.msg['eps_clip'], self.msg['entropy_coef'],
                               std, lo, hi)

    def _workspace(self, rows):
        import ctypes
        need = max((K.lib().rlp_ppo2_dense_workspace_floats if n.dense else
                    K.lib().rlp_ppo2_workspace_floats)(ctypes.byref(n.desc), rows)
                   for n in (self.net_a, self.net_c))
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(int(need), dtype=torch.float32, device=self.device)
        return self.ws

    def _net_grad(self, net, cfg, s, index, ws, loss, **kw):
        if (net.dense or net.ext) and index is not None:   # contiguous rows: gather the mini-batch
            s = s.index_select(0, index)
            kw = {k: v.index_select(0, index) for k, v in kw.items()}
            index = None
        if net.dense:   # plain layout
            K.ppo2_dense_grad(net.desc, net.flat, cfg, s, grad=net.grad, loss_sum=loss,
                              workspace=ws, **kw)
        else:
            K.mfma_pack(net.desc, net.flat, out=net.packed)
            K.ppo2_grad(net.desc, net.packed, cfg, s, index=index, grad=net.grad, loss_sum=loss,
                        workspace=ws, **kw)

    def grads(self, s, a, a_lp, adv, vt, index=None, actor_cfg=None):
        """Gradients of one step's actor and critic losses into net.grad (no optimiser step).
        actor_cfg: the loss constants (_actor_cfg()) when the caller already holds them — reading
        the actor's std / bounds from device tensors is a host synchronisation, which update()
        pays once per call instead of once per optimiser step."""
        rows = int(index.shape[0]) if index is not None else int(s.shape[0])
        ws = self._workspace(rows)
        self.loss.zero_()
        adv, vt = adv.reshape(-1), vt.reshape(-1)
        self._net_grad(self.net_a, actor_cfg if actor_cfg is not None else self._actor_cfg(), s,
                       index, ws, self.loss[0:1], a=a, a_logprob=a_lp, adv=adv)
        self._net_grad(self.net_c, K.ppo2_loss_cfg(_abi.RLP_LOSS_CRITIC), s, index, ws,
                       self.loss[1:2], v_target=vt)
        return rows

    def _allreduce_grads(self):
        flat = torch.cat([self.net_a.grad, self.net_c.grad])
        torch.distributed.all_reduce(flat, group=self.pg)
        flat /= self.world
        na = self.net_a.grad.numel()
        self.net_a.grad.copy_(flat[:na])
        self.net_c.grad.copy_(flat[na:])

    def _adam(self, net, lr, grad, clip_sqnorm=None):
        net.step += 1
        K.adam_step(net.flat, grad, net.exp_avg, net.exp_avg_sq, lr, net.step, beta1=self.betas[0],
                    beta2=self.betas[1], eps=self.eps, clip_sqnorm=clip_sqnorm,
                    max_norm=self.max_norm)

    def step(self, s, a, a_lp, adv, vt, index=None, actor_cfg=None):
        rows = self.grads(s, a, a_lp, adv, vt, index, actor_cfg)
        if self.distributed:
            self._allreduce_grads()
        clip = self.msg['use_grad_clip']
        for net, lr in ((self.net_a, self.lr["a"]), (self.net_c, self.lr["c"])):
            sq = None
            if clip:  # clip_grad_norm_(params, max_norm), :150-151 / :158-159
                net.sqnorm.zero_()
                K.grad_sqnorm(net.grad, net.sqnorm)
                sq = net.sqnorm
            self._adam(net, lr, net.grad, sq)
        return self.loss[0] / rows, self.loss[1] / rows

    def _update_dppo2(self, s, a, a_lp, adv, vt):
        """Worker.learn (DPPO2-4-CartPole/Distributed_PPO2.py:76-103): one gradient at the frozen
        local nets, then per epoch: local.grad += g, clip_grad_norm_ in place, global Adam step."""
        rows = self.grads(s, a, a_lp, adv, vt)
        if self.distributed:
            self._allreduce_grads()
        for _ in range(self.msg['K_epochs']):
            for net, lr in ((self.net_a, self.lr["a"]), (self.net_c, self.lr["c"])):
                if net.acc is None:
                    net.acc = torch.zeros_like(net.grad)
                net.acc += net.grad
                if self.msg['use_grad_clip']:
                    net.sqnorm.zero_()
                    K.grad_sqnorm(net.acc, net.sqnorm)
                    K.grad_clip(net.acc, net.sqnorm, self.max_norm)
                self._adam(net, lr, net.acc)
        return self.loss[0] / rows, self.loss[1] / rows

    def update(self, s, a, a_lp, adv, vt, generator=None, perms=None):
        """K epochs over the batch. perms (optional, one index tensor per epoch) replays recorded
        SubsetRandomSampler permutations (mini-batch mode); otherwise they are drawn from
        `generator`."""
        m = self.msg
        N = s.shape[0]
        losses = None
        s, a, a_lp = s.contiguous(), a.contiguous(), a_lp.contiguous()
        adv, vt = adv.reshape(-1).contiguous(), vt.reshape(-1).contiguous()
        if self.rule == 'dppo2':
            return self._update_dppo2(s, a, a_lp, adv, vt)
        acfg = self._actor_cfg()  # one host read of std / bounds for all K epochs
        for k in range(m['K_epochs']):
            if m['using_mini_batch']:
                perm = (perms[k].to(s.device) if perms is not None else
                        torch.randperm(N, device=s.device, generator=generator))
                mb = m['mini_batch_size']
                for i in range(0, N, mb):  # BatchSampler(..., drop_last=False)
                    losses = self.step(s, a, a_lp, adv, vt, index=perm[i:i + mb].contiguous(),
                                       actor_cfg=acfg)
            else:
                losses = self.step(s, a, a_lp, adv, vt, actor_cfg=acfg)
        return losses

    def lr_decay(self, total_steps):
        """Proximal_Policy_Optimization2.lr_decay (:165-174): lr unchanged once total_steps
        reaches max_train_steps."""
        if not self.msg['use_lr_decay'] or total_steps >= self.msg['max_train_steps']:
            return
        frac = 1 - total_steps / self.msg['max_train_steps']
        self.lr = {"a": max(self.msg['a_lr'] * frac, 1e-6), "c": max(self.msg['c_lr'] * frac, 1e-6)}
