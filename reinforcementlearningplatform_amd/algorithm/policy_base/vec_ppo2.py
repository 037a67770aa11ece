"""VecPPO2 — PPO2 over a batch of n envs on one GPU: the DPPO2 worker loop
(demonstration/DPPO2/DPPO2-4-CartPole/Distributed_PPO2.py:115-172) with the per-env Python loop
replaced by one fused HIP rollout launch per segment.

One iteration:
  rollout     rlp_rollout: T steps x n envs (reset, actor + sample, critic, env step, append)
  advantages  rlp_value_fixup (V(s') of time-outs), rlp_reward_norm (Normalization), rlp_gae +
              rlp_adv_normalize. Under torch.distributed both statistics are global by default
              (ppo_msg 'norm_scope': 'global'): the ranks' reward chunk statistics and
              advantage (count, mean, M2) partials are gathered (one small all-reduce each) and
              merged in global env order, so W ranks of n envs normalise exactly as one rank of
              W * n envs; 'rank' keeps one normaliser per rank, as each DPPO2 worker keeps its own
  update      K epochs of the PPO2 clipped objective (Proximal_Policy_Optimization2.py:102-160)
              on librlp's kernels (NativePPO2Learner: rlp_ppo2_grad + rlp_adam_step; learner=
              "torch" selects the torch-autograd PPO2Learner below, the parity reference); under
              torch.distributed the actor+critic gradients are averaged in ONE flat all-reduce per
              step (RCCL over xGMI) — synchronous data parallelism instead of the reference's
              Hogwild shared-memory updates.
"""
import numpy as np
import torch
import torch.nn.functional as F

from ... import _abi
from ... import kernels as K
from ...utils.classes import GPUNet

DEFAULT_PPO_MSG = {
    # demonstration/PPO2/PPO2-4-CartPole/train.py:145-161
    'gamma': 0.999, 'K_epochs': 30, 'eps_clip': 0.2, 'a_lr': 3e-4, 'c_lr': 1e-3,
    'set_adam_eps': True, 'lmd': 0.95, 'use_adv_norm': True, 'mini_batch_size': 64,
    'entropy_coef': 0.01, 'use_grad_clip': False, 'use_lr_decay': False,
    'max_train_steps': int(5e6), 'using_mini_batch': False,
}


class PPO2Learner:
    """The K-epoch PPO2 update (Proximal_Policy_Optimization2.py:102-174) on any torch device, with
    synchronous data-parallel gradient averaging under torch.distributed (one flat all-reduce of the
    actor+critic gradients per optimiser step: ~539 KB for the CartPole nets, latency-bound on
    xGMI, so one bucket)."""

    def __init__(self, actor, critic, msg, process_group=None, device=None):
        self.msg = msg
        self.device = torch.device(device) if device is not None else next(actor.parameters()).device
        self.actor, self.critic = actor.to(self.device), critic.to(self.device)
        for name in ("a_min", "a_max", "off", "gain", "std"):
            v = getattr(self.actor, name, None)
            if torch.is_tensor(v):
                setattr(self.actor, name, v.to(self.device))
        self.pg = process_group
        self.distributed = process_group is not None or (
            torch.distributed.is_available() and torch.distributed.is_initialized()
            and torch.distributed.get_world_size() > 1)
        self.world = torch.distributed.get_world_size(process_group) if self.distributed else 1
        if self.distributed:
            self.broadcast_params()
        eps = dict(eps=1e-5) if msg['set_adam_eps'] else {}
        betas = tuple(msg.get('adam_betas', (0.9, 0.999)))   # SharedAdam: (0.9, 0.99)
        self.opt_a = torch.optim.Adam(self.actor.parameters(), lr=msg['a_lr'], betas=betas, **eps)
        self.opt_c = torch.optim.Adam(self.critic.parameters(), lr=msg['c_lr'], betas=betas, **eps)
        self.max_norm = float(msg.get('grad_clip_norm', 0.5))
        self.rule = msg.get('update_rule', 'ppo2')   # see native_ppo2.py's docstring
        if self.rule not in ('ppo2', 'dppo2'):
            raise ValueError(f"PPO2Learner: update_rule {self.rule!r} (ppo2 | dppo2)")
        self.acc = None
        self.total_steps = 0

    def params(self):
        return list(self.actor.parameters()) + list(self.critic.parameters())

    def broadcast_params(self):
        """Every rank starts from rank 0's replica (the reference's global nets)."""
        src = 0 if self.pg is None else torch.distributed.get_global_rank(self.pg, 0)
        with torch.no_grad():
            flat = torch.cat([p.data.reshape(-1) for p in self.params()])
            torch.distributed.broadcast(flat, src=src, group=self.pg)
            off = 0
            for p in self.params():
                p.data.copy_(flat[off:off + p.numel()].view_as(p))
                off += p.numel()

    def _allreduce_grads(self):
        params = [p for p in self.params() if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        torch.distributed.all_reduce(flat, group=self.pg)
        flat /= self.world
        off = 0
        for p in params:
            p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
            off += p.numel()

    def step(self, s, a, a_lp, adv, vt):
        m = self.msg
        dist = self.actor.get_dist(s)
        ent = dist.entropy().sum(1, keepdim=True)
        ratios = torch.exp(dist.log_prob(a).sum(1, keepdim=True) - a_lp.sum(1, keepdim=True))
        surr1 = ratios * adv
        surr2 = torch.clamp(ratios, 1 - m['eps_clip'], 1 + m['eps_clip']) * adv
        actor_loss = (-torch.min(surr1, surr2) - m['entropy_coef'] * ent).mean()
        critic_loss = F.mse_loss(vt, self.critic(s))
        self.opt_a.zero_grad()
        self.opt_c.zero_grad()
        actor_loss.backward()
        critic_loss.backward()   # the critic loss does not depend on the actor: order is free
        if self.distributed:
            self._allreduce_grads()
        if m['use_grad_clip']:
            torch.nn.utils.clip_grad_norm_(self.actor.parameters(), self.max_norm)
            torch.nn.utils.clip_grad_norm_(self.critic.parameters(), self.max_norm)
        self.opt_a.step()
        self.opt_c.step()
        return actor_loss.detach(), critic_loss.detach()

    def _update_dppo2(self, s, a, a_lp, adv, vt):
        """Worker.learn (demonstration/DPPO2/DPPO2-4-CartPole/Distributed_PPO2.py:76-103): the
        local nets are frozen during learn(), so each epoch's gradient is the same; it is added to
        the never-zeroed local .grad buffers, clipped in place, and the global Adam steps on them."""
        m = self.msg
        dist = self.actor.get_dist(s)
        ent = dist.entropy().sum(1, keepdim=True)
        ratios = torch.exp(dist.log_prob(a).sum(1, keepdim=True) - a_lp.sum(1, keepdim=True))
        surr1 = ratios * adv
        surr2 = torch.clamp(ratios, 1 - m['eps_clip'], 1 + m['eps_clip']) * adv
        actor_loss = (-torch.min(surr1, surr2) - m['entropy_coef'] * ent).mean()
        critic_loss = F.mse_loss(vt, self.critic(s))
        pa, pc = list(self.actor.parameters()), list(self.critic.parameters())
        g = list(torch.autograd.grad(actor_loss, pa)) + list(torch.autograd.grad(critic_loss, pc))
        if self.distributed:
            flat = torch.cat([t.reshape(-1) for t in g])
            torch.distributed.all_reduce(flat, group=self.pg)
            flat /= self.world
            off = 0
            for t in g:
                t.copy_(flat[off:off + t.numel()].view_as(t))
                off += t.numel()
        if self.acc is None:
            self.acc = [torch.zeros_like(t) for t in g]
        for _ in range(m['K_epochs']):
            for params, opt, lo in ((pa, self.opt_a, 0), (pc, self.opt_c, len(pa))):
                for j, p in enumerate(params):
                    self.acc[lo + j] += g[lo + j]
                    p.grad = self.acc[lo + j]          # the global nets alias the local grads
                if m['use_grad_clip']:
                    torch.nn.utils.clip_grad_norm_(params, self.max_norm)
                opt.step()
        return actor_loss.detach(), critic_loss.detach()

    def update(self, s, a, a_lp, adv, vt, generator=None, perms=None):
        m = self.msg
        N = s.shape[0]
        losses = None
        if self.rule == 'dppo2':
            return self._update_dppo2(s, a, a_lp, adv, vt)
        for k in range(m['K_epochs']):
            if m['using_mini_batch']:
                perm = (perms[k].to(s.device) if perms is not None else
                        torch.randperm(N, device=s.device, generator=generator))
                mb = m['mini_batch_size']
                for i in range(0, N, mb):  # BatchSampler(..., drop_last=False)
                    idx = perm[i:i + mb]
                    losses = self.step(s[idx], a[idx], a_lp[idx], adv[idx], vt[idx])
            else:
                losses = self.step(s, a, a_lp, adv, vt)
        return losses

    def lr_decay(self, total_steps):
        """Proximal_Policy_Optimization2.lr_decay (:165-174): no change once total_steps reaches
        max_train_steps."""
        if not self.msg['use_lr_decay'] or total_steps >= self.msg['max_train_steps']:
            return
        frac = 1 - total_steps / self.msg['max_train_steps']
        for g, lr in ((self.opt_a, self.msg['a_lr']), (self.opt_c, self.msg['c_lr'])):
            for p in g.param_groups:
                p['lr'] = max(lr * frac, 1e-6)


class VecPPO2:
    def __init__(self, env, actor, critic, ppo_msg=None, T=128, success_rule=None, seed=None,
                 process_group=None, device=None, learner="auto"):
        self.env = env
        self.kind, self.params = env.KIND, env.params
        self.n, self.T = env.n_envs, int(T)
        self.device = torch.device(device) if device is not None else env.device
        self.msg = dict(DEFAULT_PPO_MSG, **(ppo_msg or {}))
        if 'k_epo' in self.msg:                       # DPPO2 drivers name it k_epo
            self.msg['K_epochs'] = self.msg['k_epo']
        if learner not in ("auto", "native", "torch"):
            raise ValueError(f"VecPPO2: learner {learner!r} (auto | native | torch)")
        from .native_ppo2 import NativePPO2Learner, dense_fits
        if learner == "auto":  # librlp's update (native_ppo2._update_kind): the f16x3 FD / wgrad
            # kernels for [S<=8 or 41..44 -> 256 -> 256 -> A<=4] tanh nets (the lidar env's
            # 41-input nets included, their layer 1 on exact f32), the exact-f32 dense GEMMs for
            # other Linear/Tanh stacks (the PPO2-SOI demo's 4-128-64-32 / 4-64-64 nets;
            # ppo_msg['update_kernels'] = 'dense' opts any net into them); else torch autograd
            fits = all(dense_fits(m, a) for m, a in ((actor, True), (critic, False)))
            learner = "native" if fits else "torch"
        cls = NativePPO2Learner if learner == "native" else PPO2Learner
        self.learner = cls(actor, critic, self.msg, process_group, self.device)
        self.actor, self.critic = self.learner.actor, self.learner.critic
        self.world = self.learner.world
        self.gpu_actor = GPUNet(self.actor, True, self.device)
        self.gpu_critic = GPUNet(self.critic, False, self.device)
        # the fused rollout kernels take [S->256->256->A] / [S->256->256->1] tanh nets (packed);
        # any other Linear/Tanh stack (the PPO2-SOI demo's 4-128-64-32-2 / 4-64-64-1) runs
        # rlp_rollout's plain-layout path (per-step MLP kernels, same draws and buffers)
        fused = all(n.mfma_ok and n.desc.n_layers == 3 and n.desc.dims[1] == 256
                    for n in (self.gpu_actor, self.gpu_critic))
        self.plain = not fused
        if self.plain and self.gpu_actor.desc.act[self.gpu_actor.desc.n_layers - 1] != _abi.RLP_ACT_TANH:
            raise ValueError("VecPPO2: the actor's output layer must be tanh (mean = tanh * gain + off)")
        rule, flag = success_rule or (_abi.RLP_SUCCESS_DONE_AND_FLAG_NE, _abi.timeout_flag(self.kind))
        self.rule, self.flag = rule, flag
        lo, hi = _abi.action_bounds(self.kind, self.params)
        self.lo, self.hi = lo, hi
        self.seed = int(seed) if seed is not None else env.seed
        self.env_id0 = env.env_id0
        self.step0 = 0
        self.need = torch.ones(self.n, dtype=torch.uint8, device=self.device)
        self.bufs = K.rollout_buffers(self.kind, self.T, self.n, self.device)
        f32 = dict(dtype=torch.float32, device=self.device)
        self._rnorm = torch.empty((self.T, self.n), **f32)
        self._rnorm_stale = False
        self.adv = torch.empty((self.T, self.n), **f32)
        self.v_target = torch.empty((self.T, self.n), **f32)
        self.rms = torch.zeros(4, dtype=torch.float64, device=self.device)
        self.work = K.reward_norm_workspace(self.T, self.n, self.device)
        self.norm_scope = self.msg.get('norm_scope', 'global')
        if self.norm_scope not in ('global', 'rank'):
            raise ValueError(f"VecPPO2: norm_scope {self.norm_scope!r} (global | rank)")
        self.global_norm = self.norm_scope == 'global' and self.world > 1
        if self.global_norm:
            # the gathers size every rank's slot as this rank's, and the merges count n envs per
            # rank chunk: every rank must hold the same number of envs
            nn_ = torch.tensor([self.n, -self.n], dtype=torch.int64,
                               device=self.device if self.device.type == "cuda" else "cpu")
            torch.distributed.all_reduce(nn_, op=torch.distributed.ReduceOp.MAX,
                                         group=self.learner.pg)
            if int(nn_[0]) != -int(nn_[1]):
                raise ValueError(f"VecPPO2: norm_scope='global' needs the same n_envs on every rank "
                                 f"(min {-int(nn_[1])}, max {int(nn_[0])}); use norm_scope='rank'")
        self.adv_parts = K.adv_stats_parts(self.n)
        self.stats = K.adv_stats_buffer(self.n, self.world if self.global_norm else 1, self.device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(self.seed + 7919 * (self.env_id0 + 1))
        self.total_steps = 0

    # ------------------------------------------------------------------------------------------
    def std_list(self):
        std = torch.as_tensor(self.actor.std, dtype=torch.float32).reshape(-1).cpu().numpy()
        return list(np.broadcast_to(std, (len(self.lo),)))

    def _net_buf(self, net):
        return net.flat if self.plain else net.packed

    def rollout(self):
        cfg = K.make_rollout_cfg(self.T, self.n, self.seed, self.step0, self.env_id0,
                                 self.std_list(), self.lo, self.hi, self.rule, self.flag,
                                 plain=self.plain)
        self._rollout_ws = K.rollout(self.kind, self.params, self.env.state, self.need,
                                     self.gpu_actor.desc, self._net_buf(self.gpu_actor),
                                     self.gpu_critic.desc, self._net_buf(self.gpu_critic), cfg,
                                     self.bufs, workspace=getattr(self, "_rollout_ws", None))
        self.step0 += self.T
        self.total_steps += self.T * self.n * self.world

    def _gather(self, local):
        """Every rank's `local` (same size) in rank order, on every rank: each rank fills its slot
        of a zero buffer and one all-reduce sums them (x + 0 is exact, so this is a gather)."""
        rank = torch.distributed.get_rank(self.learner.pg)
        out = torch.zeros(self.world * local.numel(), dtype=local.dtype, device=local.device)
        out[rank * local.numel():(rank + 1) * local.numel()] = local.reshape(-1)
        torch.distributed.all_reduce(out, group=self.learner.pg)
        return out

    def advantages(self):
        b = self.bufs
        if self.plain:   # V(s') of the done && !success rows through the generic forward
            mask = (b["done"] & (1 - b["success"])).view(-1).contiguous()
            K.mlp_forward(self.gpu_critic.desc, self.gpu_critic.flat,
                          b["obs_next"].view(-1, self.env.state_dim), mask=mask,
                          out=b["value_next"].view(-1, 1))
        else:
            K.value_fixup(self.gpu_critic.desc, self.gpu_critic.packed, b["obs_next"], b["done"],
                          b["success"], b["value_next"])
        if self.global_norm:
            parts = self._gather(K.reward_norm_stats(b["reward"], self.work))
            K.reward_norm_finish(b["reward"], self.rms, self.work, parts, self.world, out=self._rnorm)
            self._rnorm_stale = False
            K.gae(self._rnorm, b["value"], b["value_next"], b["done"], b["success"],
                  self.msg['gamma'], self.msg['lmd'], adv=self.adv, v_target=self.v_target,
                  stats=self.stats)
            if self.msg['use_adv_norm']:
                parts = self.adv_parts
                local = self.stats[:3 * parts].clone()
                self.stats[:3 * parts * self.world] = self._gather(local)
                K.adv_normalize(self.adv, self.stats, parts * self.world)
        else:  # one rank's statistics: the rewards normalised as GAE loads them (not stored)
            K.reward_norm_statistics(b["reward"], self.rms, self.work)
            self._rnorm_stale = True
            K.gae_normalized(b["reward"], self.work, b["value"], b["value_next"], b["done"],
                             b["success"], self.msg['gamma'], self.msg['lmd'], adv=self.adv,
                             v_target=self.v_target, stats=self.stats)
            if self.msg['use_adv_norm']:
                K.adv_normalize(self.adv, self.stats, self.adv_parts)

    @property
    def rnorm(self):
        """the normalised rewards learn() consumed (computed on demand on the one-rank path, which
        normalises them inside the GAE scan instead of storing them; valid until the next
        rollout() overwrites the rewards)"""
        if self._rnorm_stale:
            K.reward_norm_apply(self.bufs["reward"], self.work, out=self._rnorm)
            self._rnorm_stale = False
        return self._rnorm

    def update(self):
        b = self.bufs
        S, Ad = self.env.state_dim, self.env.action_dim
        losses = self.learner.update(b["obs"].view(-1, S), b["action"].view(-1, Ad),
                                     b["logp"].view(-1, Ad), self.adv.view(-1, 1),
                                     self.v_target.view(-1, 1), self.gen)
        self.gpu_actor.refresh()
        self.gpu_critic.refresh()
        if self.learner.rule == 'ppo2':   # the DPPO2 Worker stores use_lr_decay but never decays
            self.learner.lr_decay(self.total_steps)
        return losses

    def iteration(self, learn=True):
        self.rollout()
        self.advantages()
        out = {}
        if learn:
            al, cl = self.update()
            out = {"actor_loss": al, "critic_loss": cl}
        return out

    def episode_stats(self):
        """(finished episodes, sum of their raw rewards is not tracked per-episode on device) —
        mean raw reward per env-step and terminal-flag histogram of the last segment."""
        b = self.bufs
        flags = torch.bincount(b["flag"].view(-1).to(torch.int64) + 0, minlength=5)
        return {"mean_reward": float(b["reward"].mean()), "episodes": int(b["done"].sum()),
                "flags": flags.cpu().tolist()}
