"""Proximal_Policy_Optimization2 — drop-in for algorithm/policy_base/Proximal_Policy_Optimization2.py.

Same constructor (env_msg, ppo_msg, actor, critic), attributes (buffer, buffer2, actor, critic,
cnt, ...) and methods (choose_action, evaluate, learn, lr_decay, action_linear_trans, save_ac,
PPO2_info). What runs where:
  choose_action / evaluate   actor forward on fp32 MFMA + Philox Gaussian sample (librlp)
  learn(): V(s), V(s')       critic forward on fp32 MFMA (librlp)
           GAE(lambda)       rlp_gae (bit-identical to the reference's NumPy-2 loop)
           K epochs          learner="native" (default for the drivers' Linear/Tanh nets):
                             librlp's update kernels (NativePPO2Learner: f16x3 for [S,256,256,A],
                             exact f32 GEMMs for other widths); learner="torch": torch
                             autograd + Adam on the same GPU. Both pinned to the reference's
                             learn() (tests/test_learn_golden.py, tests/test_gpu_transcript.py).
The reference pins PPO2 to the CPU (:11-13); here everything lives on `device` (default cuda).
"""
import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data.sampler import BatchSampler, SubsetRandomSampler

from ... import _abi
from ... import kernels as K
from ...utils.classes import GPUNet, PPOActor_Gaussian, PPOCritic, RolloutBuffer, RolloutBuffer2

_ACTOR_TENSOR_ATTRS = ("a_min", "a_max", "off", "gain", "std")


class Proximal_Policy_Optimization2:
    def __init__(self, env_msg: dict = None, ppo_msg: dict = None, actor=None, critic=None,
                 device=None, seed=None, learner=None):
        self.env_msg = env_msg
        self.ppo_msg = ppo_msg
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.gamma = ppo_msg['gamma']
        self.K_epochs = ppo_msg['K_epochs']
        self.eps_clip = ppo_msg['eps_clip']
        self.buffer = RolloutBuffer(ppo_msg['buffer_size'], env_msg['state_dim'], env_msg['action_dim'],
                                    device=self.device)
        self.buffer2 = RolloutBuffer2(env_msg['state_dim'], env_msg['action_dim'])
        self.actor_lr = ppo_msg['a_lr']
        self.critic_lr = ppo_msg['c_lr']
        self.set_adam_eps = ppo_msg['set_adam_eps']
        self.lmd = ppo_msg['lmd']
        self.use_adv_norm = ppo_msg['use_adv_norm']
        self.mini_batch_size = ppo_msg['mini_batch_size']
        self.entropy_coef = ppo_msg['entropy_coef']
        self.use_grad_clip = ppo_msg['use_grad_clip']
        self.use_lr_decay = ppo_msg['use_lr_decay']
        self.max_train_steps = ppo_msg['max_train_steps']
        self.using_mini_batch = ppo_msg['using_mini_batch']

        self.actor = (actor if actor is not None else PPOActor_Gaussian()).to(self.device)
        self.critic = (critic if critic is not None else PPOCritic()).to(self.device)
        self._sync_actor_attrs()
        eps = dict(eps=1e-5) if self.set_adam_eps else {}
        self.optimizer_actor = torch.optim.Adam(self.actor.parameters(), lr=self.actor_lr, **eps)
        self.optimizer_critic = torch.optim.Adam(self.critic.parameters(), lr=self.critic_lr, **eps)
        self.loss = torch.nn.MSELoss()
        self.gpu_actor = GPUNet(self.actor, is_actor=True, device=self.device)
        self.gpu_critic = GPUNet(self.critic, is_actor=False, device=self.device)
        self.seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
        self.sample_counter = 0
        self.cnt = 0
        from .native_ppo2 import NativePPO2Learner, dense_fits
        fits = all(dense_fits(m, a)
                   for m, a in ((self.actor, True), (self.critic, False)))
        self.learner = learner or ("native" if fits else "torch")
        self.native = None
        if self.learner == "native":
            if not fits:
                raise ValueError("learner='native' needs Linear/Tanh nets (tanh hidden layers, "
                                 "tanh * gain + off actor head, linear critic head)")
            self.native = NativePPO2Learner(self.actor, self.critic, ppo_msg, device=self.device)
        elif self.learner != "torch":
            raise ValueError(f"learner {learner!r} (native | torch)")

    # driver-defined actors keep a_min / a_max / gain / off / std as plain tensor attributes;
    # keep them on the learner's device
    def _sync_actor_attrs(self):
        for name in _ACTOR_TENSOR_ATTRS:
            v = getattr(self.actor, name, None)
            if torch.is_tensor(v) and v.device != self.device:
                setattr(self.actor, name, v.to(self.device))

    def _std_list(self):
        std = torch.as_tensor(self.actor.std, dtype=torch.float32).reshape(-1).cpu().numpy()
        A = self.env_msg['action_dim']
        return list(np.broadcast_to(std, (A,)))

    def evaluate(self, state):
        s = torch.as_tensor(np.asarray(state, dtype=np.float32), device=self.device).view(1, -1)
        return self.gpu_actor(s).cpu().numpy().flatten()

    def choose_action(self, state: np.ndarray, noise=None):
        """mean = actor(s); a = clamp(mean + std * eps, a_min, a_max); log_prob(a) per dim.
        eps is a Philox N(0,1) draw, or `noise` ([action_dim] float32) when given — the injected
        exploration noise a transcript replay uses (tests/test_gpu_transcript.py)."""
        self._sync_actor_attrs()
        s = torch.as_tensor(np.asarray(state, dtype=np.float32), device=self.device).view(1, -1)
        mean = self.gpu_actor(s).contiguous()
        a_min = torch.as_tensor(self.actor.a_min).reshape(-1).cpu().tolist()
        a_max = torch.as_tensor(self.actor.a_max).reshape(-1).cpu().tolist()
        nz = None
        if noise is not None:
            nz = torch.as_tensor(np.asarray(noise, np.float32).reshape(mean.shape), device=self.device)
        a, lp = K.policy_sample(mean, self._std_list(), a_min, a_max, noise=nz, seed=self.seed,
                                counter=self.sample_counter)
        self.sample_counter += 1
        return a.cpu().numpy().flatten(), lp.cpu().numpy().flatten()

    def compute_gae(self, r, vs, vs_, done, success):
        """Proximal_Policy_Optimization2.py:88-98 on the GPU (flat buffer = one env, T = B)."""
        B = r.shape[0]
        col = lambda t: t.reshape(B, 1).contiguous()
        u8 = lambda t: (t.reshape(B, 1) > 0.5).to(torch.uint8).contiguous()
        adv, v_target = K.gae(col(r), col(vs), col(vs_), u8(done), u8(success), self.gamma, self.lmd)
        return adv.view(-1, 1), v_target.view(-1, 1)

    def learn(self, current_steps, buf_num: int = 1):
        self._sync_actor_attrs()
        buf = self.buffer if buf_num == 1 else self.buffer2
        s, a, a_lp, r, s_, done, success = buf.to_tensor(self.device)
        with torch.no_grad():
            vs = self.gpu_critic(s)
            vs_ = self.gpu_critic(s_)
            adv, v_target = self.compute_gae(r, vs, vs_, done, success)
            if self.use_adv_norm:  # Trick 1: advantage normalisation
                adv = (adv - adv.mean()) / (adv.std() + 1e-5)
        self.update(s, a, a_lp, adv, v_target)
        if self.use_lr_decay:
            self.lr_decay(current_steps)

    def _epoch(self, s, a, a_lp, adv, v_target):
        dist_now = self.actor.get_dist(s)
        dist_entropy = dist_now.entropy().sum(1, keepdim=True)
        a_logprob_now = dist_now.log_prob(a)
        ratios = torch.exp(a_logprob_now.sum(1, keepdim=True) - a_lp.sum(1, keepdim=True))
        surr1 = ratios * adv
        surr2 = torch.clamp(ratios, 1 - self.eps_clip, 1 + self.eps_clip) * adv
        actor_loss = -torch.min(surr1, surr2) - self.entropy_coef * dist_entropy
        self.optimizer_actor.zero_grad()
        actor_loss.mean().backward()
        if self.use_grad_clip:
            torch.nn.utils.clip_grad_norm_(self.actor.parameters(), 0.5)
        self.optimizer_actor.step()
        critic_loss = F.mse_loss(v_target, self.critic(s))
        self.optimizer_critic.zero_grad()
        critic_loss.backward()
        if self.use_grad_clip:
            torch.nn.utils.clip_grad_norm_(self.critic.parameters(), 0.5)
        self.optimizer_critic.step()

    def update(self, s, a, a_lp, adv, v_target):
        """K epochs of clipped-surrogate + entropy (actor) and MSE (critic), :102-160."""
        if self.native is not None:
            perms = None
            if self.using_mini_batch:   # SubsetRandomSampler's draws (torch's global CPU RNG)
                perms = [torch.randperm(s.shape[0]) for _ in range(self.K_epochs)]
            self.native.update(s, a, a_lp, adv, v_target, perms=perms)
            self.gpu_actor.refresh()
            self.gpu_critic.refresh()
            return
        for _ in range(self.K_epochs):
            if self.using_mini_batch:
                for idx in BatchSampler(SubsetRandomSampler(range(s.shape[0])), self.mini_batch_size, False):
                    idx = torch.as_tensor(idx, device=self.device)
                    self._epoch(s[idx], a[idx], a_lp[idx], adv[idx], v_target[idx])
            else:
                self._epoch(s, a, a_lp, adv, v_target)
        self.gpu_actor.refresh()
        self.gpu_critic.refresh()

    def lr_decay(self, total_steps):
        if total_steps < self.max_train_steps:
            lr_a = max(self.actor_lr * (1 - total_steps / self.max_train_steps), 1e-6)
            lr_c = max(self.critic_lr * (1 - total_steps / self.max_train_steps), 1e-6)
            for p in self.optimizer_actor.param_groups:
                p['lr'] = lr_a
            for p in self.optimizer_critic.param_groups:
                p['lr'] = lr_c
            if self.native is not None:
                self.native.lr = {"a": lr_a, "c": lr_c}

    def action_linear_trans(self, action):
        out = []
        for i in range(self.env_msg['action_dim']):
            a = min(max(action[i], -1), 1)
            lo, hi = self.env_msg['action_range'][i][0], self.env_msg['action_range'][i][1]
            out.append((hi - lo) / 2 * a + (hi + lo) / 2)
        return np.array(out)

    def save_ac(self, msg, path):
        """Same files and key names as the reference (datasave/.../actor, critic)."""
        torch.save(self.actor.state_dict(), path + 'actor' + msg)
        torch.save(self.critic.state_dict(), path + 'critic' + msg)

    def PPO2_info(self):
        print('agent name：', self.env_msg['name'])
        print('state_dim:', self.env_msg['state_dim'])
        print('action_dim:', self.env_msg['action_dim'])
        print('action_range:', self.env_msg['action_range'])
