"""SAC (algorithm/actor_critic/Soft_Actor_Critic.py:12-129) with the replay buffer resident in HBM.

Same constructor, attributes and methods as the reference. What a driver sees differently:
  * memory is utils.classes.ReplayBuffer on the device (rlp_replay_* kernels); sample_buffer
    returns device fp32 tensors, so learn() has no host round trip;
  * choose_action also takes a batch of states ([n][S], one row per env of a VecEnv): the actor
    trunk then runs through rlp_mlp_forward and the squashed-Gaussian sample + clamp through
    rlp_sac_sample (Philox noise), returning a device tensor [n][A];
  * learn() (twin-Q target with the entropy term, actor loss alpha * log_pi - min(Q1, Q2), critic
    MSE on both heads, adaptive temperature, soft target update) runs natively — ONE
    rlp_sac_update call (native_sac.py) — for the drivers' SACActor / SACCritic structure
    (native="auto" checks it on a probe batch; native=True requires it; otherwise, or with
    native=False, the reference's torch code on the device). The native path draws its Gaussian
    noise from Philox (seed, device counter, row) instead of torch's generator;
  * graph=True captures one whole learn iteration — uniform batch indices (torch Philox), the
    replay gather, the update with capturable Adam, the soft update and the GPU actor's weight
    refresh — in a HIP graph (torch.cuda.CUDAGraph) and replays it: one launch instead of
    ~200 small kernels per update. Same arithmetic; the batch indices come from torch's
    generator instead of the Philox (seed, count) stream.
"""
import numpy as np
import torch
import torch.nn.functional as func

from ... import kernels as K
from ...utils.classes import GPUSACActor, ReplayBuffer


class _Snapshot:
    """Values of parameters and optimizer states, to undo graph warm-up updates in place (the
    tensors themselves must stay the ones the graph captures)."""

    def __init__(self, params, opts):
        self.params = list(params)
        self.saved = [p.detach().clone() for p in self.params]
        self.opts = list(opts)
        self.state = {id(t): t.detach().clone() for o in self.opts for st in o.state.values()
                      for t in st.values() if torch.is_tensor(t)}

    def restore(self):
        with torch.no_grad():
            for p, v in zip(self.params, self.saved):
                p.copy_(v)
            for o in self.opts:
                for st in o.state.values():
                    for t in st.values():
                        if torch.is_tensor(t):
                            if id(t) in self.state:
                                t.copy_(self.state[id(t)])
                            else:   # state created by the warm-up: back to a fresh Adam
                                t.zero_()


def _capture(body, device, modules, opts, extra_params=()):
    """Warm `body` up on a side stream (optimizer states, library workspaces), undo the warm-up
    updates, then capture one call of it in a HIP graph (torch.cuda.CUDAGraph)."""
    params = [p for m in modules for p in m.parameters()] + list(extra_params)
    snap = _Snapshot(params, opts)
    # torch.distributions' argument checks read values back to the host, which a stream under
    # capture cannot do: off while warming up and capturing
    validate = torch.distributions.Distribution._validate_args
    torch.distributions.Distribution.set_default_validate_args(False)
    try:
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(3):
                body()
        torch.cuda.current_stream(device).wait_stream(side)
        snap.restore()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            body()
    finally:
        torch.distributions.Distribution.set_default_validate_args(validate)
    return graph


class SAC:
    def __init__(self, env_msg: dict, gamma: float = 0.99, critic_tau: float = 0.005,
                 memory_capacity: int = 5000, batch_size: int = 256, actor=None, critic=None,
                 target_critic=None, a_lr: float = 3e-4, c_lr: float = 1e-4,
                 alpha_lr: float = 3e-4, adaptive_alpha: bool = True, device=None, seed=None,
                 graph: bool = False, native="auto"):
        if actor is None or critic is None or target_critic is None:
            raise ValueError("SAC: pass actor / critic / target_critic (utils.classes.SACActor, "
                             "SACCritic or the driver's own)")
        self.env_msg = env_msg
        self.gamma = gamma
        self.tau = critic_tau
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
        self.memory = ReplayBuffer(memory_capacity, batch_size, env_msg['state_dim'],
                                   env_msg['action_dim'], self.device, self.seed)
        self.actor = actor.to(self.device)
        self.critic = critic.to(self.device)
        self.target_critic = target_critic.to(self.device)
        self.a_lr, self.c_lr, self.alpha_lr = a_lr, c_lr, alpha_lr
        self.graph = bool(graph)
        cap = dict(capturable=True) if self.graph else {}
        self.actor_optimizer = torch.optim.Adam(self.actor.parameters(), lr=self.a_lr, **cap)
        self.critic_optimizer = torch.optim.Adam(self.critic.parameters(), lr=self.c_lr, **cap)
        self.adaptive_alpha = adaptive_alpha
        if self.adaptive_alpha:  # target entropy -dim(A); learn log_alpha so alpha > 0
            self.target_entropy = -env_msg['action_dim']
            self.log_alpha = torch.zeros(1).to(self.device)
            self.log_alpha.requires_grad = True
            # (graph mode: no autograd edge kept alive into log_alpha — a live edge would tie
            # log_alpha's gradient accumulator to this stream and break capture)
            self.alpha = self.log_alpha.detach().exp() if self.graph else self.log_alpha.exp()
            self.alpha_optimizer = torch.optim.Adam([self.log_alpha], lr=self.alpha_lr, **cap)
        else:
            self.alpha = 0.2
        self.a_min = torch.FloatTensor(np.asarray(env_msg['action_range'])[:, 0])
        self.a_max = torch.FloatTensor(np.asarray(env_msg['action_range'])[:, 1])
        self.episode = 0
        self.gpu_actor = None
        self.noise_counter = 0
        self._graph = None
        self._native = None
        if native:
            from .native_sac import SACNativeUpdate
            if native != "auto" or SACNativeUpdate.fits(self):
                self._native = SACNativeUpdate(self)

    def choose_action(self, s, deterministic=False):
        batched = (torch.is_tensor(s) and s.dim() == 2) or (not torch.is_tensor(s) and np.ndim(s) == 2)
        if not batched:  # the reference path, one env (:63-67)
            s_t = torch.unsqueeze(torch.tensor(s, dtype=torch.float), 0).to(self.device)
            with torch.no_grad():
                a, _ = self.actor(s_t, deterministic, False)
            a = torch.maximum(torch.minimum(a.cpu(), self.a_max), self.a_min)
            return a.data.numpy().flatten()
        if self.gpu_actor is None:
            self.gpu_actor = GPUSACActor(self.actor, self.device)
        self.noise_counter += 1
        a, _ = self.gpu_actor(torch.as_tensor(s, dtype=torch.float32, device=self.device),
                              deterministic=deterministic, with_logprob=False,
                              a_min=self.a_min.tolist(), a_max=self.a_max.tolist(),
                              seed=self.seed, counter=self.noise_counter)
        return a

    def choose_action_random(self, n=None):
        if n is None:
            a = torch.rand(self.env_msg['action_dim']) * (self.a_max - self.a_min) + self.a_min
            return a.cpu().detach().numpy().flatten()
        lo, hi = self.a_min.to(self.device), self.a_max.to(self.device)
        return torch.rand((n, len(lo)), device=self.device) * (hi - lo) + lo

    def learn(self, is_reward_ascent=False, iter=1):
        if self.memory.mem_counter < self.memory.batch_size:
            return None
        if self.graph and not is_reward_ascent:
            return self._learn_graphed(iter)
        out = None
        for _ in range(iter):
            s, a, r, s_, dw = self.memory.sample_buffer(is_reward_ascent=is_reward_ascent)
            out = self.update(s, a, r, s_, dw)
        return out

    # -- HIP-graph learn: sample -> gather -> update -> soft update -> actor refresh, one replay
    def _graph_body(self):
        mem = self.memory
        idx = (torch.rand(mem.batch_size, device=self.device) * self._gmax).long()
        idx.clamp_(max=mem.mem_size - 1)
        s, a, r, s_, dw = K.replay_gather(mem.rb, idx, out=self._gbuf)
        # alpha without an autograd edge to log_alpha: the reference's actor-loss gradient into
        # log_alpha is zeroed by alpha_optimizer.zero_grad() before it is used, so the values
        # are the same, and no autograd node outlives an iteration of the graph
        if self._native is not None:  # losses straight into the graph's buffer
            self._native.update(s, a, r, s_, dw, out=self._gloss)
        else:
            c, al = self._update_core(s, a, r, s_, dw, self.log_alpha.detach().exp()
                                      if self.adaptive_alpha else self.alpha)
            self._gloss[0].copy_(c)
            self._gloss[1].copy_(al)
        self.gpu_actor.copy_from_actor()

    def _learn_graphed(self, iters):
        mem = self.memory
        if self._graph is None:
            if self.gpu_actor is None:
                self.gpu_actor = GPUSACActor(self.actor, self.device)
            B, S, A = mem.batch_size, mem.rb.S, mem.rb.A
            f32 = dict(dtype=torch.float32, device=self.device)
            self._gbuf = (torch.empty((B, S), **f32), torch.empty((B, A), **f32),
                          torch.empty(B, **f32), torch.empty((B, S), **f32), torch.empty(B, **f32))
            self._gmax = torch.zeros((), **f32)
            self._gloss = torch.zeros(2, **f32)
            self._gmax.fill_(float(min(mem.mem_counter, mem.mem_size)))
            opts = [self.actor_optimizer, self.critic_optimizer] + (
                [self.alpha_optimizer] if self.adaptive_alpha else [])
            extra = ([self.log_alpha] if self.adaptive_alpha else []) + (
                self._native.state_tensors() if self._native else [])
            self._graph = _capture(self._graph_body, self.device,
                                   [self.actor, self.critic, self.target_critic], opts, extra)
        for _ in range(iters):
            self._gmax.fill_(float(min(mem.mem_counter, mem.mem_size)))
            self._graph.replay()
        if self.adaptive_alpha:
            self.alpha = self.log_alpha.detach().exp()
        return self._gloss[0], self._gloss[1]

    def update(self, batch_s, batch_a, batch_r, batch_s_, batch_dw, noise=None):
        """One SAC update (:73-124); batch_dw is the buffer's fifth column, as in the reference.
        noise ([2][B][A]: eps of the s' draw, then of the s draw) replays a recorded tape on the
        native path."""
        if self._native is not None:
            out = self._native.update(batch_s, batch_a, batch_r, batch_s_, batch_dw, noise)
        else:
            if noise is not None:
                raise ValueError("SAC.update: noise is a native-path argument")
            out = self._update_core(batch_s, batch_a, batch_r, batch_s_, batch_dw, self.alpha)
        if self.adaptive_alpha:
            self.alpha = self.log_alpha.exp()
        if self.gpu_actor is not None:
            self.gpu_actor.refresh()
        return out

    def _update_core(self, batch_s, batch_a, batch_r, batch_s_, batch_dw, alpha):
        if self._native is not None:
            return self._native.update(batch_s, batch_a, batch_r, batch_s_, batch_dw)
        batch_r = batch_r.reshape(-1, 1)
        batch_dw = batch_dw.reshape(-1, 1)
        with torch.no_grad():
            batch_a_, log_pi_ = self.actor(batch_s_)  # a' from the current policy
            target_Q1, target_Q2 = self.target_critic(batch_s_, batch_a_)
            target_Q = batch_r + self.gamma * (1 - batch_dw) * (torch.min(target_Q1, target_Q2) -
                                                                 alpha * log_pi_)
        a, log_pi = self.actor(batch_s)
        Q1, Q2 = self.critic(batch_s, a)
        Q = torch.min(Q1, Q2)
        actor_loss = (alpha * log_pi - Q).mean()
        current_Q1, current_Q2 = self.critic(batch_s, batch_a)
        critic_loss = func.mse_loss(current_Q1, target_Q) + func.mse_loss(current_Q2, target_Q)
        alpha_loss = 0.
        if self.adaptive_alpha:
            alpha_loss = -(self.log_alpha.exp() * (log_pi + self.target_entropy).detach()).mean()
        self.actor_optimizer.zero_grad()
        actor_loss.backward()
        self.actor_optimizer.step()
        self.critic_optimizer.zero_grad()
        critic_loss.backward()
        self.critic_optimizer.step()
        if self.adaptive_alpha:
            self.alpha_optimizer.zero_grad()
            alpha_loss.backward()
            self.alpha_optimizer.step()
        with torch.no_grad():
            for param, target_param in zip(self.critic.parameters(), self.target_critic.parameters()):
                target_param.data.copy_(self.tau * param.data + (1 - self.tau) * target_param.data)
        return critic_loss.detach(), actor_loss.detach()

    def save_ac(self, msg, path):
        torch.save(self.actor.state_dict(), path + 'actor' + msg)
        torch.save(self.critic.state_dict(), path + 'critic' + msg)
        torch.save(self.target_critic.state_dict(), path + 'target_critic' + msg)

    def SAC_info(self):
        print('agent name：', self.env_msg['name'])
        print('state_dim:', self.env_msg['state_dim'])
        print('action_dim:', self.env_msg['action_dim'])
        print('action_range:', self.env_msg['action_range'])
