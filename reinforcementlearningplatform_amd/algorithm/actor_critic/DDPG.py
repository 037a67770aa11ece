"""DDPG (algorithm/actor_critic/DDPG.py:14-130) with the replay buffer resident in HBM.

Same constructor, attributes and methods as the reference. Differences that matter to a driver:
  * memory is utils.classes.ReplayBuffer on the device (rlp_replay_* kernels); sample_buffer
    returns device fp32 tensors, so learn() has no host round trip;
  * choose_action also takes a batch of states ([n][S], one row per env of a VecEnv): the actor
    forward then runs through librlp (GPUNet; the drivers' ReLU nets go through the generic MLP
    kernel) and the N(0, sigma^2) exploration noise + clip through rlp_policy_sample (Philox),
    returning a device tensor;
  * the update (critic MSE to the target r + gamma * (1 - done) * Q'(s', mu'(s')), actor loss
    -Q(s, mu(s)), Adam, soft target updates) runs natively — ONE rlp_ddpg_update call
    (native_ddpg.py) — for the drivers' relu nets (native="auto" checks the nets' forward on a
    probe batch; native=True requires it; native=False or any other net: the reference's torch
    code on the device);
  * graph=True captures one whole learn iteration (uniform batch indices from torch's generator,
    the replay gather, the update with the nets' Adam switched to capturable, the soft updates
    and the GPU actor's weight refresh) in a HIP graph and replays it.
"""
import numpy as np
import torch
import torch.nn.functional as func

from ... import kernels as K
from ...utils.classes import GPUNet, ReplayBuffer


class DDPG:
    def __init__(self, env_msg: dict, gamma: float = 0.99, actor_soft_update: float = 1e-2,
                 critic_soft_update: float = 1e-2, memory_capacity: int = 5000,
                 batch_size: int = 512, actor=None, target_actor=None, critic=None,
                 target_critic=None, device=None, seed=None, graph=False, native="auto"):
        if actor is None or target_actor is None or critic is None or target_critic is None:
            raise ValueError("DDPG: pass the driver's actor/target_actor/critic/target_critic "
                             "(the reference's default-argument placeholder nets have no forward)")
        self.env_msg = env_msg
        self.gamma = gamma
        self.actor_tau = actor_soft_update
        self.critic_tau = critic_soft_update
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
        self.memory = ReplayBuffer(memory_capacity, batch_size, env_msg['state_dim'],
                                   env_msg['action_dim'], self.device, self.seed)
        self.actor, self.target_actor = actor.to(self.device), target_actor.to(self.device)
        self.critic, self.target_critic = critic.to(self.device), target_critic.to(self.device)
        for m in (self.actor, self.target_actor):
            for name in ("a_min", "a_max", "off", "gain"):
                v = getattr(m, name, None)
                if torch.is_tensor(v):
                    setattr(m, name, v.to(self.device))
        self.target_actor.load_state_dict(self.actor.state_dict())
        self.target_critic.load_state_dict(self.critic.state_dict())
        self.a_min = np.asarray(env_msg['action_range'])[:, 0]
        self.a_max = np.asarray(env_msg['action_range'])[:, 1]
        self.episode = 0
        self.reward = 0
        self.gpu_actor = None
        self.noise_counter = 0
        self.graph = bool(graph)
        self._graph = None
        self._native = None
        if native:
            from .native_ddpg import DDPGNativeUpdate
            if native != "auto" or DDPGNativeUpdate.fits(self):
                self._native = DDPGNativeUpdate(self)

    def choose_action_random(self, n=None):
        if n is None:
            return np.random.uniform(low=self.a_min, high=self.a_max)
        lo = torch.as_tensor(self.a_min, dtype=torch.float32, device=self.device)
        hi = torch.as_tensor(self.a_max, dtype=torch.float32, device=self.device)
        return lo + (hi - lo) * torch.rand((n, len(self.a_min)), device=self.device)

    def choose_action(self, state, is_optimal=False, sigma: np.ndarray = np.zeros(1)):
        batched = (torch.is_tensor(state) and state.dim() == 2) or np.ndim(state) == 2
        if not batched:  # the reference path, one env
            t_state = torch.tensor(state, dtype=torch.float, device=self.device)
            mu = self.actor(t_state)
            if not is_optimal:
                noise = np.random.multivariate_normal(np.zeros_like(sigma), np.diag(sigma ** 2))
                mu = mu.cpu().detach().numpy().flatten() + noise
            else:
                mu = mu.cpu().detach().numpy().flatten()
            return np.clip(mu, self.a_min, self.a_max)
        if self.gpu_actor is None:
            self.gpu_actor = GPUNet(self.actor, True, self.device)
        s = torch.as_tensor(state, dtype=torch.float32, device=self.device).contiguous()
        mean = self.gpu_actor(s).contiguous()
        A = mean.shape[1]
        std = np.broadcast_to(np.asarray(sigma, dtype=np.float32).reshape(-1), (A,))
        if is_optimal:
            std = np.zeros(A, np.float32)
        self.noise_counter += 1
        a, _ = K.policy_sample(mean, std, self.a_min, self.a_max, seed=self.seed,
                               counter=self.noise_counter)
        return a

    def evaluate(self, state):
        t_state = torch.tensor(state, dtype=torch.float, device=self.device)
        return self.target_actor(t_state).cpu().detach().numpy().flatten()

    def learn(self, is_reward_ascent=True, iter=1):
        if self.memory.mem_counter < self.memory.batch_size:
            return None
        if self.graph and not is_reward_ascent:
            return self._learn_graphed(iter)
        critic_loss = actor_loss = None
        for _ in range(iter):
            s, a, r, s_, done = self.memory.sample_buffer(is_reward_ascent=is_reward_ascent)
            critic_loss, actor_loss = self.update(s, a, r, s_, done)
        return critic_loss, actor_loss

    # -- HIP-graph learn (see the module docstring)
    def _graph_body(self):
        mem = self.memory
        idx = (torch.rand(mem.batch_size, device=self.device) * self._gmax).long()
        idx.clamp_(max=mem.mem_size - 1)
        s, a, r, s_, done = K.replay_gather(mem.rb, idx, out=self._gbuf)
        if self._native is not None:  # losses straight into the graph's buffer
            self._native.update(s, a, r, s_, done, out=self._gloss)
        else:
            c, al = self._update_core(s, a, r, s_, done)
            self._gloss[0].copy_(c)
            self._gloss[1].copy_(al)
        self.gpu_actor.copy_from_module()  # (no copy when it aliases the native parameters)

    def _learn_graphed(self, iters):
        from .Soft_Actor_Critic import _capture
        mem = self.memory
        if self._graph is None:
            if self.gpu_actor is None:
                self.gpu_actor = GPUNet(self.actor, True, self.device)
            for opt in (self.critic.optimizer, self.actor.optimizer):
                for grp in opt.param_groups:
                    grp["capturable"] = True
            B, S, A = mem.batch_size, mem.rb.S, mem.rb.A
            f32 = dict(dtype=torch.float32, device=self.device)
            self._gbuf = (torch.empty((B, S), **f32), torch.empty((B, A), **f32),
                          torch.empty(B, **f32), torch.empty((B, S), **f32), torch.empty(B, **f32))
            self._gmax = torch.zeros((), **f32)
            self._gloss = torch.zeros(2, **f32)
            self._gmax.fill_(float(min(mem.mem_counter, mem.mem_size)))
            self._graph = _capture(self._graph_body, self.device,
                                   [self.actor, self.target_actor, self.critic, self.target_critic],
                                   [self.critic.optimizer, self.actor.optimizer],
                                   self._native.state_tensors() if self._native else ())
        for _ in range(iters):
            self._gmax.fill_(float(min(mem.mem_counter, mem.mem_size)))
            self._graph.replay()
        return self._gloss[0], self._gloss[1]

    def update(self, s, a, r, s_, done):
        """One DDPG update on a sampled batch (done = the buffer's 1 - done column), :83-109."""
        out = self._update_core(s, a, r, s_, done)
        if self.gpu_actor is not None:
            self.gpu_actor.refresh()
        return out

    def _update_core(self, s, a, r, s_, done):
        if self._native is not None:
            return self._native.update(s, a, r, s_, done)
        with torch.no_grad():
            Q_ = self.target_critic(s_, self.target_actor(s_))
            target_Q = r.unsqueeze(1) + self.gamma * done.unsqueeze(1) * Q_
        current_Q = self.critic(s, a)
        critic_loss = func.mse_loss(target_Q, current_Q)
        self.critic.optimizer.zero_grad()
        critic_loss.backward()
        self.critic.optimizer.step()
        for params in self.critic.parameters():
            params.requires_grad = False
        actor_loss = -self.critic(s, self.actor(s)).mean()
        self.actor.optimizer.zero_grad()
        actor_loss.backward()
        self.actor.optimizer.step()
        for params in self.critic.parameters():
            params.requires_grad = True
        self.update_network_parameters()
        return critic_loss.detach(), actor_loss.detach()

    def update_network_parameters(self):
        with torch.no_grad():
            for tp, p in zip(self.target_critic.parameters(), self.critic.parameters()):
                tp.data.copy_(tp.data * (1.0 - self.critic_tau) + p.data * self.critic_tau)
            for tp, p in zip(self.target_actor.parameters(), self.actor.parameters()):
                tp.data.copy_(tp.data * (1.0 - self.actor_tau) + p.data * self.actor_tau)

    def save_ac(self, msg, path):
        torch.save(self.actor.state_dict(), path + 'actor' + msg)
        torch.save(self.target_actor.state_dict(), path + 'target_actor' + msg)
        torch.save(self.critic.state_dict(), path + 'critic' + msg)
        torch.save(self.target_critic.state_dict(), path + 'target_critic' + msg)

    def DDPG_info(self):
        print('agent name：', self.env_msg['name'])
        print('state_dim:', self.env_msg['state_dim'])
        print('action_dim:', self.env_msg['action_dim'])
        print('action_range:', self.env_msg['action_range'])
