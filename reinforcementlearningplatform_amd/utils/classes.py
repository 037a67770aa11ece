"""Buffers, normalisers and the PPO2 driver networks (utils/classes.py of the reference, the parts on
the PPO2 hot path), plus GPUNet: the adapter that runs a driver-defined Linear/Tanh network through
librlp's MFMA kernels.
"""
import numpy as np
import torch
import torch.nn as nn

from .. import _abi
from .. import kernels as K


# ---------------------------------------------------------------------------------------------
# Running statistics (utils/classes.py:626-673)
# ---------------------------------------------------------------------------------------------
class RunningMeanStd:
    """Welford running mean/std; the first sample sets std = x (reference behaviour, :634-637)."""

    def __init__(self, shape):
        self.n = 0
        self.mean = np.zeros(shape)
        self.S = np.zeros(shape)
        self.std = np.sqrt(self.S)

    def update(self, x):
        x = np.array(x)
        self.n += 1
        if self.n == 1:
            self.mean, self.std = x, x
            return
        prev = self.mean.copy()
        self.mean = prev + (x - prev) / self.n
        self.S = self.S + (x - prev) * (x - self.mean)
        self.std = np.sqrt(self.S / self.n)


class Normalization:
    def __init__(self, shape):
        self.running_ms = RunningMeanStd(shape=shape)

    def __call__(self, x, update=True):
        if update:
            self.running_ms.update(x)
        return (x - self.running_ms.mean) / (self.running_ms.std + 1e-8)


class RewardScaling:
    def __init__(self, shape, gamma):
        self.shape, self.gamma = shape, gamma
        self.running_ms = RunningMeanStd(shape=shape)
        self.R = np.zeros(shape)

    def __call__(self, x):
        self.R = self.gamma * self.R + x
        self.running_ms.update(self.R)
        return x / (self.running_ms.std + 1e-8)

    def reset(self):
        self.R = np.zeros(self.shape)


# ---------------------------------------------------------------------------------------------
# Rollout buffer (utils/classes.py:250-310): same API; the storage is a float64 host array as in
# the reference (a single env appends one row per step), to_tensor() hands fp32 tensors to the
# learner's device.
# ---------------------------------------------------------------------------------------------
class ReplayBuffer:
    """utils/classes.py:189-247 ReplayBuffer with the columns resident in HBM (rlp_replay_*).

    Same constructor and methods; store_transition also takes a batch (leading axis n: the n
    envs of one step, stored in env order as n sequential store_transition calls would), and
    sample_buffer returns device fp32 tensors (s, a, r, s_, end[, log_probs]) — what DDPG.learn
    turns the reference's numpy arrays into. Sampling draws from a Philox stream keyed by
    (seed, sample count) instead of numpy's / random's global generators."""

    def __init__(self, max_size: int, batch_size: int, state_dim: int, action_dim: int,
                 device=None, seed=None):
        self.mem_size = int(max_size)
        self.mem_counter = 0
        self.batch_size = int(batch_size)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.cols, self.rb = K.replay_alloc(self.mem_size, state_dim, action_dim, self.device)
        self.s_mem, self.a_mem, self.r_mem = self.cols["s"], self.cols["a"], self.cols["r"]
        self._s_mem, self.end_mem = self.cols["s_next"], self.cols["end"]
        self.log_prob_mem = torch.zeros(self.mem_size, dtype=torch.float32, device=self.device)
        self.sorted_index = []
        self.resort_count = 0
        self.seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
        self.sample_count = 0
        self._ws = None

    def _dev(self, x, dtype, cols=None):
        t = torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x, device=self.device)
        t = t.to(dtype)
        return t.reshape(-1, cols) if cols else t.reshape(-1)

    def store_transition(self, state, action, reward, state_, done, log_p=0.,
                         has_log_prob: bool = False):
        S, A = self.rb.S, self.rb.A
        s = self._dev(state, torch.float32, S)
        n = s.shape[0]
        if has_log_prob:
            rows = (self.mem_counter + torch.arange(n, device=self.device)) % self.mem_size
            self.log_prob_mem[rows] = self._dev(log_p, torch.float32).expand(n)
        K.replay_store(self.rb, self.mem_counter, s, self._dev(action, torch.float32, A),
                       self._dev(reward, torch.float64), self._dev(state_, torch.float32, S),
                       self._dev(np.asarray(done) if not torch.is_tensor(done) else done,
                                 torch.uint8))
        self.mem_counter += n

    def get_reward_sort(self):
        """Indices of the stored rows sorted by reward, ascending (stable) — :212-217."""
        m = min(self.mem_counter, self.mem_size)
        self.sorted_index = torch.sort(self.r_mem[:m], stable=True).indices

    def store_transition_per_episode(self, states, actions, rewards, states_, dones, log_ps=None,
                                     has_log_prob: bool = False):
        self.resort_count += 1
        self.store_transition(states, actions, rewards, states_, dones,
                              0. if log_ps is None else log_ps, has_log_prob)

    def sample_index(self, is_reward_ascent: bool = True):
        max_mem = min(self.mem_counter, self.mem_size)
        self.sample_count += 1
        if is_reward_ascent:
            if self._ws is None:
                self._ws = K.replay_workspace(self.mem_size, self.device)
            return K.replay_sample_reward_top(self.rb, max_mem, self.batch_size, self.seed,
                                              self.sample_count, self._ws)
        return K.replay_sample_uniform(max_mem, self.batch_size, self.seed, self.sample_count,
                                       device=self.device)

    def sample_buffer(self, is_reward_ascent: bool = True, has_log_prob: bool = False):
        idx = self.sample_index(is_reward_ascent)
        s, a, r, s_, end = K.replay_gather(self.rb, idx)
        if has_log_prob:
            return s, a, r, s_, end, self.log_prob_mem[idx]
        return s, a, r, s_, end


class RolloutBuffer:
    FIELDS = ("s", "a", "a_lp", "r", "s_", "done", "success")

    def __init__(self, batch_size: int, state_dim: int, action_dim: int, device=None):
        self.batch_size, self.state_dim, self.action_dim = batch_size, state_dim, action_dim
        self.device = device
        self.s = np.zeros((batch_size, state_dim))
        self.a = np.zeros((batch_size, action_dim))
        self.a_lp = np.zeros((batch_size, action_dim))
        self.r = np.zeros((batch_size, 1))
        self.s_ = np.zeros((batch_size, state_dim))
        self.done = np.zeros((batch_size, 1))
        self.success = np.zeros((batch_size, 1))
        self.index = 0

    def append(self, s, a, log_prob, r, s_, done, success, index):
        self.s[index], self.a[index], self.a_lp[index] = s, a, log_prob
        self.r[index], self.s_[index] = r, s_
        self.done[index], self.success[index] = done, success

    def append_traj(self, s, a, log_prob, r, s_, done, success):
        for i in range(len(done)):
            if self.index == self.batch_size:
                self.index = 0
                return True
            self.append(s[i], a[i], log_prob[i], r[i], s_[i], done[i], success[i], self.index)
            self.index += 1
        return False

    def to_tensor(self, device=None):
        dev = device or self.device or "cpu"
        return tuple(torch.tensor(getattr(self, f), dtype=torch.float, device=dev) for f in self.FIELDS)

    def print_size(self):
        print('==== RolloutBuffer ====')
        for f in self.FIELDS:
            print(f'{f}: {getattr(self, f).size}')


class RolloutBuffer2:
    """Growing trajectory buffer (utils/classes.py:313-376)."""

    def __init__(self, state_dim: int, action_dim: int):
        self.state_dim, self.action_dim = state_dim, action_dim
        self.clean()

    def clean(self):
        self.index = 0
        for f in RolloutBuffer.FIELDS:
            setattr(self, f, np.atleast_2d([]).astype(np.float32))

    def append_traj(self, s, a, log_prob, r, s_, done, success):
        vals = dict(s=s, a=a, a_lp=log_prob, r=r, s_=s_, done=done, success=success)
        for f, v in vals.items():
            v = np.atleast_2d(v).astype(np.float32)
            setattr(self, f, v if self.index == 0 else np.vstack((getattr(self, f), v)))
        self.index += len(done)

    def to_tensor(self, device=None):
        return tuple(torch.tensor(getattr(self, f), dtype=torch.float, device=device or "cpu")
                     for f in RolloutBuffer.FIELDS)


# ---------------------------------------------------------------------------------------------
# PPO2 driver networks (demonstration/PPO2/PPO2-4-CartPole/train.py:39-125): same constructor
# arguments and parameter names (fc1 / fc2 / mean_layer, fc1 / fc2 / fc3) so the shipped
# datasave/net checkpoints load unchanged.
# ---------------------------------------------------------------------------------------------
def _orthogonal(layer, gain=1.0):
    nn.init.orthogonal_(layer.weight, gain=gain)
    nn.init.constant_(layer.bias, 0)


class PPOActor_Gaussian(nn.Module):
    def __init__(self, state_dim: int = 3, action_dim: int = 3, a_min=np.zeros(3), a_max=np.ones(3),
                 init_std: float = 0.5, use_orthogonal_init: bool = True, hidden: int = 256):
        super().__init__()
        self.fc1 = nn.Linear(state_dim, hidden)
        self.fc2 = nn.Linear(hidden, hidden)
        self.mean_layer = nn.Linear(hidden, action_dim)
        self.activate_func = nn.Tanh()
        self.a_min = torch.tensor(a_min, dtype=torch.float)
        self.a_max = torch.tensor(a_max, dtype=torch.float)
        self.off = (self.a_min + self.a_max) / 2.0
        self.gain = self.a_max - self.off
        self.action_dim = action_dim
        self.std = torch.tensor(init_std, dtype=torch.float)
        if use_orthogonal_init:
            self.orthogonal_init_all()

    def orthogonal_init_all(self):
        _orthogonal(self.fc1)
        _orthogonal(self.fc2)
        _orthogonal(self.mean_layer, gain=0.01)

    def _apply(self, fn, *args, **kwargs):  # keep the non-parameter tensors on the module's device
        super()._apply(fn, *args, **kwargs)
        self.a_min, self.a_max = fn(self.a_min), fn(self.a_max)
        self.off, self.gain = fn(self.off), fn(self.gain)
        self.std = fn(self.std) if torch.is_tensor(self.std) else self.std
        return self

    def forward(self, s):
        s = self.activate_func(self.fc1(s))
        s = self.activate_func(self.fc2(s))
        return torch.tanh(self.mean_layer(s)) * self.gain + self.off

    def get_dist(self, s):
        mean = self.forward(s)
        std = torch.as_tensor(self.std, dtype=mean.dtype, device=mean.device).expand_as(mean)
        return torch.distributions.Normal(mean, std)

    def evaluate(self, state):
        with torch.no_grad():
            t = torch.tensor(state, dtype=torch.float, device=self.fc1.weight.device).unsqueeze(0)
            return self.forward(t).cpu().numpy().flatten()


class PPOCritic(nn.Module):
    def __init__(self, state_dim=3, use_orthogonal_init: bool = True, hidden: int = 256):
        super().__init__()
        self.fc1 = nn.Linear(state_dim, hidden)
        self.fc2 = nn.Linear(hidden, hidden)
        self.fc3 = nn.Linear(hidden, 1)
        self.activate_func = nn.Tanh()
        if use_orthogonal_init:
            self.orthogonal_init_all()

    def orthogonal_init_all(self):
        _orthogonal(self.fc1)
        _orthogonal(self.fc2)
        _orthogonal(self.fc3)

    def forward(self, s):
        s = self.activate_func(self.fc1(s))
        s = self.activate_func(self.fc2(s))
        return self.fc3(s)

    def init(self, use_orthogonal_init):
        if use_orthogonal_init:
            self.orthogonal_init_all()
        else:
            for m in (self.fc1, self.fc2, self.fc3):
                m.reset_parameters()


# ---------------------------------------------------------------------------------------------
# GPUNet: a driver-defined Linear/Tanh stack on librlp's MFMA kernels
# ---------------------------------------------------------------------------------------------
class GPUNet:
    """Runs `module`'s forward through librlp: the Linear layers (registration order) become an
    rlp_mlp_desc with tanh (PPO drivers) or ReLU (DDPG drivers) hidden activations — found by
    checking the module's own forward on a probe batch; an actor with `gain`/`off` gets
    tanh * gain + off on the last layer, a critic the identity. An architecture that matches
    neither raises instead of silently diverging."""

    def __init__(self, module: nn.Module, is_actor: bool, device="cuda", hidden_act=None):
        self.module = module
        self.is_actor = is_actor
        self.device = torch.device(device)
        self.linears = [m for m in module.modules() if isinstance(m, nn.Linear)]
        if not self.linears:
            raise ValueError("GPUNet: module has no nn.Linear layers")
        dims = [self.linears[0].in_features] + [l.out_features for l in self.linears]
        for a, b in zip(self.linears[:-1], self.linears[1:]):
            if a.out_features != b.in_features:
                raise ValueError("GPUNet: Linear layers do not chain")
        last = _abi.RLP_ACT_TANH if is_actor else _abi.RLP_ACT_NONE
        cands = [hidden_act] if hidden_act is not None else [_abi.RLP_ACT_TANH, _abi.RLP_ACT_RELU]
        err = None
        for act in cands:
            self.desc = _abi.MLPDesc.make(dims, [act] * (len(self.linears) - 1) + [last])
            self.packed = None
            self.flat = None
            self.refresh()
            err = self._mismatch()
            if err is None:
                break
        if err is not None:
            raise ValueError("GPUNet: module forward is not a Linear/Tanh or Linear/ReLU stack this "
                             f"adapter maps (max diff {err:.3g})")

    @property
    def mfma_ok(self):
        return self.packed is not None

    def refresh(self):
        """Re-read the module's parameters (call after every optimiser step)."""
        with torch.no_grad():
            region = self._params_region() if self.flat is not None else None
            if region is None or region.data_ptr() != self.flat.data_ptr():  # aliased: current
                self.flat = torch.cat([t.detach().reshape(-1).to(self.device, torch.float32)
                                       for l in self.linears for t in (l.weight, l.bias)]).contiguous()
            cnt = K.lib().rlp_mfma_packed_count(__import__("ctypes").byref(self.desc))
            self.packed = K.mfma_pack(self.desc, self.flat, out=self.packed) if cnt > 0 else None

    def _params_region(self):
        """The module's (weight, bias) tensors as one contiguous region of a single buffer (a
        native update's flat parameters: module parameters are views of it), or None."""
        ts = [t for l in self.linears for t in (l.weight, l.bias)]
        # against the flat buffer's device: self.device may be an index-less torch.device('cuda')
        # while the parameters report cuda:0
        if any(t.device != self.flat.device or t.dtype != torch.float32 or not t.is_contiguous()
               for t in ts):
            return None
        base = ts[0].data_ptr()
        off = 0
        for t in ts:
            if t.untyped_storage().data_ptr() != ts[0].untyped_storage().data_ptr() or \
                    t.data_ptr() != base + 4 * off:
                return None
            off += t.numel()
        st = ts[0].storage_offset()
        # detached: the alias is plain data (no autograd view of the parameters)
        return torch.as_strided(ts[0].detach(), (off,), (1,), st)

    def copy_from_module(self):
        """refresh() in place (graph-capturable: the same flat / packed tensors). When the
        module's parameters are views of one flat buffer in this layout (a native update's), the
        flat tensor aliases it and nothing is copied; otherwise one torch.cat launch."""
        with torch.no_grad():
            region = self._params_region()
            if region is not None and region.data_ptr() == self.flat.data_ptr():
                pass  # aliased: already current
            elif region is not None and region.numel() == self.flat.numel():
                self.flat = region  # alias from now on (the first call runs before a capture)
            else:
                torch.cat([t.reshape(-1) for l in self.linears for t in (l.weight, l.bias)],
                          out=self.flat)
            if self.packed is not None:
                K.mfma_pack(self.desc, self.flat, out=self.packed)

    def raw(self, x):
        """Last-layer output (tanh already applied for an actor, before gain/off)."""
        x = x.to(self.device, torch.float32).contiguous()
        if self.packed is not None and self.desc.dims[1] == 256:
            return K.mfma_forward(self.desc, self.packed, x)
        return K.mlp_forward(self.desc, self.flat, x)

    def __call__(self, x):
        y = self.raw(x)
        if self.is_actor:
            gain = torch.as_tensor(self.module.gain, device=self.device)
            off = torch.as_tensor(self.module.off, device=self.device)
            y = y * gain + off
        return y

    def _mismatch(self):
        """None if the mapping reproduces module(x) on a probe batch, else the max difference."""
        g = torch.Generator().manual_seed(0)
        x = torch.rand(64, self.desc.dims[0], generator=g) * 4 - 2
        with torch.no_grad():
            p = next(self.module.parameters())
            ref = self.module(x.to(p.device, p.dtype)).float().to(self.device)
        got = self(x.to(self.device))
        if torch.allclose(got, ref, rtol=1e-4, atol=1e-4):
            return None
        return float((got - ref).abs().max())


# ---------------------------------------------------------------------------------------------
# SAC networks: utils/classes.py:438-527 (SACActor / SACCritic). With std_min / std_scale given,
# SACActor is the SAC demo drivers' copy (demonstration/SAC/SAC-4-UGVForward/train.py:33-88),
# whose log_std clamp is per action dim instead of (-20, 2). Parameter names match the
# reference so state_dicts load unchanged.
# ---------------------------------------------------------------------------------------------
class SACActor(nn.Module):
    def __init__(self, state_dim: int = 3, action_dim: int = 3, a_min=np.zeros(3), a_max=np.ones(3),
                 use_orthogonal_init: bool = True, std_min=None, std_scale=None):
        super().__init__()
        self.fc1 = nn.Linear(state_dim, 128)
        self.fc2 = nn.Linear(128, 64)
        self.mean_layer = nn.Linear(64, action_dim)
        self.log_std_layer = nn.Linear(64, action_dim)
        self.a_min = torch.tensor(a_min, dtype=torch.float)
        self.a_max = torch.tensor(a_max, dtype=torch.float)
        self.off = (self.a_min + self.a_max) / 2.0
        self.gain = self.a_max - self.off
        self.std_min, self.std_scale = std_min, std_scale
        if use_orthogonal_init:
            self.orthogonal_init_all()

    def orthogonal_init_all(self):
        _orthogonal(self.fc1)
        _orthogonal(self.fc2)
        _orthogonal(self.mean_layer, gain=0.01)
        _orthogonal(self.log_std_layer, gain=0.01)

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)
        self.a_min, self.a_max = fn(self.a_min), fn(self.a_max)
        self.off, self.gain = fn(self.off), fn(self.gain)
        return self

    def log_std_bounds(self):
        """(lo, hi) of the log_std clamp, per action dim, float32 — as forward() computes them."""
        A = self.mean_layer.out_features
        if self.std_min is None:
            return torch.full((A,), -20.0), torch.full((A,), 2.0)
        lo = torch.log(self.std_min * (self.a_max - self.a_min) / 2)
        hi = (self.a_max - self.a_min) / 2 / self.std_scale
        return lo.cpu(), hi.cpu()

    def forward(self, x, deterministic=False, with_logprob=True):
        x = torch.relu(self.fc1(x))
        x = torch.relu(self.fc2(x))
        mean = self.mean_layer(x)
        log_std = self.log_std_layer(x)
        if self.std_min is None:
            log_std = torch.clamp(log_std, -20, 2)
        else:
            log_std = torch.clamp(log_std, torch.log(self.std_min * (self.a_max - self.a_min) / 2),
                                  (self.a_max - self.a_min) / 2 / self.std_scale)
        std = torch.exp(log_std)
        dist = torch.distributions.Normal(mean, std)
        a = mean if deterministic else dist.rsample()
        if with_logprob:  # Spinning Up's tanh-squash correction
            log_pi = dist.log_prob(a).sum(dim=1, keepdim=True)
            log_pi -= (2 * (np.log(2) - a - torch.nn.functional.softplus(-2 * a))).sum(dim=1, keepdim=True)
        else:
            log_pi = None
        a = torch.tanh(a) * self.gain + self.off
        return a, log_pi


class SACCritic(nn.Module):
    def __init__(self, state_dim: int = 3, action_dim: int = 1, use_orthogonal_init: bool = True):
        super().__init__()
        self.fc1 = nn.Linear(state_dim + action_dim, 128)
        self.fc2 = nn.Linear(128, 64)
        self.fc3 = nn.Linear(64, 1)
        self.fc4 = nn.Linear(state_dim + action_dim, 128)
        self.fc5 = nn.Linear(128, 64)
        self.fc6 = nn.Linear(64, 1)
        if use_orthogonal_init:
            self.orthogonal_init_all()

    def orthogonal_init_all(self):
        for m in (self.fc1, self.fc2, self.fc3, self.fc4, self.fc5, self.fc6):
            _orthogonal(m)

    def forward(self, s, a):
        s_a = torch.cat([s, a], 1)
        q1 = self.fc3(torch.relu(self.fc2(torch.relu(self.fc1(s_a)))))
        q2 = self.fc6(torch.relu(self.fc5(torch.relu(self.fc4(s_a)))))
        return q1, q2


class GPUSACActor:
    """SACActor.forward for a batch on librlp: the ReLU trunk + both heads as one
    [S -> 128 -> 64 -> 2A] MLP (rlp_mlp_forward) and the squashed-Gaussian sample, log-prob and
    action clamp in rlp_sac_sample (Philox noise)."""

    def __init__(self, actor: SACActor, device="cuda"):
        self.actor = actor
        self.device = torch.device(device)
        S, A = actor.fc1.in_features, actor.mean_layer.out_features
        self.A = A
        self.desc = _abi.MLPDesc.make([S, 128, 64, 2 * A], [_abi.RLP_ACT_RELU, _abi.RLP_ACT_RELU,
                                                             _abi.RLP_ACT_NONE])
        self.refresh()

    def refresh(self):
        a = self.actor
        with torch.no_grad():
            parts = [a.fc1.weight, a.fc1.bias, a.fc2.weight, a.fc2.bias,
                     torch.cat([a.mean_layer.weight, a.log_std_layer.weight], 0),
                     torch.cat([a.mean_layer.bias, a.log_std_layer.bias], 0)]
            self.flat = torch.cat([t.detach().reshape(-1).to(self.device, torch.float32)
                                   for t in parts]).contiguous()
        lo, hi = a.log_std_bounds()
        self.ls_lo, self.ls_hi = lo.tolist(), hi.tolist()
        self.gain, self.off = a.gain.cpu().tolist(), a.off.cpu().tolist()

    def copy_from_actor(self):
        """refresh() of the weights in place (graph-capturable: no new tensors; one launch)."""
        a = self.actor
        with torch.no_grad():
            torch.cat([t.reshape(-1) for t in (a.fc1.weight, a.fc1.bias, a.fc2.weight, a.fc2.bias,
                                               a.mean_layer.weight, a.log_std_layer.weight,
                                               a.mean_layer.bias, a.log_std_layer.bias)],
                      out=self.flat)

    def head(self, s):
        return K.mlp_forward(self.desc, self.flat, s.to(self.device, torch.float32).contiguous())

    def __call__(self, s, deterministic=False, with_logprob=True, a_min=None, a_max=None,
                 seed=0, counter=0, env_id0=0, noise=None):
        return K.sac_sample(self.head(s), self.ls_lo, self.ls_hi, self.gain, self.off, a_min, a_max,
                            deterministic, noise, seed, counter, env_id0, with_logprob)
