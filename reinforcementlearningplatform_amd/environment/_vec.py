"""VecEnv: the rl_base environment API over n_envs environments stepped by librlp's HIP kernels.

With n_envs == 1 an env behaves like the reference's scalar env (current_state / next_state are
shape-[S] float64 arrays, reward a float, is_terminal a bool); with n_envs > 1 every per-step
attribute gains a leading env axis. Physics state stays on the device in float64.

Randomness: reset(random=True) draws from a counter-based Philox stream keyed by (seed, reset
counter, env id) instead of numpy's global MT19937; `seed` defaults to a draw from numpy's global
RNG, so `np.random.seed(s)` before construction still makes a run reproducible.
"""
import numpy as np
import torch

from .. import _abi
from .. import kernels as K
from ..algorithm.rl_base import rl_base


class VecEnv(rl_base):
    KIND = None
    TIME_INDEX = None   # component of the physics state that holds env.time

    def __init__(self, params, n_envs: int = 1, device=None, seed=None, env_id0: int = 0):
        rl_base.__init__(self)
        self.params = params
        self.n_envs = int(n_envs)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        D, S, A = _abi.ENV_DIMS[self.KIND]
        self._D = D
        self.state_dim, self.action_dim = S, A
        self.state = torch.zeros((D, self.n_envs), dtype=torch.float64, device=self.device)
        self.seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
        self.reset_counter = 0
        self.env_id0 = int(env_id0)
        self.state_num = [np.inf] * S
        self.state_step = [None] * S
        self.state_space = [None] * S
        self.isStateContinuous = [True] * S
        self.action_num = [np.inf] * A
        self.action_step = [None] * A
        self.action_space = [None] * A
        self.isActionContinuous = True
        lo, hi = _abi.action_bounds(self.KIND, params)
        self.action_range = np.array([[l, h] for l, h in zip(lo, hi)], dtype=float)
        self.terminal_flag = 0

    # -- subclass hook: the deterministic (random=False) initial physics state, shape [D]
    def initial_physics(self) -> np.ndarray:
        raise NotImplementedError

    # -- subclass hooks for reset(random=False): the [D][n] device state it restores, and what a
    # random reset records (the obstacle-avoidance env replays its last random episode start)
    def _initial_state_tensor(self):
        init = np.repeat(self.initial_physics().reshape(self._D, 1), self.n_envs, axis=1)
        return torch.from_numpy(np.ascontiguousarray(init)).to(self.device)

    def _after_random_reset(self, mask):
        pass

    # -- helpers
    def _squeeze(self, x):
        x = x.detach().cpu().numpy()
        return x[0] if self.n_envs == 1 else x

    def physics(self):
        """Host copy of the physics state, [D] (n_envs == 1) or [D][n]."""
        st = self.state.cpu().numpy()
        return st[:, 0] if self.n_envs == 1 else st

    def set_physics(self, st):
        st = np.asarray(st, dtype=np.float64).reshape(self._D, -1)
        if st.shape[1] == 1 and self.n_envs > 1:
            st = np.repeat(st, self.n_envs, axis=1)
        self.state.copy_(torch.from_numpy(np.ascontiguousarray(st)))

    def _component(self, i):
        v = self.state[i].cpu().numpy()
        return float(v[0]) if self.n_envs == 1 else v

    @property
    def time(self):
        return self._component(self.TIME_INDEX)

    # -- rl_base API
    def get_state(self):
        obs = K.env_observe(self.KIND, self.params, self.state)
        return self._squeeze(obs).astype(np.float64)

    def reset(self, random: bool = False, mask=None):
        m = None
        if mask is not None:
            m = torch.as_tensor(np.asarray(mask, dtype=np.uint8), device=self.device)
        if random:
            K.env_reset(self.KIND, self.params, self.state, mask=m, seed=self.seed,
                        counter=self.reset_counter, env_id0=self.env_id0)
            self.reset_counter += 1
            self._after_random_reset(m)
        else:
            K.env_reset(self.KIND, self.params, self.state, mask=m,
                        init_state=self._initial_state_tensor())
        obs = self.get_state()
        self.current_state = obs.copy()
        self.next_state = obs.copy()
        self.current_action = np.zeros(self.action_dim) if self.n_envs == 1 else \
            np.zeros((self.n_envs, self.action_dim))
        if self.n_envs == 1:
            self.reward, self.is_terminal, self.terminal_flag = 0.0, False, 0
        else:
            self.reward = np.zeros(self.n_envs)
            self.is_terminal = np.zeros(self.n_envs, dtype=bool)
            self.terminal_flag = np.zeros(self.n_envs, dtype=np.int32)

    def step_update(self, action):
        """One env step for every env: action [A] (n_envs == 1) or [n][A]; float32 is the dtype
        choose_action hands over in the reference drivers."""
        a = np.asarray(action, dtype=np.float32).reshape(self.n_envs, self.action_dim)
        oc, on, r, f, d = K.env_step(self.KIND, self.params, self.state,
                                     torch.from_numpy(np.ascontiguousarray(a)).to(self.device))
        self.current_action = np.array(action, copy=True)
        self.current_state = self._squeeze(oc).astype(np.float64)
        self.next_state = self._squeeze(on).astype(np.float64)
        rr, ff, dd = r.cpu().numpy(), f.cpu().numpy(), d.cpu().numpy().astype(bool)
        if self.n_envs == 1:
            self.reward, self.terminal_flag, self.is_terminal = float(rr[0]), int(ff[0]), bool(dd[0])
        else:
            self.reward, self.terminal_flag, self.is_terminal = rr, ff, dd

    def is_Terminal(self, param=None):
        return self.is_terminal

    def get_reward(self, param=None):
        return self.reward

    def visualization(self):
        """OpenCV rendering is outside the accelerated path: no-op."""
        return None
