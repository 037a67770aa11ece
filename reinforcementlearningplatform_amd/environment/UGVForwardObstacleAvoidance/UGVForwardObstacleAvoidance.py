"""UGVForwardObstacleAvoidance (unicycle + 37-beam fake lidar against circular obstacles) —
environment/UGVForwardObstacleAvoidance/UGVForwardObstacleAvoidance.py on MI355X.

The lidar (get_fake_laser :274-397), the map generator (map.py:152-174) and the dynamics run in
librlp's HIP kernels, one env per lane, physics and obstacles resident in HBM as f64 SoA
[x y vel phi omega time tx ty | (cx cy r) x 15]. variant 'ppo2' / 'dppo2' selects the demo copies
(dt 0.05, shaped reward, obsNum 15 for DPPO2; see _abi.ugv_oa_params).

As in the reference, construction ends with reset(random=True), and reset(random=False) replays the
start, heading, target and obstacles of the last random reset.
"""
import numpy as np
import torch

from ... import _abi
from .._vec import VecEnv


class UGVForwardObstacleAvoidance(VecEnv):
    KIND = _abi.RLP_ENV_UGV_OBSTACLE_AVOIDANCE
    TIME_INDEX = 5

    def __init__(self, pos0=np.array([1., 1.]), phi0: float = 0., map_size=np.array([5.0, 5.0]),
                 target=np.array([2.5, 2.5]), n_envs: int = 1, variant="env", device=None,
                 seed=None, env_id0=0):
        p = _abi.ugv_oa_params(variant)
        p.map_size[0], p.map_size[1] = float(map_size[0]), float(map_size[1])
        super().__init__(p, n_envs, device, seed, env_id0)
        self.name = 'UGVForwardObstacleAvoidance'
        self.init_pos, self.init_phi = np.array(pos0, float), float(phi0)
        self.map_size, self.init_target = np.array(map_size, float), np.array(target, float)
        self.dt, self.time_max, self.v_max = p.dt, p.time_max, p.v_max
        self.e_max = np.linalg.norm(self.map_size) / 2
        self.e_phi_max, self.omega_max = p.e_phi_max, p.omega_max
        self.a_linear_max, self.a_angular_max = p.a_linear_max, p.a_angular_max
        self.r_vehicle = p.r_vehicle
        self.laserDis, self.laserBlind, self.laserRange = p.laser_dis, p.laser_blind, p.laser_range
        self.laserState = _abi.RLP_UGVOA_NLASER
        self.static_gain = p.static_gain
        self.obsNum = int(p.n_obs)
        self._episode_init = None
        self.reset(random=True)

    def initial_physics(self):
        ph = np.zeros(self._D)
        ph[[0, 1, 3, 6, 7]] = [*self.init_pos, self.init_phi, *self.init_target]
        ph[8::3], ph[9::3], ph[10::3] = -1000.0 - 10.0 * np.arange(_abi.RLP_UGVOA_NOBS), -1000.0, \
            self.params.r_min
        return ph

    def _after_random_reset(self, mask):
        if self._episode_init is None or mask is None:
            self._episode_init = self.state.clone()
        else:
            m = mask.bool()
            self._episode_init[:, m] = self.state[:, m]

    def _initial_state_tensor(self):
        if self._episode_init is None:
            return super()._initial_state_tensor()
        return self._episode_init

    pos = property(lambda self: np.array([self._component(0), self._component(1)]))
    vel = property(lambda self: self._component(2))
    phi = property(lambda self: self._component(3))
    omega = property(lambda self: self._component(4))
    target = property(lambda self: np.array([self._component(6), self._component(7)]))

    @property
    def obs(self):
        """Obstacles as the reference's Map.obs list [['circle', center, [r]], ...] (n_envs == 1),
        else an [n][obsNum][3] array of (cx, cy, r)."""
        st = self.state[8:8 + 3 * self.obsNum].reshape(self.obsNum, 3, self.n_envs)
        st = st.permute(2, 0, 1).cpu().numpy()
        if self.n_envs == 1:
            return [['circle', np.array(c[:2]), [float(c[2])]] for c in st[0]]
        return st

    def set_map(self, start, phi, target, obstacles, env=None):
        """Install one episode start (start [2], phi, target [2], obstacles [(cx, cy, r)]) in env
        `env` (all envs when None), as reset(random=False) would replay it."""
        ph = self.initial_physics()
        ph[[0, 1, 3, 6, 7]] = [start[0], start[1], phi, target[0], target[1]]
        for k, (cx, cy, r) in enumerate(obstacles):
            ph[8 + 3 * k:11 + 3 * k] = [cx, cy, r]
        t = torch.from_numpy(ph).to(self.state)
        if env is None:
            self.state.copy_(t.view(-1, 1).expand_as(self.state))
        else:
            self.state[:, env] = t
        self._episode_init = self.state.clone()
