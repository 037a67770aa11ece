"""UGVForward (unicycle, forward only) — environment/UGV/UGVForward.py on MI355X; variant
'ppo2' / 'dppo2' selects the demo copies' deltas."""
import numpy as np

from ... import _abi
from .._vec import VecEnv


class UGVForward(VecEnv):
    KIND = _abi.RLP_ENV_UGV_FORWARD
    TIME_INDEX = 5

    def __init__(self, pos0=np.array([1., 1.]), vel0: float = 0., phi0: float = 0., omega0: float = 0.,
                 map_size=np.array([5.0, 5.0]), target=np.array([2.5, 2.5]), n_envs: int = 1,
                 variant="env", device=None, seed=None, env_id0=0):
        p = _abi.ugv_params(self.KIND, variant)
        p.map_size[0], p.map_size[1] = float(map_size[0]), float(map_size[1])
        super().__init__(p, n_envs, device, seed, env_id0)
        self.name = 'UGVForward' if self.KIND == _abi.RLP_ENV_UGV_FORWARD else 'UGVBidirectional'
        self.init_pos, self.init_vel, self.init_phi, self.init_omega = \
            np.array(pos0, float), vel0, phi0, omega0
        self.map_size, self.init_target = np.array(map_size, float), np.array(target, float)
        self.dt, self.time_max, self.v_max = p.dt, p.time_max, p.v_max
        self.e_max = np.linalg.norm(self.map_size) / 2
        self.reset(random=False)

    def initial_physics(self):
        return np.array([*self.init_pos, self.init_vel, self.init_phi, self.init_omega, 0.,
                         *self.init_target])

    pos = property(lambda self: np.array([self._component(0), self._component(1)]))
    vel = property(lambda self: self._component(2))
    phi = property(lambda self: self._component(3))
    omega = property(lambda self: self._component(4))
