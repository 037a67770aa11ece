"""SecondOrderIntegration (2-D point mass) — environment/SecondOrderIntegration/
SecondOrderIntegration.py on MI355X; variant 'dppo2' / 'ddpg' selects the demo copies' deltas."""
import numpy as np

from ... import _abi
from .._vec import VecEnv


class SecondOrderIntegration(VecEnv):
    KIND = _abi.RLP_ENV_SOI
    TIME_INDEX = 4

    def __init__(self, pos0=np.array([1.0, 1.0]), vel0=np.array([0.0, 0.0]),
                 map_size=np.array([5.0, 5.0]), target=np.array([2.5, 2.5]), n_envs: int = 1,
                 variant="env", device=None, seed=None, env_id0=0):
        p = _abi.soi_params(variant)
        p.map_size[0], p.map_size[1] = float(map_size[0]), float(map_size[1])
        super().__init__(p, n_envs, device, seed, env_id0)
        self.name = 'SecondOrderIntegration'
        self.init_pos, self.init_vel = np.array(pos0, float), np.array(vel0, float)
        self.map_size, self.init_target = np.array(map_size, float), np.array(target, float)
        self.dt, self.time_max, self.vMax = p.dt, p.time_max, p.v_max
        self.fMax, self.fMin, self.k, self.mass = p.f_max, -p.f_max, p.k, p.mass
        self.static_gain = p.obs_gain
        self.reset(random=False)

    def initial_physics(self):
        return np.array([*self.init_pos, *self.init_vel, 0., *self.init_target])

    pos = property(lambda self: np.array([self._component(0), self._component(1)]))
    vel = property(lambda self: np.array([self._component(2), self._component(3)]))
    target = property(lambda self: np.array([self._component(5), self._component(6)]))
