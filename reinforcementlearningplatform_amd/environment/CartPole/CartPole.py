"""CartPole (angle + position, 4 observations) — environment/CartPole/CartPole.py on MI355X.

Same constructor and rl_base attributes as the reference class; variant='dppo2' selects the
reset law of demonstration/DPPO2/DPPO2-4-CartPole/CartPole.py:273-274."""
import numpy as np

from ... import _abi
from .._vec import VecEnv


class CartPole(VecEnv):
    KIND = _abi.RLP_ENV_CARTPOLE
    TIME_INDEX = 4

    def __init__(self, initTheta: float = 0., initX: float = 0., n_envs: int = 1, variant="ppo2",
                 device=None, seed=None, env_id0=0):
        p = _abi.cartpole_params(variant)
        super().__init__(p, n_envs, device, seed, env_id0)
        self.name = 'CartPole'
        self.initTheta, self.initX = initTheta, initX
        self.theta_max, self.dtheta_max = p.theta_max, p.dtheta_max
        self.x_max, self.dx_max, self.staticGain = p.x_max, p.dx_max, p.static_gain
        self.M, self.m, self.g, self.ell, self.kf, self.fm = p.M, p.m, p.g, p.ell, p.kf, p.fm
        self.dt, self.timeMax = p.dt, p.time_max
        self.state_range = [[-self.theta_max, self.theta_max], [-self.dtheta_max, self.dtheta_max],
                            [-self.x_max, self.x_max], [-self.dx_max, self.dx_max]]
        self.reset(random=False)

    def initial_physics(self):
        return np.array([self.initTheta, 0., self.initX, 0., 0.])

    theta = property(lambda self: self._component(0))
    dtheta = property(lambda self: self._component(1))
    x = property(lambda self: self._component(2))
    dx = property(lambda self: self._component(3))
    etheta = property(lambda self: 0. - self._component(0))
    ex = property(lambda self: 0. - self._component(2))

    @property
    def force(self):
        a = np.asarray(self.current_action, dtype=float)
        return float(a.reshape(-1)[0]) if self.n_envs == 1 else a.reshape(self.n_envs, -1)[:, 0]
