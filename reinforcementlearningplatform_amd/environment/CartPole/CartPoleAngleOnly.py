"""CartPoleAngleOnly (2 observations) on MI355X.

variant 'env' (default, this module's reference path): environment/CartPole/CartPoleAngleOnly.py —
dt 0.01 in 10 RK4 sub-steps, fm 8, timeMax 6, the angle-increment reward, no success flag.
variant 'ppo2' (== 'dppo2'): the demo copy demonstration/PPO2/PPO2-4-CartPoleAngleOnly/
cartpole_angleonly.py that BASELINE config 1 trains (dt 0.02, fm 5, timeMax 5, quadratic reward)."""
import numpy as np

from ... import _abi
from .._vec import VecEnv


class CartPoleAngleOnly(VecEnv):
    KIND = _abi.RLP_ENV_CARTPOLE_ANGLEONLY
    TIME_INDEX = 4

    def __init__(self, initTheta: float = 0., n_envs: int = 1, variant="env", device=None,
                 seed=None, env_id0=0):
        p = _abi.angleonly_params(variant)
        super().__init__(p, n_envs, device, seed, env_id0)
        self.variant = variant
        self.name = 'CartPoleAngleOnly'
        self.initTheta = initTheta
        self.thetaMax, self.staticGain = p.theta_max, p.static_gain
        self.norm_4_boundless_state = p.norm_dtheta
        self.M, self.m, self.g, self.ell, self.kf, self.fm = p.M, p.m, p.g, p.ell, p.kf, p.fm
        self.dt, self.timeMax = p.dt, p.time_max
        if variant == "env":   # CartPoleAngleOnly.py:50-51, :60
            self.state_range = [[-self.thetaMax, self.thetaMax],
                                [-self.norm_4_boundless_state, self.norm_4_boundless_state]]
            self.action_range = np.array([[-self.fm, self.fm]])
        else:                  # cartpole_angleonly.py:52-53, :61
            self.state_range = [[-self.staticGain, self.staticGain], [-np.inf, np.inf]]
            self.action_range = [[-self.fm, self.fm]]
        self.reset(random=False)

    def initial_physics(self):
        return np.array([self.initTheta, 0., 0., 0., 0.])

    theta = property(lambda self: self._component(0))
    dtheta = property(lambda self: self._component(1))
    x = property(lambda self: self._component(2))
    dx = property(lambda self: self._component(3))
