"""uav_hover_outer_loop — environment/UavRobust/UavHoverOuterLoop.py on MI355X: the 6-DoF
quadrotor (uav.py) with its FNTSMC attitude loop (FNTSMC.py) inside the env step, the RL action
being the outer-loop virtual acceleration. The FNTSMC integrator s1 and the attitude reference
are carried across resets, as in the reference (UavHoverOuterLoop.py:152-208)."""
import numpy as np

from ... import _abi
from .._vec import VecEnv


class uav_hover_outer_loop(VecEnv):
    KIND = _abi.RLP_ENV_UAV_HOVER_OUTER_LOOP
    TIME_INDEX = 12

    def __init__(self, params=None, target0=np.array([-1, 3, 2]), n_envs: int = 1, device=None,
                 seed=None, env_id0=0):
        p = params if params is not None else _abi.uav_hover_params()
        super().__init__(p, n_envs, device, seed, env_id0)
        self.name = 'uav_hover_outer_loop'
        self.target0 = np.array(target0, float)
        self.dt, self.time_max = p.dt, p.time_max
        self.action_range = [[p.u_min, p.u_max]] * 3
        self.msg_print_flag = False
        self.reset(random=False)

    def initial_physics(self):
        p = self.params
        st = np.zeros(self._D)
        st[0:3], st[3:6], st[6:9], st[9:12] = p.pos0[:], p.vel0[:], p.angle0[:], p.pqr0[:]
        st[13:16] = self.target0
        return st

    def reset(self, random: bool = False, mask=None):
        if not random and getattr(self, "_carry_ready", False):
            # keep s1 / att_ref (hidden controller state) across a deterministic reset too
            keep = self.state[16:22].clone()
            super().reset(random=False, mask=mask)
            self.state[16:22] = keep
            return
        super().reset(random=random, mask=mask)
        self._carry_ready = True

    pos_ref = property(lambda self: self.physics()[13:16])

    def uav_pos(self):
        return self.physics()[0:3]

    def uav_vel(self):
        return self.physics()[3:6]

    def uav_att(self):
        return self.physics()[6:9]
