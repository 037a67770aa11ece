"""rl_base — the environment interface the reference's drivers program against
(algorithm/rl_base.py:4-162). Attribute names and method signatures are kept; the batched envs
of this package add a leading env axis to the per-step attributes when n_envs > 1."""


class rl_base:
    def __init__(self):
        self.state_dim = 0          # dimension of the RL state (observation)
        self.state_num = []         # per-dimension cardinality (inf for continuous)
        self.state_step = []        # per-dimension step (None for continuous)
        self.state_space = []       # per-dimension value list (None for continuous)
        self.isStateContinuous = []
        self.action_dim = 0
        self.action_num = []
        self.action_step = []
        self.action_space = []
        self.isActionContinuous = []
        self.state_range = []       # [[min, max], ...]
        self.action_range = []      # [[min, max], ...]
        self.use_norm = True
        self.current_state = []
        self.next_state = []
        self.current_action = []
        self.reward = 0.0
        self.is_terminal = False

    def step_update(self, action):
        pass

    def get_reward(self, param=None):
        return 0.

    def is_Terminal(self, param=None):
        return False

    def draw_init_image(self):
        pass

    def visualization(self):
        pass

    def get_state(self):
        return []

    def reset(self, random: bool = True):
        pass
