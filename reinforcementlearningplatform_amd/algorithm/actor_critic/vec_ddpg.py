"""VecDDPG — the DDPG-SOI driver loop (demonstration/DDPG/DDPG-4-SecondOrderIntegration/
train.py:205-251) over n envs on one GPU, replay buffer in HBM (BASELINE config 3).

One step() = for every env: actor forward (librlp MLP kernel), N(0, sigma^2) exploration + clip
(rlp_policy_sample), env step (rlp_env_step, the DDPG copy of SecondOrderIntegration), n
transitions into the replay ring (rlp_replay_store, env order), auto-reset of terminated envs
(rlp_env_reset, Philox) — then `learn_iters` DDPG updates of `batch_size` rows sampled from HBM
(rlp_replay_sample_uniform + rlp_replay_gather). Nothing round-trips through the host.
"""
import numpy as np
import torch

from ... import kernels as K


class VecDDPG:
    def __init__(self, env, agent, sigma0=None, learn_iters=1, is_reward_ascent=False):
        self.env, self.agent = env, agent
        self.n = env.n_envs
        self.kind, self.params = env.KIND, env.params
        lo, hi = np.asarray(env.action_range)[:, 0], np.asarray(env.action_range)[:, 1]
        self.sigma0 = np.asarray(sigma0 if sigma0 is not None else (hi - lo) / 2 / 3, np.float32)
        self.learn_iters = int(learn_iters)
        self.is_reward_ascent = is_reward_ascent
        self.obs = K.env_observe(self.kind, self.params, env.state)
        self.steps = 0

    def step(self, sigma=None, learn=True):
        sigma = self.sigma0 if sigma is None else np.asarray(sigma, np.float32)
        a = self.agent.choose_action(self.obs, False, sigma=sigma)
        oc, on, r, f, d = K.env_step(self.kind, self.params, self.env.state, a, want_obs_cur=False)
        mem = self.agent.memory
        K.replay_store(mem.rb, mem.mem_counter, self.obs, a, r, on, d)
        mem.mem_counter += self.n
        self.env.reset_counter += 1
        K.env_reset(self.kind, self.params, self.env.state, mask=d, seed=self.env.seed,
                    counter=self.env.reset_counter, env_id0=self.env.env_id0)
        self.obs = K.env_observe(self.kind, self.params, self.env.state, out=self.obs)
        self.steps += 1
        out = None
        if learn:
            out = self.agent.learn(is_reward_ascent=self.is_reward_ascent, iter=self.learn_iters)
        return r, d, out
