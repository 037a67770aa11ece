"""VecSAC — the SAC driver loop (demonstration/SAC/SAC-4-UGVForward/train.py:216-253) over n envs
on one GPU, replay buffer in HBM (SURVEY §8(f) f3 / BASELINE config 5 with
UGVForwardObstacleAvoidance: 131 072 envs = 16 384 per GPU over 8 GPUs, env shards, no data-path
collective).

One step() = for every env: actor trunk (rlp_mlp_forward) + squashed-Gaussian sample + clamp
(rlp_sac_sample, Philox), env step (for the obstacle-avoidance env: rlp_lidar.hip's beam-per-lane
lidar kernel), n transitions into the replay ring (rlp_replay_store, env order) with the driver's
done argument `0.0 if is_terminal and terminal_flag != 3 else 1.0`, auto-reset of finished envs
(rlp_env_reset: on the GPU map generator) — then `learn_iters` SAC updates of `batch_size` rows
sampled from HBM. Nothing round-trips through the host.
"""
import torch

from ... import kernels as K


class VecSAC:
    def __init__(self, env, agent, learn_iters=1, is_reward_ascent=False, success_flag=3):
        self.env, self.agent = env, agent
        self.n = env.n_envs
        self.kind, self.params = env.KIND, env.params
        self.learn_iters = int(learn_iters)
        self.is_reward_ascent = is_reward_ascent
        self.success_flag = int(success_flag)
        self.obs = K.env_observe(self.kind, self.params, env.state)
        self.steps = 0

    def step(self, learn=True, deterministic=False):
        a = self.agent.choose_action(self.obs, deterministic=deterministic)
        _, on, r, f, d = K.env_step(self.kind, self.params, self.env.state, a, want_obs_cur=False)
        # train.py:241: store_transition(..., 0.0 if is_terminal and terminal_flag != 3 else 1.0)
        dw_arg = 1 - (d.bool() & (f != self.success_flag)).to(torch.uint8)
        mem = self.agent.memory
        K.replay_store(mem.rb, mem.mem_counter, self.obs, a, r, on, dw_arg)
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
