"""N=1 PPO2 driver transcripts replayed through the drop-in classes on the GPU (SURVEY §8c, §4
tier 3; BASELINE config 1 = CartPoleAngleOnly PPO2 with one env, and the CartPole PPO2 demo).

tests/golden/ppo2_transcript_{cartpole,angleonly}.npz hold one buffer of the reference driver
loop (demonstration/PPO2/PPO2-4-CartPole/train.py:184-224 and the AngleOnly copy) — the episode
starts the env drew, the exploration noise choose_action drew, every buffer row, and the actor /
critic after the learn() that follows. The replay runs the same loop with the drop-in env
(environment/CartPole/*), Normalization, and Proximal_Policy_Optimization2 (the GPU MLP, the
Philox-free injected noise, librlp's env step), then learn(); buffer rows and after-weights are
compared with explicit bounds.
"""
import numpy as np
import pytest
import torch

from reinforcementlearningplatform_amd.algorithm.policy_base.Proximal_Policy_Optimization2 import \
    Proximal_Policy_Optimization2
from reinforcementlearningplatform_amd.environment.CartPole.CartPole import CartPole
from reinforcementlearningplatform_amd.environment.CartPole.CartPoleAngleOnly import CartPoleAngleOnly
from reinforcementlearningplatform_amd.utils.classes import (Normalization, PPOActor_Gaussian,
                                                             PPOCritic)

pytestmark = pytest.mark.gpu


def _load(m, flat):
    off = 0
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.as_tensor(flat[off:off + p.numel()]).view_as(p))
            off += p.numel()


def _replay(g, key, learner):
    if key == "cartpole":
        env = CartPole(0., 0.)
        over = {}
    else:
        env = CartPoleAngleOnly(0., variant="ppo2")
        over = {'use_grad_clip': True, 'use_lr_decay': True}
    ar = np.array(env.action_range)
    actor = PPOActor_Gaussian(env.state_dim, env.action_dim, ar[:, 0], ar[:, 1],
                              init_std=float(g["std"]))
    critic = PPOCritic(env.state_dim)
    _load(actor, g["before_actor"])
    _load(critic, g["before_critic"])
    B = int(g["B"])
    ppo_msg = {'gamma': 0.999, 'K_epochs': 30, 'eps_clip': 0.2, 'buffer_size': B,
               'state_dim': env.state_dim, 'action_dim': env.action_dim, 'a_lr': 3e-4, 'c_lr': 1e-3,
               'set_adam_eps': True, 'lmd': 0.95, 'use_adv_norm': True, 'mini_batch_size': 64,
               'entropy_coef': 0.01, 'use_grad_clip': False, 'use_lr_decay': False,
               'max_train_steps': int(5e6), 'using_mini_batch': False, **over}
    env_msg = {'state_dim': env.state_dim, 'action_dim': env.action_dim, 'name': env.name,
               'action_range': env.action_range}
    agent = Proximal_Policy_Optimization2(env_msg, ppo_msg, actor=actor, critic=critic,
                                          learner=learner)
    reward_norm = Normalization(shape=1)
    resets, noise = list(g["resets"]), g["noise"].reshape(-1, env.action_dim)
    env.is_terminal = True
    idx, k, j = 0, 0, 0
    raw = []
    while idx < B:                       # train.py:184-217
        if env.is_terminal:
            env.initTheta = float(resets[k][0])
            if key == "cartpole":
                env.initX = float(resets[k][1])
            env.reset(False)             # the recorded reset(True) draw
            k += 1
        else:
            env.current_state = env.next_state.copy()
            a, a_lp = agent.choose_action(env.current_state, noise=noise[j])
            j += 1
            env.step_update(a)
            success = 0 if (env.is_terminal and env.terminal_flag == 3) else \
                (1 if env.is_terminal else 0)
            raw.append(env.reward)
            agent.buffer.append(s=env.current_state, a=a, log_prob=a_lp, r=reward_norm(env.reward),
                                s_=env.next_state, done=1.0 if env.is_terminal else 0.0,
                                success=success, index=idx)
            idx += 1
    assert k == len(resets) and j == noise.shape[0]
    b = agent.buffer
    rows = dict(s=b.s, a=b.a, a_lp=b.a_lp, r=b.r[:, 0], s_=b.s_, done=b.done[:, 0],
                success=b.success[:, 0], raw_reward=np.array(raw))
    agent.learn(B, buf_num=1)
    flat = lambda m: torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
    return rows, flat(agent.actor), flat(agent.critic)


def _within(got, want, rtol, atol, what):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    err = np.abs(got - want)
    lim = atol + rtol * np.abs(want)
    assert (err <= lim).all(), f"{what}: max err {err.max():.3e}, {int((err > lim).sum())} outside"


@pytest.mark.parametrize("key", ["cartpole", "angleonly"])
@pytest.mark.parametrize("learner", ["torch", "native"])
def test_transcript_replay(golden, key, learner):
    g = golden(f"ppo2_transcript_{key}")
    rows, wa, wc = _replay(g, key, learner)
    # episode structure is exact: the same steps end the same episodes with the same flags
    np.testing.assert_array_equal(rows["done"], g["done"])
    np.testing.assert_array_equal(rows["success"], g["success"])
    # per-step values: the GPU's f32 MLP differs from torch's CPU GEMM by ~1e-7 relative and the
    # closed loop carries it forward along each episode (<= 250 steps, unstable dynamics)
    _within(rows["s"], g["s"], 1e-5, 1e-6, "s")
    _within(rows["s_"], g["s_"], 1e-5, 1e-6, "s_")
    _within(rows["a"], g["a"], 1e-5, 1e-5, "a")
    _within(rows["a_lp"], g["a_lp"], 1e-5, 1e-5, "a_lp")
    _within(rows["raw_reward"], g["raw_reward"], 1e-5, 1e-6, "raw reward")
    _within(rows["r"], g["r"], 1e-5, 1e-5, "normalised reward")
    # 30 full-batch Adam epochs on the replayed buffer
    _within(wa, g["after_actor"], 1e-5, 5e-6, "actor after learn()")
    _within(wc, g["after_critic"], 1e-5, 5e-6, "critic after learn()")
