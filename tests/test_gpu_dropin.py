"""GPU tests of the drop-in surface: rl_base envs, Proximal_Policy_Optimization2, VecPPO2 and
Distributed_PPO2 used the way the reference's demonstration drivers use them."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd.algorithm.policy_base.Distributed_PPO2 import Distributed_PPO2
from reinforcementlearningplatform_amd.algorithm.policy_base.Proximal_Policy_Optimization2 import \
    Proximal_Policy_Optimization2 as PPO2
from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import VecPPO2
from reinforcementlearningplatform_amd.environment.CartPole.CartPole import CartPole
from reinforcementlearningplatform_amd.environment.CartPole.CartPoleAngleOnly import CartPoleAngleOnly
from reinforcementlearningplatform_amd.environment.UavRobust.UavHoverOuterLoop import uav_hover_outer_loop
from reinforcementlearningplatform_amd.environment.UGV.UGVForward import UGVForward
from reinforcementlearningplatform_amd.environment.SecondOrderIntegration.SecondOrderIntegration import \
    SecondOrderIntegration
from reinforcementlearningplatform_amd.utils.classes import Normalization, PPOActor_Gaussian, PPOCritic

pytestmark = pytest.mark.gpu

PPO_MSG = {'gamma': 0.999, 'K_epochs': 3, 'eps_clip': 0.2, 'buffer_size': 200, 'state_dim': 4,
           'action_dim': 1, 'a_lr': 3e-4, 'c_lr': 1e-3, 'set_adam_eps': True, 'lmd': 0.95,
           'use_adv_norm': True, 'mini_batch_size': 64, 'entropy_coef': 0.01, 'use_grad_clip': False,
           'use_lr_decay': False, 'max_train_steps': int(5e6), 'using_mini_batch': False}


def shipped_actor_critic(golden, std=8 / 3):
    g = golden("ppo2_cartpole_nets")
    actor = PPOActor_Gaussian(4, 1, np.array([-8.]), np.array([8.]), init_std=std)
    critic = PPOCritic(4)
    for m, flat in ((actor, g["actor_params"]), (critic, g["critic_params"])):
        off = 0
        sd = {}
        for k, v in m.state_dict().items():
            sd[k] = torch.from_numpy(flat[off:off + v.numel()].reshape(v.shape).copy())
            off += v.numel()
        m.load_state_dict(sd)
    return actor, critic


@pytest.mark.parametrize("cls,kind,golden_name", [
    (CartPole, A.RLP_ENV_CARTPOLE, "cartpole_ppo2"),
    (lambda: CartPoleAngleOnly(variant="ppo2"), A.RLP_ENV_CARTPOLE_ANGLEONLY, "angleonly_ppo2"),
    (CartPoleAngleOnly, A.RLP_ENV_CARTPOLE_ANGLEONLY, "angleonly_env"),
    (SecondOrderIntegration, A.RLP_ENV_SOI, "soi_env"),
    (UGVForward, A.RLP_ENV_UGV_FORWARD, "ugvf_env"),
    (uav_hover_outer_loop, A.RLP_ENV_UAV_HOVER_OUTER_LOOP, "uav_hover")])
def test_env_single_matches_reference(golden, cls, kind, golden_name):
    """n_envs == 1 behaves like the reference's scalar env (teacher-forced golden steps)."""
    g = golden(golden_name)
    env = cls()
    for i in range(0, len(g["action"]), max(1, len(g["action"]) // 25)):
        env.set_physics(g["state"][i])
        env.current_state = env.next_state.copy()
        env.step_update(g["action"][i])
        np.testing.assert_allclose(env.next_state, g["obs_next"][i], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(env.current_state, g["obs_cur"][i], rtol=1e-6, atol=1e-7)
        assert abs(env.reward - g["reward"][i]) <= 1e-7 * abs(g["reward"][i]) + 1e-9
        assert env.terminal_flag == g["flag"][i] and env.is_terminal == bool(g["done"][i])
        np.testing.assert_allclose(env.physics(), g["state_next"][i], rtol=1e-9, atol=1e-12)
    assert isinstance(env.reward, float) and env.current_state.shape == (env.state_dim,)


def test_reset_law_and_batched_env():
    env = CartPole(0., 0., n_envs=20000, seed=3407)
    env.reset(random=True)
    th, x = env.theta, env.x
    assert np.abs(th).max() <= env.theta_max * 0.5 and np.abs(x).max() <= env.x_max * 0.5
    assert abs(th.mean()) < 0.01 and abs(th.std() * np.sqrt(3) / (env.theta_max * 0.5) - 1) < 0.03
    env2 = CartPole(0., 0., n_envs=20000, seed=3407)
    env2.reset(random=True)
    np.testing.assert_array_equal(env2.theta, th)            # Philox: reproducible per seed
    dppo2 = CartPole(0., 0., n_envs=20000, variant="dppo2", seed=1)
    dppo2.reset(random=True)
    assert np.abs(dppo2.theta).max() <= dppo2.theta_max / 3
    a = np.random.default_rng(0).uniform(-8, 8, (20000, 1)).astype(np.float32)
    st = env.physics().copy()
    env.step_update(a)
    _, on, r, f, d = oracle.env_step(A.RLP_ENV_CARTPOLE, env.params, st, a)
    np.testing.assert_allclose(env.next_state, on, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(env.reward, r, rtol=1e-8, atol=1e-9)


def test_ppo2_agent_shipped_net_and_known_answer(golden):
    actor, critic = shipped_actor_critic(golden)
    env = CartPole(0., 0.)
    env_msg = {'state_dim': 4, 'action_dim': 1, 'name': env.name, 'action_range': env.action_range}
    agent = PPO2(env_msg, PPO_MSG, actor, critic)
    assert abs(agent.evaluate([0.1, -0.2, 0.3, 0.05])[0] - 7.99988604) < 2e-6
    g = golden("ppo2_cartpole_nets")
    obs = g["loop_a_obs"]
    acts = np.stack([agent.evaluate(o) for o in obs[:50]])
    np.testing.assert_allclose(acts, g["loop_a_action"][:50], rtol=1e-5, atol=2e-5)
    # free-running closed loop (chaotic: only the 237-step time-out and the return's size)
    env = CartPole(0.3, 0.5)
    env.reset(False)
    ret, steps = 0.0, 0
    while not env.is_terminal:
        env.current_state = env.next_state.copy()
        env.step_update(agent.evaluate(env.current_state))
        ret += env.reward
        steps += 1
    assert steps == 237 and env.terminal_flag == 3
    assert abs(ret - g["loop_a_reward"].sum()) < 0.1 * abs(g["loop_a_reward"].sum())


def test_ppo2_driver_loop_and_checkpoint(tmp_path):
    """demonstration/PPO2/PPO2-4-CartPole/train.py:183-264 with this package's classes."""
    np.random.seed(0)
    env = CartPole(0., 0.)
    reward_norm = Normalization(shape=1)
    env_msg = {'state_dim': env.state_dim, 'action_dim': env.action_dim, 'name': env.name,
               'action_range': env.action_range}
    agent = PPO2(env_msg, PPO_MSG,
                 actor=PPOActor_Gaussian(state_dim=4, action_dim=1, a_min=np.array(env.action_range)[:, 0],
                                         a_max=np.array(env.action_range)[:, 1], init_std=env.fm / 3),
                 critic=PPOCritic(state_dim=4))
    env.is_terminal = True
    idx, episodes = 0, 0
    while idx < agent.buffer.batch_size:
        if env.is_terminal:
            env.reset(random=True)
            episodes += 1
        else:
            env.current_state = env.next_state.copy()
            a, lp = agent.choose_action(env.current_state)
            assert a.dtype == np.float32 and abs(a[0]) <= 8
            env.step_update(a)
            success = 0 if (not env.is_terminal or env.terminal_flag == 3) else 1
            agent.buffer.append(s=env.current_state, a=a, log_prob=lp, r=reward_norm(env.reward),
                                s_=env.next_state, done=1.0 if env.is_terminal else 0.0,
                                success=success, index=idx)
            idx += 1
    before = [p.detach().clone() for p in agent.actor.parameters()]
    agent.learn(200, buf_num=1)
    assert any(not torch.equal(b, p) for b, p in zip(before, agent.actor.parameters()))
    assert all(torch.isfinite(p).all() for p in agent.critic.parameters())
    agent.save_ac(msg='', path=str(tmp_path) + '/')
    sd = torch.load(str(tmp_path / 'actor'), weights_only=True)
    assert set(sd) == {'fc1.weight', 'fc1.bias', 'fc2.weight', 'fc2.bias', 'mean_layer.weight',
                       'mean_layer.bias'}
    # choose_action after learn() uses the refreshed weights
    np.testing.assert_allclose(agent.evaluate(env.next_state),
                               agent.actor(torch.tensor(env.next_state, dtype=torch.float,
                                                        device="cuda").view(1, -1)).detach().cpu().numpy().ravel(),
                               rtol=1e-5, atol=1e-5)


def test_learn_gae_matches_reference(golden):
    g = golden("gae")
    actor, critic = PPOActor_Gaussian(1, 1), PPOCritic(1)
    agent = PPO2({'state_dim': 1, 'action_dim': 1, 'name': 'g', 'action_range': [[-1, 1]]},
                 dict(PPO_MSG, buffer_size=1000, state_dim=1), actor, critic)
    t = lambda k: torch.tensor(g[f"c1_{k}"].astype(np.float32), device="cuda")
    adv, vt = agent.compute_gae(t("r"), t("v"), t("vn"), t("done"), t("success"))
    np.testing.assert_array_equal(adv.cpu().numpy().ravel(), g["c1_adv"])
    np.testing.assert_array_equal(vt.cpu().numpy().ravel(), g["c1_v_target"])


def _oa_env(n_envs, seed, **kw):
    from reinforcementlearningplatform_amd.environment.UGVForwardObstacleAvoidance import \
        UGVForwardObstacleAvoidance
    return UGVForwardObstacleAvoidance(n_envs=n_envs, seed=seed, variant="ppo2", **kw)


@pytest.mark.parametrize("cls,kwargs", [(CartPole, {}), (uav_hover_outer_loop, {}), (_oa_env, {})],
                         ids=["cartpole", "uav", "ugv_obstacle_avoidance"])
def test_vec_ppo2_iterations(cls, kwargs):
    """VecPPO2 iterations (rlp_rollout + advantages + K epochs); the lidar env's 41-input nets
    (the PPO2-UGVForwardObstacleAvoidance demo shape) roll out through rlp_rollout's per-step
    kernel sequence and update on librlp's f16x3 kernels with layer 1 on the exact-f32 GEMM
    (learner='auto' picks the native learner for every Linear/Tanh stack; mini-batches of the
    41-input nets are gathered before the gradient)."""
    env = cls(n_envs=4096, seed=5, **kwargs)
    ar = np.array(env.action_range)
    actor = PPOActor_Gaussian(env.state_dim, env.action_dim, ar[:, 0], ar[:, 1],
                              init_std=float((ar[0, 1] - ar[0, 0]) / 6))
    critic = PPOCritic(env.state_dim)
    agent = VecPPO2(env, actor, critic, {'K_epochs': 2, 'using_mini_batch': True,
                                         'mini_batch_size': 32768}, T=32)
    assert type(agent.learner).__name__ == "NativePPO2Learner"
    assert not agent.learner.net_a.dense and agent.learner.net_a.ext == (env.state_dim > 8)
    for _ in range(3):
        out = agent.iteration()
    assert torch.isfinite(out["actor_loss"]) and torch.isfinite(out["critic_loss"])
    st = agent.episode_stats()
    assert np.isfinite(st["mean_reward"]) and sum(st["flags"]) == 4096 * 32


def test_dppo2_single_process(tmp_path):
    env = CartPole(n_envs=2048, seed=3)
    eval_env = CartPole()
    ag = Distributed_PPO2(env, actor_lr=1e-4, critic_lr=1e-3, num_of_pro=1, path=str(tmp_path) + '/',
                          ppo_msg={'k_epo': 2, 'gamma': 0.99}, T=16, eval_env=eval_env)
    rec = ag.start_multi_process(iterations=2, eval_every=2)
    assert len(rec) == 2 and os.path.exists(str(tmp_path) + '/trainNum_2/actor')
    assert len(ag.evaluate_record[-1]) == 10
