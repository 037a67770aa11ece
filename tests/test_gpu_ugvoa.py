"""GPU parity of UGVForwardObstacleAvoidance: the HIP fake lidar / dynamics /
map generator behind the reference env API, against the reference's own step() outputs
(tests/golden/ugvoa_*.npz, made by tests/golden/make_golden.py) and the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle
from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd import kernels as K
from reinforcementlearningplatform_amd.environment.UGVForwardObstacleAvoidance import \
    UGVForwardObstacleAvoidance

from test_oracle_golden import check_oa_maps  # noqa: E402

pytestmark = pytest.mark.gpu
KIND = A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE


@pytest.mark.parametrize("variant", ["env", "ppo2", "dppo2"])
def test_env_class_vs_reference(golden, variant):
    """Batched env object, teacher-forced with the reference's states: the rl_base attributes
    (current_state, next_state, reward, terminal_flag, is_terminal) match the reference's step."""
    g = golden("ugvoa_" + variant)
    n = len(g["reward"])
    env = UGVForwardObstacleAvoidance(n_envs=n, variant=variant, seed=1)
    env.set_physics(g["state"].T)
    env.step_update(g["action"])
    np.testing.assert_allclose(env.current_state, g["obs_cur"].astype(np.float32), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(env.next_state, g["obs_next"].astype(np.float32), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(env.reward, g["reward"], rtol=1e-9, atol=1e-9)
    np.testing.assert_array_equal(env.terminal_flag, g["flag"])
    np.testing.assert_array_equal(env.is_terminal, g["done"].astype(bool))
    np.testing.assert_allclose(env.physics().T, g["state_next"], rtol=1e-9, atol=1e-12)


def test_scalar_env_api_and_replay_reset():
    """n_envs == 1 behaves like the reference object: shapes, Map.obs list, and reset(False)
    replaying the last random episode start (UGVForwardObstacleAvoidance.py:520-540)."""
    env = UGVForwardObstacleAvoidance(seed=3)
    assert env.state_dim == 41 and env.action_dim == 2 and env.current_state.shape == (41,)
    assert len(env.obs) == 10 and env.obs[0][0] == 'circle'
    start = env.physics().copy()
    for _ in range(5):
        env.step_update(np.array([1.0, 0.5], np.float32))
    assert env.time > 0.49
    env.reset(random=False)
    np.testing.assert_array_equal(env.physics(), start)
    env.reset(random=True)
    assert not np.array_equal(env.physics(), start)


@pytest.mark.parametrize("variant", ["env", "dppo2"])
def test_gpu_reset_maps_legal_and_bit_exact(variant):
    p = A.ugv_oa_params(variant)
    n = 65_536
    st = torch.zeros((A.RLP_UGVOA_D, n), dtype=torch.float64, device="cuda")
    K.env_reset(KIND, p, st, seed=11, counter=2, env_id0=77)
    got = st.cpu().numpy()
    placed = check_oa_maps(got, p)
    assert placed[:p.n_obs].mean() > (0.9999 if variant == "env" else 0.97)
    ref = np.zeros_like(got[:, :4096])
    oracle.env_reset(KIND, p, ref, seed=11, counter=2, env_id0=77)
    np.testing.assert_array_equal(got[:, :4096], ref)


def test_lidar_vs_oracle_rollout():
    """Closed loop: 40 steps of random actions with auto-reset on the GPU and in the oracle, from
    the same reset maps; every observation (4 + 37 beams) matches."""
    p = A.ugv_oa_params("env")
    n, T = 2048, 40
    rng = np.random.default_rng(9)
    st = np.zeros((A.RLP_UGVOA_D, n))
    oracle.env_reset(KIND, p, st, seed=5, counter=0)
    g = torch.from_numpy(st).cuda()
    lo, hi = A.action_bounds(KIND, p)
    for t in range(T):
        a = rng.uniform(lo, hi, (n, 2)).astype(np.float32)
        _, on, r, f, d = K.env_step(KIND, p, g, torch.from_numpy(a).cuda(), want_obs_cur=False)
        _, o_on, o_r, o_f, o_d = oracle.env_step(KIND, p, st, a, want_obs_cur=False)
        np.testing.assert_allclose(on.cpu().numpy(), o_on, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(r.cpu().numpy(), o_r, rtol=1e-8, atol=1e-9)
        np.testing.assert_array_equal(f.cpu().numpy(), o_f)
        K.env_reset(KIND, p, g, mask=d, seed=5, counter=t + 1)
        oracle.env_reset(KIND, p, st, mask=o_d, seed=5, counter=t + 1)
        np.testing.assert_allclose(g.cpu().numpy(), st, rtol=1e-9, atol=1e-12)
