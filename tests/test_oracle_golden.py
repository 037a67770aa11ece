"""Pin the CPU oracle (oracle/rlp_oracle.c) against the golden vectors the reference itself
produced (tests/golden/make_golden.py). CPU-only; these tests make the oracle a trustworthy
parity checker for the HIP kernels."""
import numpy as np
import pytest

from oracle import oracle
from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd import kernels as K

ENV_CASES = [
    ("cartpole_ppo2", A.RLP_ENV_CARTPOLE, lambda: A.cartpole_params("ppo2")),
    ("cartpole_dppo2", A.RLP_ENV_CARTPOLE, lambda: A.cartpole_params("dppo2")),
    ("angleonly_ppo2", A.RLP_ENV_CARTPOLE_ANGLEONLY, lambda: A.angleonly_params("ppo2")),
    ("angleonly_env", A.RLP_ENV_CARTPOLE_ANGLEONLY, lambda: A.angleonly_params("env")),
    ("soi_env", A.RLP_ENV_SOI, lambda: A.soi_params("env")),
    ("soi_dppo2", A.RLP_ENV_SOI, lambda: A.soi_params("dppo2")),
    ("ugvf_env", A.RLP_ENV_UGV_FORWARD, lambda: A.ugv_params(A.RLP_ENV_UGV_FORWARD, "env")),
    ("ugvf_ppo2", A.RLP_ENV_UGV_FORWARD, lambda: A.ugv_params(A.RLP_ENV_UGV_FORWARD, "ppo2")),
    ("ugvf_dppo2", A.RLP_ENV_UGV_FORWARD, lambda: A.ugv_params(A.RLP_ENV_UGV_FORWARD, "dppo2")),
    ("ugvb_env", A.RLP_ENV_UGV_BIDIRECTIONAL,
     lambda: A.ugv_params(A.RLP_ENV_UGV_BIDIRECTIONAL, "env")),
    ("ugvb_ppo2", A.RLP_ENV_UGV_BIDIRECTIONAL,
     lambda: A.ugv_params(A.RLP_ENV_UGV_BIDIRECTIONAL, "ppo2")),
    ("uav_hover", A.RLP_ENV_UAV_HOVER_OUTER_LOOP, A.uav_hover_params),
    ("ugvoa_env", A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE, lambda: A.ugv_oa_params("env")),
    ("ugvoa_ppo2", A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE, lambda: A.ugv_oa_params("ppo2")),
    ("ugvoa_dppo2", A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE, lambda: A.ugv_oa_params("dppo2")),
]


def _close(a, b, rtol, atol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b) - (atol + rtol * np.abs(b))
    return np.max(err) <= 0, float(np.max(np.abs(a - b)))


@pytest.mark.parametrize("name,kind,pf", ENV_CASES, ids=[c[0] for c in ENV_CASES])
def test_env_step_matches_reference(golden, name, kind, pf):
    g = golden(name)
    params = pf()
    state = np.ascontiguousarray(g["state"].T)  # [D][n]
    oc, on, r, f, d = oracle.env_step(kind, params, state, g["action"])
    # physics in f64: the same IEEE operations as numpy except libm ulps / BLAS sum order
    ok, e = _close(state.T, g["state_next"], 1e-9, 1e-12)
    assert ok, f"state_next max err {e}"
    ok, e = _close(oc, g["obs_cur"].astype(np.float32), 1e-6, 1e-7)
    assert ok, f"obs_cur max err {e}"
    ok, e = _close(on, g["obs_next"].astype(np.float32), 1e-6, 1e-7)
    assert ok, f"obs_next max err {e}"
    ok, e = _close(r, g["reward"], 1e-7, 1e-9)
    assert ok, f"reward max err {e}"
    np.testing.assert_array_equal(f, g["flag"])
    np.testing.assert_array_equal(d, g["done"])


def test_cartpole_substep_regimes(golden):
    """CartPole.rk44's fp64 `while time < tt` runs 10 sub-steps for the first 100 steps and mostly
    11 afterwards; an episode times out after 237 steps."""
    g = golden("cartpole_ppo2")
    tt = g["time_table"]
    p = A.cartpole_params()
    st = np.zeros((5, 1))
    times = []
    for k in range(len(tt)):
        times.append(st[4, 0])
        oracle.env_step(A.RLP_ENV_CARTPOLE, p, st, np.zeros((1, 1), np.float32))
    np.testing.assert_array_equal(np.array(times), tt)   # bit-identical fp64 time sequence
    assert np.argmax(np.array(times) + 0.02 > 5.0) <= 237


def _net_descs():
    act = A.MLPDesc.make([4, 256, 256, 1], [A.RLP_ACT_TANH] * 3)
    crit = A.MLPDesc.make([4, 256, 256, 1], [A.RLP_ACT_TANH, A.RLP_ACT_TANH, A.RLP_ACT_NONE])
    return act, crit


def test_mlp_forward_shipped_nets(golden):
    g = golden("ppo2_cartpole_nets")
    ad, cd = _net_descs()
    pre = oracle.mlp_forward(A.MLPDesc.make([4, 256, 256, 1], [1, 1, 0]), g["actor_params"], g["x"])
    np.testing.assert_allclose(pre, g["actor_pre"], rtol=1e-5, atol=2e-6)
    mean = oracle.mlp_forward(ad, g["actor_params"], g["x"]) * np.float32(8) + np.float32(0)
    np.testing.assert_allclose(mean, g["actor_mean"], rtol=1e-5, atol=2e-6)
    v = oracle.mlp_forward(cd, g["critic_params"], g["x"])
    np.testing.assert_allclose(v, g["critic_v"], rtol=1e-5, atol=2e-5)
    assert abs(mean[0, 0] - 7.99988604) < 1e-6 and abs(v[0, 0] - 42.18013000) < 2e-5


def test_policy_sample_logprob(golden):
    """choose_action: clamp(mean + std*eps) and Normal.log_prob of the clamped action."""
    g = golden("ppo2_cartpole_nets")
    mean = g["actor_mean"][:256]
    std = float(g["std"])
    a_ref, lp_ref = g["sample_a"], g["sample_logp"]
    eps = (a_ref.astype(np.float64) - mean) / std
    clamped = np.abs(a_ref) >= 8
    eps[clamped] = np.sign(a_ref[clamped]) * (np.abs(eps[clamped]) + 1.0)
    a, lp = oracle.policy_sample(mean, std, -8, 8, noise=eps.astype(np.float32))
    np.testing.assert_allclose(a, a_ref, atol=2e-6)
    np.testing.assert_allclose(lp, lp_ref, atol=2e-6)


@pytest.mark.parametrize("loop", ["a", "b"])
def test_closed_loop_known_answer(golden, loop):
    """Shipped PPO2-CartPole actor run deterministically: 237 steps, return -311.596200 (a) /
    -241.247217 (b).

    The shipped policy is bang-bang (|a| ~ 8), so the closed loop is chaotic: a 1e-8 difference in
    the fp32 MLP grows to O(1) by step ~80 (measured). Hence (1) exact parity is checked
    teacher-forced along the reference transcript (state rebuilt from the fp64 observation), and
    (2) the free-running loop only has to reach the time-out at 237 steps with a return of the
    same size."""
    g = golden("ppo2_cartpole_nets")
    ad, _ = _net_descs()
    p = A.cartpole_params()
    obs, act, rew = g[f"loop_{loop}_obs"], g[f"loop_{loop}_action"], g[f"loop_{loop}_reward"]
    tt = golden("cartpole_ppo2")["time_table"]
    # (1) teacher-forced transcript
    a_or = oracle.mlp_forward(ad, g["actor_params"], obs.astype(np.float32)) * np.float32(8)
    np.testing.assert_allclose(a_or, act, rtol=1e-5, atol=2e-5)
    scale = np.array([p.theta_max, p.dtheta_max, p.x_max, p.dx_max]) / p.static_gain
    st = np.concatenate([obs * scale, tt[:len(obs), None]], axis=1).T.copy()   # [5][237]
    _, on, r, f, d = oracle.env_step(A.RLP_ENV_CARTPOLE, p, st, act)
    np.testing.assert_allclose(on[:-1], obs[1:].astype(np.float32), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(r, rew, rtol=1e-9, atol=1e-9)
    assert d[-1] == 1 and not d[:-1].any() and f[-1] == 3
    # (2) free-running loop
    th0, x0 = g[f"loop_{loop}_init"]
    st = np.array([[th0], [0.], [x0], [0.], [0.]])
    ret, steps = 0.0, 0
    while True:
        o = oracle.env_observe(A.RLP_ENV_CARTPOLE, p, st)
        a = oracle.mlp_forward(ad, g["actor_params"], o) * np.float32(8)
        _, _, r, f, d = oracle.env_step(A.RLP_ENV_CARTPOLE, p, st, a)
        ret += r[0]
        steps += 1
        if d[0]:
            break
    assert steps == len(rew) == 237 and f[0] == 3
    np.testing.assert_allclose(ret, rew.sum(), rtol=0.1)


def test_gae_bit_exact(golden):
    g = golden("gae")
    for c in range(4):
        k = lambda n: g[f"c{c}_{n}"]
        T = len(k("r"))
        adv, vt = oracle.gae(k("r").reshape(T, 1), k("v").reshape(T, 1), k("vn").reshape(T, 1),
                             k("done").reshape(T, 1), k("success").reshape(T, 1),
                             float(g["gamma"]), float(g["lmd"]))
        np.testing.assert_array_equal(adv.ravel(), k("adv"))      # bit-exact (NumPy-2 fp32 order)
        np.testing.assert_array_equal(vt.ravel(), k("v_target"))
        a = adv.ravel()
        an = (a - a.mean(dtype=np.float64)) / (a.std(ddof=1, dtype=np.float64) + 1e-5)
        np.testing.assert_allclose(an, k("adv_norm"), rtol=2e-5, atol=2e-6)


def test_reward_normalisation(golden):
    g = golden("reward_norm")
    y, rms = oracle.reward_norm(g["x"].astype(np.float32).reshape(-1, 1))
    np.testing.assert_allclose(y.ravel(), g["y"], rtol=1e-5, atol=1e-6)
    assert y[0, 0] == 0.0 and abs(y[1, 0] - 0.99999999) < 1e-6   # first-call quirks


def test_reward_norm_batched_equals_merged_stats():
    """n > 1: the per-step merged statistics equal the statistics of all rewards so far."""
    rng = np.random.default_rng(0)
    r = rng.normal(-2, 3, (6, 257)).astype(np.float32)
    y, rms = oracle.reward_norm(r)
    allr = r.astype(np.float64).ravel()
    assert rms[0] == allr.size
    np.testing.assert_allclose(rms[1], allr.mean(), rtol=1e-12)
    np.testing.assert_allclose(rms[3], allr.std(), rtol=1e-10)


def check_oa_maps(state, p):
    """Structural properties of UGVForwardObstacleAvoidance reset maps ([D][n] physics state)
    against map.py:66-174's legality rules (shared with the GPU reset test)."""
    n = state.shape[1]
    S, T = state[0:2], state[6:8]
    m = p.st_margin
    assert (S >= m).all() and (S[0] <= p.map_size[0] - m).all() and (S[1] <= p.map_size[1] - m).all()
    assert (np.hypot(*(T - S)) >= p.safety_dis_st).all()
    assert (np.abs(state[3]) <= np.pi).all() and (state[[2, 4, 5]] == 0).all()
    C = state[8:].reshape(A.RLP_UGVOA_NOBS, 3, n)
    placed = C[:, 0] > -500
    assert not placed[p.n_obs:].any()
    for k in range(p.n_obs):
        ok = placed[k]
        c, r = C[k, :2][:, ok], C[k, 2][ok]
        assert ((r >= p.r_min) & (r <= p.r_max)).all()
        assert (c >= 0).all() and (c[0] <= p.map_size[0]).all() and (c[1] <= p.map_size[1]).all()
        assert (np.hypot(*(S[:, ok] - c)) > r + p.safety_dis_st).all()
        assert (np.hypot(*(T[:, ok] - c)) > r + p.safety_dis_st).all()
        for j in range(k):
            both = ok & placed[j]
            d = np.hypot(*(C[j, :2][:, both] - C[k, :2][:, both]))
            assert (d > C[j, 2][both] + C[k, 2][both] + p.safety_dis_obs).all()
    return placed


@pytest.mark.parametrize("variant", ["env", "dppo2"])
def test_ugvoa_reset_maps_legal(golden, variant):
    """The Philox rejection sampler obeys the reference generator's legality rules; with the
    default bound every obstacle of a 10-obstacle map is placed, and the radius distribution
    matches the reference's own maps (golden 'maps', drawn by map.py)."""
    p = A.ugv_oa_params(variant)
    n = 400
    st = np.zeros((A.RLP_UGVOA_D, n))
    oracle.env_reset(A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE, p, st, seed=7, counter=3)
    placed = check_oa_maps(st, p)
    frac = placed[:p.n_obs].mean()
    assert frac == 1.0 if variant == "env" else frac > 0.97
    ref_r = golden("ugvoa_" + variant)["maps"][..., 2].ravel()
    ours = st[10::3][:p.n_obs][placed[:p.n_obs]].ravel()
    assert abs(ours.mean() - ref_r.mean()) < 0.02


@pytest.mark.parametrize("kind", sorted(A.ROLLOUT_KINDS))
def test_oracle_forced_replay_reproduces_closed_loop(kind):
    """Teacher forcing with the oracle's own actions reproduces its closed loop bit for bit, with
    and without the nets (the GPU rollout parity tests replay the kernel's actions this way)."""
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind)
    rng = np.random.default_rng(kind)
    ad = A.MLPDesc.make([S, 32, 32, Ad], [1, 1, 1])
    cd = A.MLPDesc.make([S, 32, 32, 1], [1, 1, 0])
    ap = (rng.normal(0, 1, ad.param_count()) / 4).astype(np.float32)
    cp = (rng.normal(0, 1, cd.param_count()) / 4).astype(np.float32)
    lo, hi = A.action_bounds(kind, p)
    n, T = 67, 40
    cfg = K.make_rollout_cfg(T, n, 9, 0, 0, [(h - l) / 3 for l, h in zip(lo, hi)], lo, hi,
                             A.RLP_SUCCESS_DONE_AND_FLAG_NE, A.timeout_flag(kind))
    st0, need0 = np.zeros((D, n)), np.ones(n, np.uint8)
    ref = oracle.rollout(kind, p, st0, need0, ad, ap, cd, cp, cfg)
    for nets in (True, False):
        st, need = np.zeros((D, n)), np.ones(n, np.uint8)
        args = (ad, ap, cd, cp) if nets else (None, None, None, None)
        out = oracle.rollout(kind, p, st, need, *args, cfg, forced_action=ref["action"])
        keys = ref.keys() if nets else ("obs", "obs_next", "reward", "done", "success", "flag")
        for key in keys:
            np.testing.assert_array_equal(out[key], ref[key], err_msg=key)
        np.testing.assert_array_equal(st, st0)
        np.testing.assert_array_equal(need, need0)
