"""GPU parity of the fused rollout (rlp_rollout, the bench's hot path) against the reference's own
vectors and the CPU oracle, with explicit bounds and no allowance for mismatching elements.

(1) The reference's shipped PPO2-CartPole actor/critic (demonstration/PPO2/PPO2-4-CartPole/
    datasave/net, tests/golden/ppo2_cartpole_nets.npz) run through the fused rollout in both
    hidden-layer arithmetics (f16x3 split, exact f32): env states are placed so that the step's
    observation equals the golden inputs (the reference's random x rows and its closed-loop
    transcripts, Proximal_Policy_Optimization2.py:62-76 / CartPole.py:145-153), exploration is
    switched off (std 1e-30: a == clamp(mean)), and the stored action / V(s) must equal the
    reference's actor(x) / critic(x) / evaluate() to rtol 1e-5, atol 2e-6 (V(s): plus 1e-6 of the
    output layer's summed term magnitudes, the scale at which any f32 evaluation rounds).
(2) Action-teacher-forced physics replay at the bench size (65 536 CartPole envs x T = 128, and
    the UAV bench shard 32 768 x 64): the oracle replays the driver loop (resets included, from the
    same Philox draws) with the kernel's stored f32 actions; the f64 env state after the segment
    must agree to 1e-9, flags / done / success / need_reset exactly, observations and rewards to
    float32 rounding.
(3) Every rollout kind and envs-per-wave variant against the oracle teacher-forced the same way,
    plus the oracle's own policy (double-accumulated MLP, same Philox noise) on the kernel's
    observations: action, log-prob, V(s), V(s') to rtol 1e-5 (atol: per row from the output
    layer's term magnitudes, policy_bounds / 2e-6).
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd import _native
from reinforcementlearningplatform_amd import kernels as K

pytestmark = pytest.mark.gpu


def dev(x):
    return torch.as_tensor(np.ascontiguousarray(x)).cuda()


def host(t):
    return t.detach().cpu().numpy()


def bound(a, b, rtol, atol, what):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b)
    bad = err > atol + rtol * np.abs(b)
    assert not bad.any(), (f"{what}: {int(bad.sum())} of {bad.size} outside rtol {rtol} / atol "
                           f"{atol}; max abs err {err.max():.3e}")
    return float(err.max()) if err.size else 0.0


def f32_ulps(a, b):
    """|a - b| in units of float32 spacing at b."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    sp = np.spacing(np.maximum(np.abs(a), np.abs(b)).astype(np.float32)).astype(np.float64)
    return np.abs(a.astype(np.float64) - b.astype(np.float64)) / np.maximum(sp, 1e-45)


def policy_bounds(ad, ap, obs, a_ref, lo, hi, std):
    """Per-row absolute bounds for action and log-prob in teacher-forced comparisons, derived the
    way the V(s) bound is: the mean is tanh(z3) * gain + off with z3 = sum_j w3_j h2_j + b3 (the
    last layer of any tanh stack), a 256-term sum whose f32 evaluations (the reference's, ours, the f16x3 split's 3 * 2^-22 per
    product) differ by ~1e-6 of the TERMS' magnitude S = sum_j |w3_j h2_j| + |b3| (float64 h2 on
    the row's observation), so |d mean| <= gain * sech^2(z3) * 1e-6 * S, plus f32 rounding of the
    output (1e-7 * gain). d logp / d mean = (a - mean) / std^2."""
    ds = ad.layer_dims()
    x = np.asarray(obs, np.float64).reshape(-1, ds[0])
    prm = np.asarray(ap, np.float64)
    off, h = 0, x
    for i in range(ad.n_layers):
        W = prm[off:off + ds[i + 1] * ds[i]].reshape(ds[i + 1], ds[i])
        off += W.size
        b = prm[off:off + ds[i + 1]]
        off += b.size
        if i < ad.n_layers - 1:
            h = np.tanh(h @ W.T + b)
        else:
            z3 = h @ W.T + b
            S = np.abs(h) @ np.abs(W).T + np.abs(b)
    gain = (np.asarray(hi, np.float64) - np.asarray(lo, np.float64)) / 2
    mean = np.tanh(z3) * gain + (np.asarray(hi, np.float64) + np.asarray(lo, np.float64)) / 2
    a_atol = 1e-7 * gain + gain * (1 - np.tanh(z3) ** 2) * 1e-6 * S
    if a_ref is None:
        return mean, a_atol
    var = np.asarray(std, np.float64) ** 2
    a = np.asarray(a_ref, np.float64).reshape(mean.shape)
    lp_atol = 2e-6 + a_atol * np.abs(a - mean) / var    # per action dim, as the buffer's logp
    shp = np.asarray(a_ref).shape
    return a_atol.reshape(shp), lp_atol.reshape(shp)


def bound_rows(a, b, rtol, atol_rows, what):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b)
    lim = atol_rows.reshape(err.shape) + rtol * np.abs(b)
    bad = err > lim
    assert not bad.any(), (f"{what}: {int(bad.sum())} of {bad.size} outside rtol {rtol} + derived "
                           f"atol; max excess {np.max(err - lim):.3e}")


def orthogonal(desc, gains, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    ds = desc.layer_dims()
    for i in range(desc.n_layers):
        w = torch.empty(ds[i + 1], ds[i])
        torch.nn.init.orthogonal_(w, gain=gains[i], generator=g)
        out += [w.flatten(), 0.05 * torch.randn(ds[i + 1], generator=g)]
    return torch.cat(out).numpy()


# ---------------------------------------------------------------------------------------------
# (1) shipped nets
# ---------------------------------------------------------------------------------------------
def _cartpole_states_for_obs(p, obs):
    """f64 CartPole states whose get_state() (CartPole.py:145-153) is exactly `obs` (f32)."""
    o = np.asarray(obs, np.float32).astype(np.float64)
    st = np.zeros((5, o.shape[0]))
    for q, m in enumerate((p.theta_max, p.dtheta_max, p.x_max, p.dx_max)):
        st[q] = (o[:, q] / p.static_gain) * m
    return st


@pytest.mark.parametrize("mode", ["f16x3", "fp32"])
def test_rollout_shipped_nets_vs_reference(golden, mode):
    g = golden("ppo2_cartpole_nets")
    kind = A.RLP_ENV_CARTPOLE
    p = A.cartpole_params("ppo2")
    ad = A.MLPDesc.make([4, 256, 256, 1], [1, 1, 1])
    cd = A.MLPDesc.make([4, 256, 256, 1], [1, 1, 0])
    x = g["x"]
    la, lb = g["loop_a_obs"].astype(np.float32), g["loop_b_obs"].astype(np.float32)
    obs = np.concatenate([x, la, lb])
    n = obs.shape[0]
    st = dev(_cartpole_states_for_obs(p, obs))
    need = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cfg = K.make_rollout_cfg(1, n, 5, 0, 0, [1e-30], [-8], [8], A.RLP_SUCCESS_DONE_AND_FLAG_NE, 3,
                             mlp_precision=_native.MLP_F16X3 if mode == "f16x3" else _native.MLP_FP32)
    apk = K.mfma_pack(ad, dev(g["actor_params"]))
    cpk = K.mfma_pack(cd, dev(g["critic_params"]))
    bufs = K.rollout_buffers(kind, 1, n)
    K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(bufs["obs"][0]), obs)      # the reference's inputs exactly
    act = host(bufs["action"][0])
    nx = x.shape[0]
    # actor(x) (mean = tanh(.) * gain + off, train.py:73-78) and critic(x)
    bound(act[:nx], g["actor_mean"], 1e-5, 2e-6, f"{mode} action vs reference actor(x)")
    # the derived per-row action bound (policy_bounds) admits the reference's own float32 error,
    # and the kernel's error against float64 stays inside it
    m64, a_atol = policy_bounds(ad, g["actor_params"], x, None, [-8], [8], None)
    assert (np.abs(g["actor_mean"].reshape(m64.shape) - m64) <= a_atol).all()
    assert (np.abs(act[:nx].reshape(m64.shape) - m64) <= a_atol + 1e-5 * np.abs(m64)).all()
    # V(s) = fc3(h2): a 256-term sum whose terms reach |V| x 100 on some rows (cancellation), so
    # any two f32 evaluations (the reference's CPU GEMM, ours) differ by ~sqrt(256) f32 roundings
    # of the TERMS' scale: the bound adds 1e-6 x sum_j |w3_j h2_j| (float64 h2) to rtol 1e-5 /
    # atol 2e-6; the reference's own error against float64 is inside the same bound.
    cp = torch.as_tensor(g["critic_params"]).double()
    W1, b1 = cp[:1024].view(256, 4), cp[1024:1280]
    W2, b2 = cp[1280:1280 + 65536].view(256, 256), cp[66816:67072]
    W3 = cp[67072:67328]
    h2 = torch.tanh(torch.tanh(torch.as_tensor(x).double() @ W1.T + b1) @ W2.T + b2)
    scale = (h2 * W3).abs().sum(1).numpy() + abs(float(cp[67328]))
    v, vref = host(bufs["value"][0])[:nx].astype(np.float64), g["critic_v"][:, 0].astype(np.float64)
    lim = 1e-5 * np.abs(vref) + 2e-6 + 1e-6 * scale
    assert (np.abs(v - vref) <= lim).all(), f"{mode} V(s) vs reference critic(x): max excess " \
        f"{np.max(np.abs(v - vref) - lim):.3e}"
    v64 = (h2 @ W3 + cp[67328]).numpy()
    assert (np.abs(vref - v64) <= lim).all()     # the bound admits the reference's own error
    # the closed-loop transcripts: the reference's evaluate() on its own trajectory
    bound(act[nx:nx + len(la)], g["loop_a_action"], 1e-5, 2e-6, f"{mode} action on loop a")
    bound(act[nx + len(la):], g["loop_b_action"], 1e-5, 2e-6, f"{mode} action on loop b")


# ---------------------------------------------------------------------------------------------
# (2)/(3) teacher-forced replay
# ---------------------------------------------------------------------------------------------
def _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=1):
    st = K.new_state(kind, n)
    need = torch.ones(n, dtype=torch.uint8, device="cuda")
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    out = []
    for s in range(segments):
        cfg.step0 = s * T
        bufs = K.rollout_buffers(kind, T, n)
        K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
        out.append({k: host(v) for k, v in bufs.items()})
    torch.cuda.synchronize()
    return out, host(st), host(need)


def _oracle_forced(kind, p, n, T, cfg, gbufs, ad=None, ap=None, cd=None, cp=None):
    D, S, Ad = A.ENV_DIMS[kind]
    st = np.zeros((D, n))
    need = np.ones(n, np.uint8)
    out = []
    for s, gb in enumerate(gbufs):
        cfg.step0 = s * T
        ob = oracle.rollout(kind, p, st, need, ad, ap, cd, cp, cfg, forced_action=gb["action"])
        out.append(ob)
    return out, st, need


def _check_physics(kind, g, o, gst, ost, gneed, oneed, what):
    D, S, Ad = A.ENV_DIMS[kind]
    for gb, ob in zip(g, o):
        for key in ("done", "success", "flag"):
            np.testing.assert_array_equal(gb[key], ob[key], err_msg=f"{what}: {key}")
        for key in ("obs", "obs_next"):
            u = f32_ulps(gb[key], ob[key])
            assert u.max() <= 2, f"{what}: {key} differs by {u.max()} f32 ulps"
        bound(gb["reward"], ob["reward"], 2e-6, 1e-6, f"{what}: reward")
    np.testing.assert_array_equal(gneed, oneed, err_msg=f"{what}: need_reset")
    scale = np.abs(ost).max(axis=1, keepdims=True) + 1.0
    err = np.abs(gst - ost) / scale
    assert err.max() <= 1e-9, f"{what}: f64 state differs by {err.max():.3e} (relative to the row scale)"
    return float(err.max())


def test_forced_physics_replay_bench_size_cartpole():
    """BASELINE config 2 shard: 65 536 CartPole envs x T = 128, the bench's nets and std."""
    kind = A.RLP_ENV_CARTPOLE
    p = A.cartpole_params("ppo2")
    n, T = 65536, 128
    ad = A.MLPDesc.make([4, 256, 256, 1], [1, 1, 1])
    cd = A.MLPDesc.make([4, 256, 256, 1], [1, 1, 0])
    ap, cp = orthogonal(ad, [1, 1, 0.01], 1), orthogonal(cd, [1, 1, 1], 2)
    cfg = K.make_rollout_cfg(T, n, 3407, 0, 0, [8 / 3], [-8], [8], A.RLP_SUCCESS_DONE_AND_FLAG_NE, 3)
    g, gst, gneed = _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=2)
    assert g[0]["done"].any() and g[1]["done"].any()
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g)
    _check_physics(kind, g, o, gst, ost, gneed, oneed, "cartpole 65536x128")
    # the policy / critic of the first 2048 envs against the oracle's double-accumulated nets
    m = 2048
    sub = [{k: v[:, :m] for k, v in b.items()} for b in g]
    cfg.n = m
    o2, _, _ = _oracle_forced(kind, p, m, T, cfg, sub, ad, ap, cd, cp)
    for gb, ob in zip(sub, o2):
        a_tol, lp_tol = policy_bounds(ad, ap, gb["obs"], ob["action"], [-8], [8], [8 / 3])
        bound_rows(gb["action"], ob["action"], 1e-5, a_tol, "action")
        bound_rows(gb["logp"], ob["logp"], 1e-5, lp_tol, "log-prob")
        bound(gb["value"], ob["value"], 1e-5, 2e-6, "V(s)")
        nd = gb["done"] == 0
        bound(gb["value_next"][nd], ob["value_next"][nd], 1e-5, 2e-6, "V(s')")


def test_forced_physics_replay_bench_size_uav():
    """UavRobust bench shard: 32 768 envs x T = 64 (6-DoF + FNTSMC, 22-double state)."""
    kind = A.RLP_ENV_UAV_HOVER_OUTER_LOOP
    p = A.uav_hover_params()
    n, T = 32768, 64
    ad = A.MLPDesc.make([6, 256, 256, 3], [1, 1, 1])
    cd = A.MLPDesc.make([6, 256, 256, 1], [1, 1, 0])
    ap, cp = orthogonal(ad, [1, 1, 0.01], 3), orthogonal(cd, [1, 1, 1], 4)
    cfg = K.make_rollout_cfg(T, n, 3408, 0, 0, [8 / 3] * 3, [-8] * 3, [8] * 3,
                             A.RLP_SUCCESS_DONE_AND_FLAG_NE, 1)
    g, gst, gneed = _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=2)
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g)
    _check_physics(kind, g, o, gst, ost, gneed, oneed, "uav 32768x64")


def _nets(S, Ad, seed):
    ad = A.MLPDesc.make([S, 256, 256, Ad], [1, 1, 1])
    cd = A.MLPDesc.make([S, 256, 256, 1], [1, 1, 0])
    return ad, orthogonal(ad, [1, 1, 1.0], seed), cd, orthogonal(cd, [1, 1, 1], seed + 1)


@pytest.mark.parametrize("kind", sorted(A.FUSED_ROLLOUT_KINDS))
@pytest.mark.parametrize("sub", [1, 2, 4])
def test_rollout_teacher_forced_vs_oracle(kind, sub):
    """All kinds x envs-per-wave: physics replayed with the kernel's actions, the oracle's own
    policy and critic on the same observations; two chained segments, resets inside them."""
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind)
    ad, ap, cd, cp = _nets(S, Ad, 40 + kind)
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 6 for l, h in zip(lo, hi)]
    n, T = 2048 + 37, 48
    cfg = K.make_rollout_cfg(T, n, 3407, 0, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE,
                             A.timeout_flag(kind), sub=sub)
    g, gst, gneed = _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=2)
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g, ad, ap, cd, cp)
    _check_physics(kind, g, o, gst, ost, gneed, oneed, f"kind {kind} sub {sub}")
    for gb, ob in zip(g, o):
        a_tol, lp_tol = policy_bounds(ad, ap, gb["obs"], ob["action"], lo, hi, std)
        bound_rows(gb["action"], ob["action"], 1e-5, a_tol, "action")
        bound_rows(gb["logp"], ob["logp"], 1e-5, lp_tol, "log-prob")
        bound(gb["value"], ob["value"], 1e-5, 2e-6, "V(s)")
        nd = gb["done"] == 0
        bound(gb["value_next"][nd], ob["value_next"][nd], 1e-5, 2e-6, "V(s')")


@pytest.mark.parametrize("rule,flag", [(A.RLP_SUCCESS_DONE_AND_FLAG_NE, 1), (A.RLP_SUCCESS_FLAG_NE, 1),
                                       (A.RLP_SUCCESS_FLAG_EQ, 1)])
def test_rollout_success_rules_vs_oracle(rule, flag):
    """The three driver success rules (include/rlp.h rlp_success_rule): PPO2
    drivers' terminal && flag != timeout, DPPO2-CartPole/SOI's `0 if flag == 1 else 1` on every
    step (Distributed_PPO2.py:138), PPO-UAV's flag == F."""
    kind = A.RLP_ENV_CARTPOLE
    p = A.cartpole_params("dppo2")
    ad, ap, cd, cp = _nets(4, 1, 77)
    n, T = 4096, 128
    cfg = K.make_rollout_cfg(T, n, 11, 0, 0, [1.0], [-8], [8], rule, flag)
    g, gst, gneed = _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=2)
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g)
    _check_physics(kind, g, o, gst, ost, gneed, oneed, f"rule {rule}")
    f, d, su = (np.concatenate([gb[k] for gb in g]) for k in ("flag", "done", "success"))
    want = {A.RLP_SUCCESS_DONE_AND_FLAG_NE: (d == 1) & (f != flag),
            A.RLP_SUCCESS_FLAG_NE: f != flag, A.RLP_SUCCESS_FLAG_EQ: f == flag}[rule]
    np.testing.assert_array_equal(su, want.astype(np.uint8))
    assert (f == flag).any() and (f != flag).any()


VARIANTS = [(A.RLP_ENV_CARTPOLE_ANGLEONLY, "env"), (A.RLP_ENV_CARTPOLE, "dppo2"),
            (A.RLP_ENV_SOI, "dppo2"), (A.RLP_ENV_UGV_FORWARD, "ppo2"),
            (A.RLP_ENV_UGV_FORWARD, "dppo2"), (A.RLP_ENV_UGV_BIDIRECTIONAL, "ppo2")]


@pytest.mark.parametrize("kind,variant", VARIANTS, ids=[f"{k}-{v}" for k, v in VARIANTS])
def test_rollout_env_copies_teacher_forced(kind, variant):
    """The other env copies' params through the fused rollout (incl. the AngleOnly env file:
    10-11 sub-steps of dt/10, the angle-increment reward), teacher-forced against the oracle."""
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind, variant)
    ad, ap, cd, cp = _nets(S, Ad, 60 + kind)
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 6 for l, h in zip(lo, hi)]
    n, T = 4096, 64
    cfg = K.make_rollout_cfg(T, n, 3407, 0, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE,
                             A.timeout_flag(kind))
    g, gst, gneed = _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=2)
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g, ad, ap, cd, cp)
    _check_physics(kind, g, o, gst, ost, gneed, oneed, f"kind {kind} {variant}")
    for gb, ob in zip(g, o):
        a_tol, _ = policy_bounds(ad, ap, gb["obs"], ob["action"], lo, hi, std)
        bound_rows(gb["action"], ob["action"], 1e-5, a_tol, "action")
        bound(gb["value"], ob["value"], 1e-5, 2e-6, "V(s)")


def test_rollout_lidar_env_teacher_forced_config5_shard():
    """The lidar rollout at BASELINE config 5's shard size (131 072 / 8 = 16 384 envs), every CU
    busy (oa_policy2_kernel + oa_step_kernel<64> per step): two chained segments with resets inside,
    physics teacher-forced against the oracle for all envs (flags / done exact, state 1e-9,
    observations 2 ulps, rewards), the oracle's own policy and critic on the first 1 024 envs."""
    kind = A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind, "ppo2")
    ad, ap, cd, cp = _nets(S, Ad, 91)
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 6 for l, h in zip(lo, hi)]
    n, T = 16384, 24
    cfg = K.make_rollout_cfg(T, n, 3409, 0, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE,
                             A.timeout_flag(kind))
    g, gst, gneed = _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=2)
    assert g[0]["done"].sum() + g[1]["done"].sum() > 100   # resets inside the segments
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g)
    _check_physics(kind, g, o, gst, ost, gneed, oneed, "lidar env config-5 shard")
    m = 1024
    sub = [{k: v[:, :m] for k, v in b.items()} for b in g]
    cfg.n = m
    o2, _, _ = _oracle_forced(kind, p, m, T, cfg, sub, ad, ap, cd, cp)
    for gb, ob in zip(sub, o2):
        a_tol, lp_tol = policy_bounds(ad, ap, gb["obs"], ob["action"], lo, hi, std)
        bound_rows(gb["action"], ob["action"], 1e-5, a_tol, "action")
        bound_rows(gb["logp"], ob["logp"], 1e-5, lp_tol, "log-prob")
        bound(gb["value"], ob["value"], 1e-5, 2e-6, "V(s)")
        nd = gb["done"] == 0
        bound(gb["value_next"][nd], ob["value_next"][nd], 1e-5, 2e-6, "V(s')")


@pytest.mark.parametrize("variant,precision", [("env", "f16x3"), ("ppo2", "f16x3"), ("ppo2", "fp32")])
def test_rollout_lidar_env_teacher_forced(variant, precision):
    """UGVForwardObstacleAvoidance through rlp_rollout (round 6: two launches per step, the policy
    — oa_policy2_kernel with the f16x3 hidden layer, oa_policy_kernel on exact f32 — and
    oa_step_kernel),
    the PPO2 demo's 41 -> 256 -> 256 -> 2 / -> 1 nets
    (demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/train.py:48-50,95-97), two chained
    segments with resets inside: physics teacher-forced against the oracle (flags / done exact,
    state 1e-9, observations 2 ulps), the oracle's own policy and critic on the kernel's
    observations (action, log-prob, V(s), V(s'))."""
    kind = A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind, variant)
    ad, ap, cd, cp = _nets(S, Ad, 90)
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 6 for l, h in zip(lo, hi)]
    n, T = 1024 + 37, 40
    cfg = K.make_rollout_cfg(T, n, 3407, 0, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE,
                             A.timeout_flag(kind), mlp_precision=(_native.MLP_F16X3 if precision == "f16x3"
                                                                  else _native.MLP_FP32))
    g, gst, gneed = _gpu_segment(kind, p, n, T, ad, ap, cd, cp, cfg, segments=2)
    assert g[0]["done"].any() or g[1]["done"].any()
    o, ost, oneed = _oracle_forced(kind, p, n, T, cfg, g, ad, ap, cd, cp)
    _check_physics(kind, g, o, gst, ost, gneed, oneed, f"lidar env {variant} {precision}")
    for gb, ob in zip(g, o):
        a_tol, lp_tol = policy_bounds(ad, ap, gb["obs"], ob["action"], lo, hi, std)
        bound_rows(gb["action"], ob["action"], 1e-5, a_tol, "action")
        bound_rows(gb["logp"], ob["logp"], 1e-5, lp_tol, "log-prob")
        bound(gb["value"], ob["value"], 1e-5, 2e-6, "V(s)")
        nd = gb["done"] == 0
        bound(gb["value_next"][nd], ob["value_next"][nd], 1e-5, 2e-6, "V(s')")
