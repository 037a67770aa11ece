"""ctypes mirror of include/rlp.h (param structs, MLP descriptor, rollout config/buffers) and the
per-reference-copy parameter sets.

Every factory below reproduces the literals of one specific reference env copy (the copies diverge,
SURVEY.md §8a "Per-copy constants"); the citing path:line is relative to the reference root.
"""
import ctypes as C
import math

import numpy as np

RLP_OK = 0
RLP_EINVAL = -1000
RLP_EUNSUPPORTED = -1001

RLP_ENV_CARTPOLE = 1
RLP_ENV_CARTPOLE_ANGLEONLY = 2
RLP_ENV_SOI = 3
RLP_ENV_UGV_FORWARD = 4
RLP_ENV_UGV_BIDIRECTIONAL = 5
RLP_ENV_UAV_HOVER_OUTER_LOOP = 6
RLP_ENV_UGV_OBSTACLE_AVOIDANCE = 7

RLP_UGVOA_NOBS = 15     # obstacle slots per env (obsNum 10 or 15 by copy)
RLP_UGVOA_NLASER = 37   # int(2 * laserRange / laserStep) + 1
RLP_UGVOA_D = 8 + 3 * RLP_UGVOA_NOBS

# (D physics-state dim, S observation dim, A action dim)
ENV_DIMS = {
    RLP_ENV_CARTPOLE: (5, 4, 1),
    RLP_ENV_CARTPOLE_ANGLEONLY: (5, 2, 1),
    RLP_ENV_SOI: (7, 4, 2),
    RLP_ENV_UGV_FORWARD: (8, 4, 2),
    RLP_ENV_UGV_BIDIRECTIONAL: (8, 4, 2),
    RLP_ENV_UAV_HOVER_OUTER_LOOP: (22, 6, 3),
    RLP_ENV_UGV_OBSTACLE_AVOIDANCE: (RLP_UGVOA_D, 4 + RLP_UGVOA_NLASER, 2),
}
# kinds rlp_rollout runs: the fused one-kernel rollout ([S<=8 -> 256 -> 256 -> A<=4] nets), and the
# lidar env (S = 41: 4 + 37 beams) as a per-step kernel sequence inside the same call
FUSED_ROLLOUT_KINDS = tuple(k for k in ENV_DIMS if k != RLP_ENV_UGV_OBSTACLE_AVOIDANCE)
ROLLOUT_KINDS = tuple(ENV_DIMS)

RLP_ACT_NONE, RLP_ACT_TANH, RLP_ACT_RELU = 0, 1, 2
RLP_MLP_MAX_LAYERS = 8

RLP_SUCCESS_DONE_AND_FLAG_NE = 0
RLP_SUCCESS_FLAG_NE = 1
RLP_SUCCESS_FLAG_EQ = 2


def deg2rad(deg):
    """utils/functions.py:4-5 (same expression order: deg * pi / 180.)."""
    return deg * np.pi / 180.


class CartPoleParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "theta_max", "dtheta_max", "x_max", "dx_max", "static_gain", "M", "m", "g", "ell", "kf",
        "fm", "dt", "time_max", "reset_theta_lo", "reset_theta_hi", "reset_x_lo", "reset_x_hi",
        "Q_x", "Q_dx", "Q_theta", "Q_omega", "R")] + [("n_sub_div", C.c_int32), ("reserved", C.c_int32)]


class AngleOnlyParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "theta_max", "static_gain", "norm_dtheta", "M", "m", "g", "ell", "kf", "fm", "dt",
        "time_max", "reset_theta_lo", "reset_theta_hi", "Q_theta", "Q_omega", "R")] + [
        ("variant", C.c_int32), ("n_sub_div", C.c_int32)]


RLP_ANGLEONLY_PPO2_COPY, RLP_ANGLEONLY_ENV_FILE = 0, 1


class SOIParams(C.Structure):
    _fields_ = [("map_size", C.c_double * 2)] + [(n, C.c_double) for n in (
        "k", "mass", "dt", "time_max", "v_max", "f_max", "admissible_error", "obs_gain",
        "reset_margin", "Q_pos", "Q_vel", "Q_acc")] + [
        ("success_enabled", C.c_int32), ("reserved", C.c_int32)]


class UGVParams(C.Structure):
    _fields_ = [("map_size", C.c_double * 2)] + [(n, C.c_double) for n in (
        "dt", "time_max", "kf", "kt", "v_max", "omega_max", "a_linear_max", "a_angular_max",
        "static_gain", "reset_margin", "Q_pos", "Q_vel", "Q_phi", "Q_omega")] + [
        ("phi_gate_abs", C.c_int32), ("reserved", C.c_int32)]


_D3 = C.c_double * 3
_D32 = (C.c_double * 2) * 3


class UAVHoverParams(C.Structure):
    _fields_ = [("m", C.c_double), ("g", C.c_double), ("J", _D3), ("kr", C.c_double),
                ("kt", C.c_double), ("dt", C.c_double), ("time_max", C.c_double),
                ("pos0", _D3), ("vel0", _D3), ("angle0", _D3), ("pqr0", _D3),
                ("pos_zone", _D32), ("att_zone", _D32),
                ("att_k1", _D3), ("att_k2", _D3), ("att_alpha", _D3), ("att_beta", _D3),
                ("att_gamma", _D3), ("att_lmd", _D3), ("att_saturation", _D3),
                ("att_ctrl_dt", C.c_double), ("static_gain", C.c_double),
                ("e_pos_max", _D3), ("e_pos_min", _D3), ("vel_max", _D3), ("vel_min", _D3),
                ("dot_att_min", _D3), ("dot_att_max", _D3),
                ("u_min", C.c_double), ("u_max", C.c_double), ("target_offset", C.c_double),
                ("Qx", C.c_double), ("Qv", C.c_double), ("R", C.c_double)]


class MLPDesc(C.Structure):
    _fields_ = [("n_layers", C.c_int32), ("dims", C.c_int32 * (RLP_MLP_MAX_LAYERS + 1)),
                ("act", C.c_int32 * RLP_MLP_MAX_LAYERS)]

    @classmethod
    def make(cls, dims, acts):
        d = cls()
        d.n_layers = len(dims) - 1
        assert 1 <= d.n_layers <= RLP_MLP_MAX_LAYERS and len(acts) == d.n_layers
        for i, v in enumerate(dims):
            d.dims[i] = int(v)
        for i, a in enumerate(acts):
            d.act[i] = int(a)
        return d

    def layer_dims(self):
        return [self.dims[i] for i in range(self.n_layers + 1)]

    def param_count(self):
        ds = self.layer_dims()
        return sum(ds[i] * ds[i + 1] + ds[i + 1] for i in range(self.n_layers))


class RolloutCfg(C.Structure):
    _fields_ = [("T", C.c_int32), ("n", C.c_int32), ("seed", C.c_uint64), ("step0", C.c_uint64),
                ("env_id0", C.c_uint64), ("success_rule", C.c_int32), ("success_flag", C.c_int32),
                ("std", C.c_float * 4), ("a_min", C.c_float * 4), ("a_max", C.c_float * 4),
                # per-call kernel selection (include/rlp.h): 0 = library default, else value + 1
                ("mlp_precision", C.c_int32), ("physics", C.c_int32), ("sub", C.c_int32),
                ("net_layout", C.c_int32),
                # caller-owned device scratch (rlp_rollout_workspace_bytes)
                ("workspace", C.c_void_p), ("workspace_bytes", C.c_int64)]


class RolloutBufs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "obs", "obs_next", "action", "logp", "reward", "value", "value_next", "done", "success",
        "flag")]


RLP_LOSS_ACTOR, RLP_LOSS_CRITIC = 0, 1


class PPO2LossCfg(C.Structure):
    _fields_ = [("kind", C.c_int32), ("eps_clip", C.c_float), ("entropy_coef", C.c_float),
                ("std", C.c_float * 4), ("a_min", C.c_float * 4), ("a_max", C.c_float * 4)]


class AdamCfg(C.Structure):
    _fields_ = [("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
                ("max_norm", C.c_float), ("step", C.c_int32)]


class UGVOAParams(C.Structure):
    _fields_ = [("map_size", C.c_double * 2)] + [(n, C.c_double) for n in (
        "dt", "time_max", "kf", "kt", "v_max", "e_phi_max", "omega_max", "a_linear_max",
        "a_angular_max", "r_vehicle", "laser_dis", "laser_blind", "laser_range", "static_gain",
        "Q_pos", "Q_vel", "Q_phi", "Q_omega", "safety_dis_obs", "safety_dis_st", "r_min", "r_max",
        "st_margin")] + [(n, C.c_int32) for n in ("n_obs", "max_tries", "shaped", "reserved")]


class Replay(C.Structure):
    _fields_ = [("s", C.c_void_p), ("a", C.c_void_p), ("r", C.c_void_p), ("s_next", C.c_void_p),
                ("end", C.c_void_p), ("capacity", C.c_int64), ("S", C.c_int32), ("A", C.c_int32)]


RLP_DENSE_MAX_LAYERS = 4


class DenseNet(C.Structure):
    """rlp_dense_net: a Linear chain inside a flat fp32 parameter buffer (module.parameters()
    order; layer l's W [out][in] at offset[l], b right after it)."""
    _fields_ = [("n_layers", C.c_int32), ("dims", C.c_int32 * (RLP_DENSE_MAX_LAYERS + 1)),
                ("offset", C.c_int64 * RLP_DENSE_MAX_LAYERS), ("n_params", C.c_int64),
                ("params", C.c_void_p)]


class DDPGNets(C.Structure):
    _fields_ = [("actor", DenseNet), ("target_actor", DenseNet), ("critic", DenseNet),
                ("target_critic", DenseNet)] + [(n, C.c_void_p) for n in (
        "actor_grad", "actor_m", "actor_v", "critic_grad", "critic_m", "critic_v", "steps", "gain",
        "off")]


class DDPGCfg(C.Structure):
    _fields_ = [("batch", C.c_int32), ("gamma", C.c_float), ("actor_tau", C.c_float),
                ("critic_tau", C.c_float), ("actor_adam", AdamCfg), ("critic_adam", AdamCfg)]


class SACNets(C.Structure):
    _fields_ = [("actor", DenseNet), ("mean_offset", C.c_int64), ("log_std_offset", C.c_int64),
                ("action_dim", C.c_int32), ("q1", DenseNet), ("q2", DenseNet)] + [
        (n, C.c_void_p) for n in (
            "target_critic", "actor_grad", "actor_m", "actor_v", "critic_grad", "critic_m",
            "critic_v", "log_alpha", "alpha_grad", "alpha_m", "alpha_v", "steps", "counter", "gain",
            "off", "ls_lo", "ls_hi")]


class SACCfg(C.Structure):
    _fields_ = [("batch", C.c_int32), ("adaptive_alpha", C.c_int32), ("gamma", C.c_float),
                ("tau", C.c_float), ("target_entropy", C.c_float), ("alpha", C.c_float),
                ("seed", C.c_uint64), ("actor_adam", AdamCfg), ("critic_adam", AdamCfg),
                ("alpha_adam", AdamCfg)]


PARAM_TYPES = {
    RLP_ENV_CARTPOLE: CartPoleParams,
    RLP_ENV_CARTPOLE_ANGLEONLY: AngleOnlyParams,
    RLP_ENV_SOI: SOIParams,
    RLP_ENV_UGV_FORWARD: UGVParams,
    RLP_ENV_UGV_BIDIRECTIONAL: UGVParams,
    RLP_ENV_UAV_HOVER_OUTER_LOOP: UAVHoverParams,
    RLP_ENV_UGV_OBSTACLE_AVOIDANCE: UGVOAParams,
}


# ---------------------------------------------------------------------------------------------
# Parameter sets of the reference copies
# ---------------------------------------------------------------------------------------------
def cartpole_params(variant="ppo2"):
    """environment/CartPole/CartPole.py:27-46 (== demonstration/PPO2/PPO2-4-CartPole/CartPole.py).
    variant 'dppo2': demonstration/DPPO2/DPPO2-4-CartPole/CartPole.py:273-274 reset law."""
    p = CartPoleParams()
    p.theta_max = deg2rad(45)
    p.dtheta_max = deg2rad(90)
    p.x_max = 1.5
    p.dx_max = 3
    p.static_gain = 2.0
    p.M, p.m, p.g, p.ell, p.kf = 1.0, 0.1, 9.8, 0.2, 0.2
    p.fm = 8
    p.dt = 0.02
    p.time_max = 5
    if variant == "dppo2":
        p.reset_theta_lo, p.reset_theta_hi = -p.theta_max / 3, p.theta_max / 3
        p.reset_x_lo, p.reset_x_hi = -p.x_max / 2, p.x_max / 2
    else:
        p.reset_theta_lo, p.reset_theta_hi = -p.theta_max * 0.5, p.theta_max * 0.5
        p.reset_x_lo, p.reset_x_hi = -p.x_max * 0.5, p.x_max * 0.5
    p.Q_x, p.Q_dx, p.Q_theta, p.Q_omega, p.R = 5, 0.0, 1, 0.0, 0.01   # CartPole.py:192-196
    p.n_sub_div = 10                                                 # CartPole.py:242
    return p


def angleonly_params(variant="ppo2"):
    """variant 'ppo2' (== 'dppo2'): demonstration/PPO2/PPO2-4-CartPoleAngleOnly/
    cartpole_angleonly.py:27-41, :174-176; 'env': environment/CartPole/CartPoleAngleOnly.py:16-70
    (dt 0.01 in 10 sub-steps, fm 8, timeMax 6, the angle-increment reward; include/rlp.h)."""
    p = AngleOnlyParams()
    p.theta_max = deg2rad(45)
    p.static_gain = 2.0
    p.norm_dtheta = 4
    p.M, p.m, p.g, p.ell, p.kf = 1.0, 0.1, 9.8, 0.2, 0.2
    p.reset_theta_lo, p.reset_theta_hi = -p.theta_max * 0.5, p.theta_max * 0.5
    p.Q_theta, p.Q_omega, p.R = 10, 0.0, 0.00
    if variant == "env":
        p.fm, p.dt, p.time_max = 8, 0.01, 6
        p.variant, p.n_sub_div = RLP_ANGLEONLY_ENV_FILE, 10
    elif variant in ("ppo2", "dppo2"):
        p.fm, p.dt, p.time_max = 5, 0.02, 5
        p.variant, p.n_sub_div = RLP_ANGLEONLY_PPO2_COPY, 1
    else:
        raise ValueError(f"angleonly_params: variant {variant!r} (ppo2 | dppo2 | env)")
    return p


def soi_params(variant="env"):
    """environment/SecondOrderIntegration/SecondOrderIntegration.py:13-60, :262-264.
    variant 'dppo2'/'ddpg': demonstration/DPPO2/DPPO2-4-SecondOrderIntegration/
    SecondOrderIntegration.py:213 (obs * static_gain), :243-246 (no success), :260-261 (Q)."""
    p = SOIParams()
    p.map_size[0], p.map_size[1] = 5.0, 5.0
    p.k, p.mass, p.dt, p.time_max = 0.15, 1.0, 0.02, 5.0
    p.v_max, p.f_max, p.admissible_error = 3, 3, 0
    p.reset_margin = 0.1
    if variant in ("dppo2", "ddpg"):
        p.obs_gain = 2
        p.Q_pos, p.Q_vel, p.Q_acc = 1, 0.0, 0.0
        p.success_enabled = 0
    else:
        p.obs_gain = 1.0
        p.Q_pos, p.Q_vel, p.Q_acc = 1, 0.1, 0.05
        p.success_enabled = 1
    return p


def ugv_params(kind=RLP_ENV_UGV_FORWARD, variant="env"):
    """environment/UGV/UGVForward.py:34-63, :264-267; variants: PPO2 copy Q_vel = 0.1
    (demonstration/PPO2/PPO2-4-UGVForward/UGVForward.py:265); DPPO2 copy time_max = 5
    (demonstration/DPPO2/DPPO2-4-UGVForward/UGVForward.py:45); PPO2 UGVBidirectional copy gates
    u_phi on |e| (demonstration/PPO2/PPO2-4-UGVBidirectional/UGVBidirectional.py:271)."""
    p = UGVParams()
    p.map_size[0], p.map_size[1] = 5.0, 5.0
    p.dt, p.time_max = 0.02, 10.0
    p.kf, p.kt = 0.1, 0.1
    p.v_max, p.omega_max = 3, 2 * np.pi
    p.a_linear_max, p.a_angular_max = 3, 2 * np.pi
    p.static_gain = 1.
    p.reset_margin = 0.5
    p.Q_pos, p.Q_vel, p.Q_phi, p.Q_omega = 2., 0.0, 2., 1.0
    p.phi_gate_abs = 0
    if kind == RLP_ENV_UGV_FORWARD and variant in ("ppo2", "dppo2"):
        p.Q_vel = 0.1
        if variant == "dppo2":
            p.time_max = 5.0
    if kind == RLP_ENV_UGV_BIDIRECTIONAL and variant == "ppo2":
        p.phi_gate_abs = 1
    return p


def uav_hover_params():
    """environment/UavRobust/uav.py:12-31 with demonstration/PPO/PPO-4-UavHoverOuterLoop/
    train.py:24-56 (quadrotor + FNTSMC attitude gains) and UavHoverOuterLoop.py:33-43, :97."""
    p = UAVHoverParams()
    p.m, p.g = 0.8, 9.8
    p.J[:] = [4.212e-3, 4.212e-3, 8.255e-3]
    p.kr, p.kt = 1e-3, 1e-3
    p.dt, p.time_max = 0.01, 10
    for a in (p.pos0, p.vel0, p.angle0, p.pqr0):
        a[:] = [0, 0, 0]
    for i, (lo, hi) in enumerate([[-5, 5], [-5, 5], [0, 5]]):
        p.pos_zone[i][0], p.pos_zone[i][1] = lo, hi
    for i, (lo, hi) in enumerate([[deg2rad(-45), deg2rad(45)], [deg2rad(-45), deg2rad(45)],
                                  [deg2rad(-120), deg2rad(120)]]):
        p.att_zone[i][0], p.att_zone[i][1] = lo, hi
    p.att_k1[:] = [25, 25, 40]
    p.att_k2[:] = [0.1, 0.1, 0.2]
    p.att_alpha[:] = [2.5, 2.5, 2.5]
    p.att_beta[:] = [0.99, 0.99, 0.99]
    p.att_gamma[:] = [1.5, 1.5, 1.2]
    p.att_lmd[:] = [2.0, 2.0, 2.0]
    p.att_saturation[:] = [0.3, 0.3, 0.3]
    p.att_ctrl_dt = 0.01
    p.static_gain = 1.0
    p.e_pos_max[:] = [5., 5., 5.]
    p.e_pos_min[:] = [-5., -5., -0.]
    p.vel_max[:] = [3., 3., 3.]
    p.vel_min[:] = [-3., -3., -3.]
    p.dot_att_min[:] = [-deg2rad(60), -deg2rad(60), -deg2rad(1)]
    p.dot_att_max[:] = [deg2rad(60), deg2rad(60), deg2rad(1)]
    p.u_min, p.u_max = -8, 8
    p.target_offset = 1.0
    p.Qx, p.Qv, p.R = 1, 0.1, 0.02
    return p


def ugv_oa_params(variant="env"):
    """environment/UGVForwardObstacleAvoidance/UGVForwardObstacleAvoidance.py:12-104 (constants),
    :452-469 (Q literals), :527-537 (generate_circle_obs_training arguments: safety distances
    4 * r_vehicle, r in [0.2, 0.5], obsNum 10), map.py:66-73 (start/target margin 0.3).
    variant 'ppo2': demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/UGVForwardObstacleAvoidance.py
    (dt 0.05 :40, success ignores omega :421-427, shaped reward :449-473, rk44 pre-step vel gate
    :488-500); 'dppo2': the DPPO2 copy, identical to 'ppo2' but obsNum=15 (:543)."""
    p = UGVOAParams()
    p.map_size[0], p.map_size[1] = 5.0, 5.0
    p.dt, p.time_max = 0.1, 15.0
    p.kf, p.kt = 0.1, 0.1
    p.v_max, p.e_phi_max, p.omega_max = 3, np.pi, 2 * np.pi
    p.a_linear_max, p.a_angular_max = 3, 2 * np.pi
    p.r_vehicle = 0.15
    p.laser_dis, p.laser_blind, p.laser_range = 2.0, 0.0, deg2rad(90)
    p.static_gain = 1.
    p.Q_pos, p.Q_vel, p.Q_phi, p.Q_omega = 2., 0.0, 2., 1.0
    p.safety_dis_obs = p.safety_dis_st = 4 * p.r_vehicle
    p.r_min, p.r_max = 0.2, 0.5
    p.st_margin = 0.3
    p.n_obs, p.max_tries, p.shaped = 10, 4096, 0
    if variant in ("ppo2", "dppo2"):
        p.dt, p.shaped = 0.05, 1
        if variant == "dppo2":
            p.n_obs = 15
    elif variant != "env":
        raise ValueError(variant)
    return p


def default_params(kind, variant=None):
    if kind == RLP_ENV_CARTPOLE:
        return cartpole_params(variant or "ppo2")
    if kind == RLP_ENV_CARTPOLE_ANGLEONLY:   # the same default as CartPoleAngleOnly(variant=)
        return angleonly_params(variant or "env")
    if kind == RLP_ENV_SOI:
        return soi_params(variant or "env")
    if kind in (RLP_ENV_UGV_FORWARD, RLP_ENV_UGV_BIDIRECTIONAL):
        return ugv_params(kind, variant or "env")
    if kind == RLP_ENV_UAV_HOVER_OUTER_LOOP:
        return uav_hover_params()
    if kind == RLP_ENV_UGV_OBSTACLE_AVOIDANCE:
        return ugv_oa_params(variant or "env")
    raise ValueError(f"unknown env kind {kind}")


def action_bounds(kind, params):
    """Action ranges (rl_base.action_range) per kind."""
    if kind == RLP_ENV_CARTPOLE:
        return [-params.fm], [params.fm]
    if kind == RLP_ENV_CARTPOLE_ANGLEONLY:
        return [-params.fm], [params.fm]
    if kind == RLP_ENV_SOI:
        return [-params.f_max] * 2, [params.f_max] * 2
    if kind in (RLP_ENV_UGV_FORWARD, RLP_ENV_UGV_BIDIRECTIONAL, RLP_ENV_UGV_OBSTACLE_AVOIDANCE):
        return ([-params.a_linear_max, -params.a_angular_max],
                [params.a_linear_max, params.a_angular_max])
    if kind == RLP_ENV_UAV_HOVER_OUTER_LOOP:
        return [params.u_min] * 3, [params.u_max] * 3
    raise ValueError(kind)


def timeout_flag(kind):
    """terminal_flag value meaning 'time out' per kind (the PPO2 drivers' success rule excludes it)."""
    return {RLP_ENV_CARTPOLE: 3, RLP_ENV_CARTPOLE_ANGLEONLY: 3, RLP_ENV_SOI: 2,
            RLP_ENV_UGV_FORWARD: 2, RLP_ENV_UGV_BIDIRECTIONAL: 2,
            RLP_ENV_UAV_HOVER_OUTER_LOOP: 1, RLP_ENV_UGV_OBSTACLE_AVOIDANCE: 2}[kind]


def check_struct_sizes():
    """Sizes as seen by the C compiler (tests compare with librlp's rlp_struct_size())."""
    return {"cartpole": C.sizeof(CartPoleParams), "angleonly": C.sizeof(AngleOnlyParams),
            "soi": C.sizeof(SOIParams), "ugv": C.sizeof(UGVParams),
            "uav": C.sizeof(UAVHoverParams), "mlp_desc": C.sizeof(MLPDesc),
            "rollout_cfg": C.sizeof(RolloutCfg), "rollout_bufs": C.sizeof(RolloutBufs),
            "ppo2_loss_cfg": C.sizeof(PPO2LossCfg), "adam_cfg": C.sizeof(AdamCfg),
            "replay": C.sizeof(Replay), "ugv_oa": C.sizeof(UGVOAParams),
            "dense_net": C.sizeof(DenseNet), "ddpg_nets": C.sizeof(DDPGNets),
            "ddpg_cfg": C.sizeof(DDPGCfg), "sac_nets": C.sizeof(SACNets),
            "sac_cfg": C.sizeof(SACCfg)}


_ = math  # keep import for callers doing deg arithmetic
