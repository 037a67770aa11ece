"""Tensor-level wrappers of librlp's C-ABI (one function per entry point of include/rlp.h).

All tensors live on the ROCm device. Nothing here falls back to the CPU.
"""
import ctypes as C

import torch

from . import _abi
from ._native import RLPError, check, lib, ptr, stream_ptr


def dims(kind):
    return _abi.ENV_DIMS[kind]


def _dev(device):
    return torch.device(device) if device is not None else torch.device("cuda")


def new_state(kind, n, device=None):
    D, _, _ = dims(kind)
    return torch.zeros((D, n), dtype=torch.float64, device=_dev(device))


def env_reset(kind, params, state, mask=None, init_state=None, seed=0, counter=0, env_id0=0):
    n = state.shape[1]
    check(lib().rlp_env_reset(kind, C.byref(params), ptr(state), n, ptr(mask), ptr(init_state),
                              seed, counter, env_id0, stream_ptr()), "rlp_env_reset")


def env_observe(kind, params, state, out=None):
    _, S, _ = dims(kind)
    n = state.shape[1]
    out = out if out is not None else torch.empty((n, S), dtype=torch.float32, device=state.device)
    check(lib().rlp_env_observe(kind, C.byref(params), ptr(state), n, ptr(out), stream_ptr()),
          "rlp_env_observe")
    return out


def env_step(kind, params, state, action, want_obs_cur=True):
    _, S, A = dims(kind)
    n = state.shape[1]
    dev = state.device
    action = action.to(device=dev, dtype=torch.float32).reshape(n, A).contiguous()
    oc = torch.empty((n, S), dtype=torch.float32, device=dev) if want_obs_cur else None
    on = torch.empty((n, S), dtype=torch.float32, device=dev)
    r = torch.empty(n, dtype=torch.float64, device=dev)
    f = torch.empty(n, dtype=torch.int32, device=dev)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    check(lib().rlp_env_step(kind, C.byref(params), ptr(state), n, ptr(action), ptr(oc), ptr(on),
                             ptr(r), ptr(f), ptr(d), stream_ptr()), "rlp_env_step")
    return oc, on, r, f, d


def mlp_forward(desc, params, x, mask=None, out=None, workspace=None):
    """rlp_mlp_forward; the per-layer GEMM path's scratch (rlp_mlp_forward_workspace_bytes) is
    `workspace` (a uint8 device tensor) when it is large enough, else allocated here."""
    n = x.shape[0]
    outn = desc.dims[desc.n_layers]
    out = out if out is not None else torch.empty((n, outn), dtype=torch.float32, device=x.device)
    x_ = x.contiguous()
    need = int(lib().rlp_mlp_forward_workspace_bytes(C.byref(desc), n)) if mask is None else 0
    if need < 0:
        check(need, "rlp_mlp_forward_workspace_bytes")
    if need > 0 and (workspace is None or workspace.numel() < need):
        workspace = torch.empty(need, dtype=torch.uint8, device=x.device)
    check(lib().rlp_mlp_forward(C.byref(desc), ptr(params), ptr(x_), ptr(out), n, ptr(mask),
                                ptr(workspace) if need > 0 else None, need, stream_ptr()),
          "rlp_mlp_forward")
    return out


def mfma_pack(desc, params, out=None):
    cnt = lib().rlp_mfma_packed_count(C.byref(desc))
    if cnt < 0:
        check(int(cnt), "rlp_mfma_packed_count")
    out = out if out is not None else torch.empty(cnt, dtype=torch.float32, device=params.device)
    check(lib().rlp_mfma_pack(C.byref(desc), ptr(params), ptr(out), stream_ptr()), "rlp_mfma_pack")
    return out


def _call_precision(precision):
    """include/rlp.h per-call mlp_precision: 'fp32' (exact f32 MFMA, the default here), 'f16x3'
    (the rollout's split hidden layer) or 'default' (the library-wide rlp_set_mlp_precision)."""
    return {"default": 0, "fp32": 1, "f16x3": 2}[precision]


def mfma_forward(desc, packed, x, out=None, precision="fp32"):
    """Forward of an MFMA-packed [S->H->H->A] net (last-layer activation applied); the hidden
    layer's arithmetic is chosen per call (`precision`, see _call_precision)."""
    rows = x.shape[0]
    outn = desc.dims[desc.n_layers]
    out = out if out is not None else torch.empty((rows, outn), dtype=torch.float32, device=x.device)
    x_ = x.contiguous()
    check(lib().rlp_mfma_forward(C.byref(desc), ptr(packed), ptr(x_), ptr(out), rows,
                                 _call_precision(precision), stream_ptr()), "rlp_mfma_forward")
    return out


def value_fixup(critic_desc, critic_packed, obs_next, done, success, value_next, precision="fp32"):
    """value_next[i] = critic(obs_next[i]) where done & !success (flattened [T*n] rows)."""
    rows = done.numel()
    check(lib().rlp_value_fixup(C.byref(critic_desc), ptr(critic_packed), ptr(obs_next),
                                ptr(done), ptr(success), ptr(value_next), rows,
                                _call_precision(precision), stream_ptr()),
          "rlp_value_fixup")
    return value_next


def _host_f32(v, A):
    arr = (C.c_float * A)()
    vals = list(v) if hasattr(v, "__len__") else [v] * A
    for i in range(A):
        arr[i] = float(vals[i])
    return arr


def policy_sample(mean, std, a_min, a_max, noise=None, seed=0, counter=0, env_id0=0):
    n, A = mean.shape
    a = torch.empty_like(mean)
    lp = torch.empty_like(mean)
    mean_ = mean.contiguous()
    check(lib().rlp_policy_sample(ptr(mean_), n, A, _host_f32(std, A),
                                  _host_f32(a_min, A), _host_f32(a_max, A), ptr(noise), seed,
                                  counter, env_id0, ptr(a), ptr(lp), stream_ptr()),
          "rlp_policy_sample")
    return a, lp


def sac_sample(head, ls_lo, ls_hi, gain, off, a_min=None, a_max=None, deterministic=False,
               noise=None, seed=0, counter=0, env_id0=0, with_logprob=True):
    """rlp_sac_sample: the SAC squashed-Gaussian head on head = [n][2A] (mean | log_std)."""
    n, A2 = head.shape
    A = A2 // 2
    a = torch.empty((n, A), dtype=torch.float32, device=head.device)
    lp = torch.empty(n, dtype=torch.float32, device=head.device) if with_logprob else None
    clamp = a_min is not None
    head_ = head.contiguous()
    check(lib().rlp_sac_sample(ptr(head_), n, A, _host_f32(ls_lo, A),
                               _host_f32(ls_hi, A), _host_f32(gain, A), _host_f32(off, A),
                               _host_f32(a_min, A) if clamp else None,
                               _host_f32(a_max, A) if clamp else None, int(bool(deterministic)),
                               ptr(noise), seed, counter, env_id0, ptr(a), ptr(lp), stream_ptr()),
          "rlp_sac_sample")
    return a, lp


def rollout_buffers(kind, T, n, device=None):
    _, S, A = dims(kind)
    dev = _dev(device)
    f32 = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    return dict(obs=torch.empty((T, n, S), **f32), obs_next=torch.empty((T, n, S), **f32),
                action=torch.empty((T, n, A), **f32), logp=torch.empty((T, n, A), **f32),
                reward=torch.empty((T, n), **f32), value=torch.empty((T, n), **f32),
                value_next=torch.zeros((T, n), **f32), done=torch.empty((T, n), **u8),
                success=torch.empty((T, n), **u8), flag=torch.empty((T, n), dtype=torch.int8,
                                                                    device=dev))


def rollout_workspace_bytes(kind, actor_desc, critic_desc, cfg):
    need = int(lib().rlp_rollout_workspace_bytes(kind, C.byref(actor_desc), C.byref(critic_desc),
                                                 C.byref(cfg)))
    if need < 0:
        check(need, "rlp_rollout_workspace_bytes")
    return need


def rollout(kind, params, state, need_reset, actor_desc, actor_packed, critic_desc, critic_packed,
            cfg, bufs, workspace=None):
    """rlp_rollout. The multi-launch paths' scratch (rlp_rollout_workspace_bytes: the plain-layout
    nets and the lidar env) is `workspace` (uint8 device tensor) when large enough, else allocated
    here; the workspace used is returned so a driver loop can keep it (allocated once)."""
    need = rollout_workspace_bytes(kind, actor_desc, critic_desc, cfg)
    if need > 0 and (workspace is None or workspace.numel() < need):
        workspace = torch.empty(need, dtype=torch.uint8, device=state.device)
    cfg.workspace = workspace.data_ptr() if need > 0 else None
    cfg.workspace_bytes = workspace.numel() if need > 0 else 0
    cb = _abi.RolloutBufs(**{k: v.data_ptr() for k, v in bufs.items()})
    check(lib().rlp_rollout(kind, C.byref(params), ptr(state), ptr(need_reset), C.byref(actor_desc),
                            ptr(actor_packed), C.byref(critic_desc), ptr(critic_packed),
                            C.byref(cfg), C.byref(cb), stream_ptr()), "rlp_rollout")
    return workspace


def make_rollout_cfg(T, n, seed, step0, env_id0, std, a_min, a_max, success_rule, success_flag,
                     mlp_precision=None, physics=None, sub=None, plain=False):
    """rlp_rollout_cfg. mlp_precision (RLP_MLP_FP32 | RLP_MLP_F16X3), physics (-1 auto, 0
    register-resident, 1 shared (two 4-wave blocks per CU), 3 one 8-wave block per CU, 5 one
    4-wave block per CU; include/rlp.h) and sub (1 | 2 | 4)
    select the kernel for this call only; None keeps the library-wide defaults (rlp_set_*).
    plain: the nets are passed in the plain parameter layout (any Linear stack; net_layout 1)."""
    cfg = _abi.RolloutCfg()
    cfg.net_layout = 1 if plain else 0
    cfg.mlp_precision = 0 if mlp_precision is None else int(mlp_precision) + 1
    if physics is not None and int(physics) not in (-1, 0, 1, 3, 5):
        raise ValueError(f"make_rollout_cfg: physics={physics} (-1 auto, 0, 1, 3, 5)")
    cfg.physics = 0 if physics is None else 8 if int(physics) == -1 else int(physics) + 1
    cfg.sub = 0 if sub is None else int(sub)
    cfg.T, cfg.n, cfg.seed, cfg.step0, cfg.env_id0 = T, n, seed, step0, env_id0
    cfg.success_rule, cfg.success_flag = success_rule, success_flag
    A = len(a_min)
    stdv = list(std) if hasattr(std, "__len__") else [std] * A
    for i in range(4):
        cfg.std[i] = float(stdv[i]) if i < A else 1.0
        cfg.a_min[i] = float(a_min[i]) if i < A else 0.0
        cfg.a_max[i] = float(a_max[i]) if i < A else 0.0
    return cfg


def reward_norm_workspace(T, n, device=None):
    cnt = lib().rlp_reward_norm_workspace(int(T), int(n))
    check(cnt if cnt < 0 else 0, "rlp_reward_norm_workspace")
    return torch.empty(int(cnt), dtype=torch.float64, device=_dev(device))


def reward_norm(reward, rms, work=None, out=None):
    """reward [T][n] f32 -> normalised (in `out`, may alias); rms: f64[4] device running stats."""
    T, n = reward.shape
    work = work if work is not None else reward_norm_workspace(T, n, reward.device)
    out = out if out is not None else torch.empty_like(reward)
    check(lib().rlp_reward_norm(ptr(reward), T, n, ptr(rms), ptr(work), ptr(out), stream_ptr()),
          "rlp_reward_norm")
    return out


def reward_norm_statistics(reward, rms, work):
    """rlp_reward_norm_statistics: the running statistics over reward [T][n], step t's
    (mean_t, std_t) kept in `work` for gae_normalized (no normalised-reward array)."""
    T, n = reward.shape
    check(lib().rlp_reward_norm_statistics(ptr(reward), T, n, ptr(rms), ptr(work), stream_ptr()),
          "rlp_reward_norm_statistics")
    return work


def reward_norm_apply(reward, work, out=None):
    """the normalised rewards from the statistics a preceding reward_norm_statistics left in work"""
    T, n = reward.shape
    out = out if out is not None else torch.empty_like(reward)
    check(lib().rlp_reward_norm_apply(ptr(reward), T, n, ptr(work), ptr(out), stream_ptr()),
          "rlp_reward_norm_apply")
    return out


def reward_norm_stats(reward, work):
    """Stage 1 of a cross-rank reward normaliser: this rank's chunk statistics into work[:parts]
    (include/rlp.h rlp_reward_norm_stats); returns that view for the all-gather."""
    T, n = reward.shape
    check(lib().rlp_reward_norm_stats(ptr(reward), T, n, ptr(work), stream_ptr()),
          "rlp_reward_norm_stats")
    return work[:int(lib().rlp_reward_norm_parts(T, n))]


def reward_norm_finish(reward, rms, work, parts, world, out=None):
    """Stage 2: merge every rank's chunk statistics (`parts`, rank-major) and normalise."""
    T, n = reward.shape
    out = out if out is not None else torch.empty_like(reward)
    check(lib().rlp_reward_norm_finish(ptr(reward), T, n, int(world), ptr(parts), ptr(rms),
                                       ptr(work), ptr(out), stream_ptr()), "rlp_reward_norm_finish")
    return out


def adv_stats_parts(n):
    return int(lib().rlp_adv_stats_parts(int(n)))


def adv_stats_buffer(n, world=1, device=None):
    """f64 buffer for rlp_gae's per-block (count, mean, M2) partials of `world` ranks + (mean, std)."""
    return torch.zeros(3 * adv_stats_parts(n) * world + 2, dtype=torch.float64, device=_dev(device))


def gae(reward, value, value_next, done, success, gamma, lmd, adv=None, v_target=None, stats=None):
    """stats (nullable): adv_stats_buffer(n), receives the per-block advantage partials."""
    T, n = reward.shape
    adv = adv if adv is not None else torch.empty_like(reward)
    v_target = v_target if v_target is not None else torch.empty_like(reward)
    check(lib().rlp_gae(ptr(reward), ptr(value), ptr(value_next), ptr(done), ptr(success),
                        float(gamma), float(lmd), T, n, ptr(adv), ptr(v_target), ptr(stats),
                        stream_ptr()), "rlp_gae")
    return adv, v_target


def gae_normalized(reward_raw, reward_work, value, value_next, done, success, gamma, lmd, adv=None,
                   v_target=None, stats=None):
    """rlp_gae_normalized: GAE over the raw rewards normalised on load with the statistics a
    preceding reward_norm_statistics left in reward_work."""
    T, n = reward_raw.shape
    adv = adv if adv is not None else torch.empty_like(reward_raw)
    v_target = v_target if v_target is not None else torch.empty_like(reward_raw)
    check(lib().rlp_gae_normalized(ptr(reward_raw), ptr(reward_work), ptr(value), ptr(value_next),
                                   ptr(done), ptr(success), float(gamma), float(lmd), T, n,
                                   ptr(adv), ptr(v_target), ptr(stats), stream_ptr()),
          "rlp_gae_normalized")
    return adv, v_target


def adv_normalize(adv, stats, parts=None):
    """Normalise adv with the first `parts` partials of stats (default: one rank's, from the
    buffer's size); (mean, std) land at stats[3 * parts:3 * parts + 2]."""
    parts = (stats.numel() - 2) // 3 if parts is None else int(parts)
    check(lib().rlp_adv_normalize(ptr(adv), adv.numel(), ptr(stats), parts, stream_ptr()),
          "rlp_adv_normalize")
    return adv


# ---------------------------------------------------------------------------------------------
# PPO2 update (include/rlp.h: rlp_ppo2_grad, rlp_grad_sqnorm, rlp_adam_step)
# ---------------------------------------------------------------------------------------------
def ppo2_loss_cfg(kind, eps_clip=0.2, entropy_coef=0.01, std=(), a_min=(), a_max=()):
    c = _abi.PPO2LossCfg()
    c.kind, c.eps_clip, c.entropy_coef = int(kind), float(eps_clip), float(entropy_coef)
    for i, (sd, lo, hi) in enumerate(zip(std, a_min, a_max)):
        c.std[i], c.a_min[i], c.a_max[i] = float(sd), float(lo), float(hi)
    return c


def ppo2_workspace(desc, rows, device=None):
    n = lib().rlp_ppo2_workspace_floats(C.byref(desc), int(rows))
    check(n if n < 0 else 0, "rlp_ppo2_workspace_floats")
    return torch.empty(int(n), dtype=torch.float32, device=_dev(device))


def ppo2_grad(desc, packed, cfg, s, a=None, a_logprob=None, adv=None, v_target=None, index=None,
              grad=None, loss_sum=None, workspace=None):
    """Gradient of one PPO2 optimiser step's loss (flat torch parameter order) over the rows of
    s (or s[index]); loss_sum (float64 [1], +=) receives the summed per-row loss."""
    rows = int(index.shape[0]) if index is not None else int(s.shape[0])
    dev = s.device
    grad = grad if grad is not None else torch.empty(desc.param_count(), dtype=torch.float32,
                                                     device=dev)
    need = int(lib().rlp_ppo2_workspace_floats(C.byref(desc), rows))
    if need < 0:   # not a net rlp_ppo2_grad takes: let the call report why
        need = 0
    if workspace is None:
        workspace = ppo2_workspace(desc, rows, dev)
    elif workspace.numel() < need:
        raise RLPError(f"rlp_ppo2_grad: workspace of {workspace.numel()} floats, need {need} "
                       f"(rlp_ppo2_workspace_floats)")
    # converted tensors are bound to locals so they outlive the (asynchronous) launch
    s_, a_, lp_, adv_, vt_, idx_ = (None if t is None else t.contiguous()
                                    for t in (s, a, a_logprob, adv, v_target, index))
    check(lib().rlp_ppo2_grad(C.byref(desc), ptr(packed), C.byref(cfg), ptr(s_), ptr(a_),
                              ptr(lp_), ptr(adv_), ptr(vt_), ptr(idx_), rows, ptr(grad),
                              ptr(loss_sum), ptr(workspace), stream_ptr()), "rlp_ppo2_grad")
    return grad


def ppo2_dense_workspace(desc, rows, device=None):
    n = lib().rlp_ppo2_dense_workspace_floats(C.byref(desc), int(rows))
    check(n if n < 0 else 0, "rlp_ppo2_dense_workspace_floats")
    return torch.empty(int(n), dtype=torch.float32, device=_dev(device))


def ppo2_dense_grad(desc, params, cfg, s, a=None, a_logprob=None, adv=None, v_target=None,
                    grad=None, loss_sum=None, workspace=None):
    """rlp_ppo2_dense_grad: ppo2_grad for any tanh Linear stack, on the plain parameter layout;
    rows are the rows of s (contiguous; gather a mini-batch first)."""
    rows = int(s.shape[0])
    dev = s.device
    grad = grad if grad is not None else torch.empty(desc.param_count(), dtype=torch.float32,
                                                     device=dev)
    if workspace is None:
        workspace = ppo2_dense_workspace(desc, rows, dev)
    else:
        need = int(lib().rlp_ppo2_dense_workspace_floats(C.byref(desc), rows))
        if workspace.numel() < need:
            raise RLPError(f"rlp_ppo2_dense_grad: workspace of {workspace.numel()} floats, need "
                           f"{need} (rlp_ppo2_dense_workspace_floats)")
    s_, a_, lp_, adv_, vt_ = (None if t is None else t.contiguous()
                              for t in (s, a, a_logprob, adv, v_target))
    check(lib().rlp_ppo2_dense_grad(C.byref(desc), ptr(params), C.byref(cfg), ptr(s_), ptr(a_),
                                    ptr(lp_), ptr(adv_), ptr(vt_), rows, ptr(grad), ptr(loss_sum),
                                    ptr(workspace), stream_ptr()), "rlp_ppo2_dense_grad")
    return grad


def grad_sqnorm(grad, out):
    check(lib().rlp_grad_sqnorm(ptr(grad), grad.numel(), ptr(out), stream_ptr()), "rlp_grad_sqnorm")
    return out


def grad_clip(grad, sqnorm, max_norm):
    """clip_grad_norm_ in place on a flat gradient whose squared norm is in sqnorm (f64 [1])."""
    check(lib().rlp_grad_clip(ptr(grad), grad.numel(), ptr(sqnorm), float(max_norm), stream_ptr()),
          "rlp_grad_clip")
    return grad


def adam_step(param, grad, exp_avg, exp_avg_sq, lr, step, beta1=0.9, beta2=0.999, eps=1e-8,
              clip_sqnorm=None, max_norm=0.5):
    c = _abi.AdamCfg()
    c.lr, c.beta1, c.beta2, c.eps, c.max_norm, c.step = lr, beta1, beta2, eps, max_norm, int(step)
    check(lib().rlp_adam_step(ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(),
                              C.byref(c), ptr(clip_sqnorm), stream_ptr()), "rlp_adam_step")


# ---------------------------------------------------------------------------------------------
# Replay buffer in HBM (include/rlp.h: rlp_replay_*)
# ---------------------------------------------------------------------------------------------
def replay_alloc(capacity, S, A, device=None):
    """Device columns of a replay buffer and the rlp_replay struct pointing at them."""
    dev = _dev(device)
    f32 = dict(dtype=torch.float32, device=dev)
    cols = {"s": torch.zeros((capacity, S), **f32), "a": torch.zeros((capacity, A), **f32),
            "r": torch.zeros(capacity, **f32), "s_next": torch.zeros((capacity, S), **f32),
            "end": torch.zeros(capacity, **f32)}
    rb = _abi.Replay()
    for k, t in cols.items():
        setattr(rb, k, t.data_ptr())
    rb.capacity, rb.S, rb.A = int(capacity), int(S), int(A)
    return cols, rb


def replay_store(rb, counter, s, a, reward, s_next, done):
    n = int(s.shape[0])
    # converted tensors are bound to locals so they outlive the (asynchronous) launch
    s_, a_ = s.to(dtype=torch.float32).contiguous(), a.to(dtype=torch.float32).contiguous()
    r_, s2_ = reward.to(dtype=torch.float64).contiguous(), s_next.to(dtype=torch.float32).contiguous()
    d_ = done.to(dtype=torch.uint8).contiguous()
    check(lib().rlp_replay_store(C.byref(rb), int(counter), ptr(s_), ptr(a_), ptr(r_), ptr(s2_),
                                 ptr(d_), n, stream_ptr()), "rlp_replay_store")
    return n


def replay_sample_uniform(max_mem, batch, seed, counter, out=None, device=None):
    out = out if out is not None else torch.empty(int(batch), dtype=torch.int64, device=_dev(device))
    check(lib().rlp_replay_sample_uniform(int(max_mem), int(batch), int(seed), int(counter),
                                          ptr(out), stream_ptr()), "rlp_replay_sample_uniform")
    return out


def replay_workspace(max_mem, device=None):
    nb = lib().rlp_replay_workspace_bytes(int(max_mem))
    check(nb if nb < 0 else 0, "rlp_replay_workspace_bytes")
    return torch.empty(int(nb), dtype=torch.uint8, device=_dev(device))


def replay_sample_reward_top(rb, max_mem, batch, seed, counter, workspace=None, out=None):
    dev = torch.device("cuda")
    out = out if out is not None else torch.empty(int(batch), dtype=torch.int64, device=dev)
    ws = workspace if workspace is not None else replay_workspace(max_mem, dev)
    n_out = C.c_int64(0)
    check(lib().rlp_replay_sample_reward_top(C.byref(rb), int(max_mem), int(batch), int(seed),
                                             int(counter), ptr(out), C.byref(n_out), ptr(ws),
                                             ws.numel(), stream_ptr()),
          "rlp_replay_sample_reward_top")
    return out[:n_out.value]


def replay_gather(rb, index, out=None):
    B = int(index.shape[0])
    dev = index.device
    f32 = dict(dtype=torch.float32, device=dev)
    out = out if out is not None else (
        torch.empty((B, rb.S), **f32), torch.empty((B, rb.A), **f32), torch.empty(B, **f32),
        torch.empty((B, rb.S), **f32), torch.empty(B, **f32))
    s, a, r, s2, e = out
    index_ = index.contiguous()
    check(lib().rlp_replay_gather(C.byref(rb), ptr(index_), B, ptr(s), ptr(a), ptr(r),
                                  ptr(s2), ptr(e), stream_ptr()), "rlp_replay_gather")
    return out


# ---------------------------------------------------------------------------------------------
# Native DDPG update (include/rlp.h: rlp_ddpg_workspace, rlp_ddpg_update)
# ---------------------------------------------------------------------------------------------
def dense_net(flat, dims, offsets):
    """rlp_dense_net over a flat fp32 parameter tensor: dims [in, h..., out], offsets of each
    layer's W (floats; its b follows it)."""
    n = _abi.DenseNet()
    n.n_layers = len(dims) - 1
    if not 1 <= n.n_layers <= _abi.RLP_DENSE_MAX_LAYERS or len(offsets) != n.n_layers:
        raise ValueError(f"dense_net: {len(dims) - 1} layers (1..{_abi.RLP_DENSE_MAX_LAYERS})")
    for i, d in enumerate(dims):
        n.dims[i] = int(d)
    for i, o in enumerate(offsets):
        n.offset[i] = int(o)
    n.n_params, n.params = flat.numel(), flat.data_ptr()
    return n


def ddpg_workspace(nets, batch, device=None):
    nf = lib().rlp_ddpg_workspace(C.byref(nets), int(batch))
    check(nf if nf < 0 else 0, "rlp_ddpg_workspace")
    return torch.empty(int(nf), dtype=torch.float32, device=_dev(device))


def ddpg_update(nets, cfg, s, a, r, s_next, end, work, losses):
    """One DDPG learn() iteration on a sampled batch (all device fp32, contiguous); losses [2]."""
    check(lib().rlp_ddpg_update(C.byref(nets), C.byref(cfg), ptr(s), ptr(a), ptr(r), ptr(s_next),
                                ptr(end), ptr(work), ptr(losses), stream_ptr()), "rlp_ddpg_update")
    return losses


def sac_workspace(nets, batch, device=None):
    nf = lib().rlp_sac_workspace(C.byref(nets), int(batch))
    check(nf if nf < 0 else 0, "rlp_sac_workspace")
    return torch.empty(int(nf), dtype=torch.float32, device=_dev(device))


def sac_update(nets, cfg, s, a, r, s_next, dw, noise, work, losses):
    """One SAC learn() iteration (include/rlp.h rlp_sac_update); noise None or [2][B][A]."""
    check(lib().rlp_sac_update(C.byref(nets), C.byref(cfg), ptr(s), ptr(a), ptr(r), ptr(s_next),
                               ptr(dw), ptr(noise), ptr(work), ptr(losses), stream_ptr()),
          "rlp_sac_update")
    return losses
