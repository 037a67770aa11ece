"""CPU ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product package).

numpy/ctypes front-end of oracle/rlp_oracle.c, the plain-C restatement of the reference's
per-env arithmetic (see that file's header). Used by tests/ (parity checker), by
__graft_entry__.smoke() and by bench.py's `cpu_baseline` leg.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from reinforcementlearningplatform_amd import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "librlp_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def dims(kind):
    return _abi.ENV_DIMS[kind]


def env_step(kind, params, state, action, want_obs_cur=True):
    """state: f64 [D][n] (modified in place); action f32 [n][A]."""
    D, S, A = dims(kind)
    n = state.shape[1]
    action = np.ascontiguousarray(action, dtype=np.float32).reshape(n, A)
    oc = np.zeros((n, S), np.float32) if want_obs_cur else None
    on = np.zeros((n, S), np.float32)
    r = np.zeros(n, np.float64)
    f = np.zeros(n, np.int32)
    d = np.zeros(n, np.uint8)
    rc = lib().oracle_env_step(kind, C.byref(params), _p(state), n, _p(action), _p(oc), _p(on),
                               _p(r), _p(f), _p(d))
    assert rc == 0
    return oc, on, r, f, d


def env_observe(kind, params, state):
    D, S, A = dims(kind)
    n = state.shape[1]
    o = np.zeros((n, S), np.float32)
    assert lib().oracle_env_observe(kind, C.byref(params), _p(state), n, _p(o)) == 0
    return o


def env_reset(kind, params, state, mask=None, init_state=None, seed=0, counter=0, env_id0=0):
    n = state.shape[1]
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    ini = None if init_state is None else np.ascontiguousarray(init_state, dtype=np.float64)
    assert lib().oracle_env_reset(kind, C.byref(params), _p(state), n, _p(m), _p(ini),
                                  C.c_uint64(seed), C.c_uint64(counter), C.c_uint64(env_id0)) == 0


def mlp_forward(desc, params, x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = x.shape[0]
    y = np.zeros((n, desc.dims[desc.n_layers]), np.float32)
    params = np.ascontiguousarray(params, dtype=np.float32)
    assert lib().oracle_mlp_forward(C.byref(desc), _p(params), _p(x), _p(y), n) == 0
    return y


def policy_sample(mean, std, a_min, a_max, noise=None, seed=0, counter=0, env_id0=0):
    mean = np.ascontiguousarray(mean, dtype=np.float32)
    n, A = mean.shape
    f = lambda v: np.ascontiguousarray(np.broadcast_to(np.asarray(v, np.float32), (A,)))
    std, a_min, a_max = f(std), f(a_min), f(a_max)
    nz = None if noise is None else np.ascontiguousarray(noise, dtype=np.float32)
    a = np.zeros((n, A), np.float32)
    lp = np.zeros((n, A), np.float32)
    assert lib().oracle_policy_sample(_p(mean), n, A, _p(std), _p(a_min), _p(a_max), _p(nz),
                                      C.c_uint64(seed), C.c_uint64(counter), C.c_uint64(env_id0),
                                      _p(a), _p(lp)) == 0
    return a, lp


def philox_normal(seed, counter, env_id, A):
    out = np.zeros(A, np.float32)
    lib().oracle_philox_normal_f32(C.c_uint64(seed), C.c_uint64(counter), C.c_uint64(env_id), A,
                                   _p(out))
    return out


def gae(r, v, vn, done, success, gamma, lmd):
    T, n = r.shape
    cv = lambda a, t: np.ascontiguousarray(a, dtype=t)
    r, v, vn = cv(r, np.float32), cv(v, np.float32), cv(vn, np.float32)
    done, success = cv(done, np.uint8), cv(success, np.uint8)
    adv = np.zeros((T, n), np.float32)
    vt = np.zeros((T, n), np.float32)
    lib().oracle_gae.argtypes = [C.c_void_p] * 5 + [C.c_double, C.c_double, C.c_int, C.c_int,
                                                     C.c_void_p, C.c_void_p]
    assert lib().oracle_gae(_p(r), _p(v), _p(vn), _p(done), _p(success), gamma, lmd, T, n,
                            _p(adv), _p(vt)) == 0
    return adv, vt


def reward_norm(r, rms=None):
    r = np.ascontiguousarray(r, dtype=np.float32)
    T, n = r.shape
    rms = np.zeros(4, np.float64) if rms is None else rms
    out = np.zeros((T, n), np.float32)
    assert lib().oracle_reward_norm(_p(r), T, n, _p(rms), _p(out)) == 0
    return out, rms


def set_threads(n):
    """Host threads of the oracle's env / row loops (OpenMP); returns the count in effect."""
    return lib().oracle_set_threads(int(n))


def rollout(kind, params, state, need_reset, actor_desc, actor_params, critic_desc,
            critic_params, cfg, want_buffers=True, forced_action=None):
    """Whole rollout segment on the CPU (the reference driver loop batched over n envs).

    forced_action [T][n][A] f32: teacher forcing — the envs step with these actions while the
    buffers record the oracle's own policy output / values (actor_params None: physics only)."""
    D, S, A = dims(kind)
    T, n = cfg.T, cfg.n
    bufs = None
    arrays = None
    if want_buffers:
        arrays = dict(obs=np.zeros((T, n, S), np.float32), obs_next=np.zeros((T, n, S), np.float32),
                      action=np.zeros((T, n, A), np.float32), logp=np.zeros((T, n, A), np.float32),
                      reward=np.zeros((T, n), np.float32), value=np.zeros((T, n), np.float32),
                      value_next=np.zeros((T, n), np.float32), done=np.zeros((T, n), np.uint8),
                      success=np.zeros((T, n), np.uint8), flag=np.zeros((T, n), np.int8))
        bufs = _abi.RolloutBufs(**{k: v.ctypes.data for k, v in arrays.items()})
    nets = actor_params is not None
    ap = np.ascontiguousarray(actor_params, dtype=np.float32) if nets else None
    cp = np.ascontiguousarray(critic_params, dtype=np.float32) if nets else None
    fa = None
    if forced_action is not None:
        fa = np.ascontiguousarray(forced_action, dtype=np.float32).reshape(T, n, A)
    rc = lib().oracle_rollout_forced(kind, C.byref(params), _p(state), _p(need_reset),
                                     C.byref(actor_desc) if nets else None, _p(ap),
                                     C.byref(critic_desc) if nets else None, _p(cp), C.byref(cfg),
                                     C.byref(bufs) if bufs is not None else None, _p(fa))
    assert rc == 0
    return arrays
