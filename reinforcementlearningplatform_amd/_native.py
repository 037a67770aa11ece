"""ctypes binding of librlp.so (the HIP/gfx950 library behind include/rlp.h).

There is no CPU fallback: if the library is missing or a call fails, this module raises. Device
buffers are torch tensors on a ROCm device; every call is ordered on the caller's current stream.
"""
import ctypes as C
import os

import torch  # import first: its libamdhip64 is the runtime librlp.so binds to (same SONAME)

from . import _abi

_LIB_NAME = "librlp.so"
ABI_VERSION = 3  # include/rlp.h RLP_ABI_VERSION
_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


class RLPError(RuntimeError):
    pass


def lib_path():
    return os.environ.get("RLP_LIBRARY", os.path.join(_HERE, _LIB_NAME))


def _declare(lib):
    vp, i32, i64, u64, dbl = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_double
    sig = {
        "rlp_abi_version": (i32, []),
        "rlp_last_error_string": (C.c_char_p, []),
        "rlp_struct_size": (i64, [i32]),
        "rlp_env_dims": (i32, [i32, vp, vp, vp]),
        "rlp_env_reset": (i32, [i32, vp, vp, i32, vp, vp, u64, u64, u64, vp]),
        "rlp_env_observe": (i32, [i32, vp, vp, i32, vp, vp]),
        "rlp_env_step": (i32, [i32, vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]),
        "rlp_mlp_param_count": (i64, [vp]),
        "rlp_mlp_forward_workspace_bytes": (i64, [vp, i32]),
        "rlp_mlp_forward": (i32, [vp, vp, vp, vp, i32, vp, vp, i64, vp]),
        "rlp_mfma_packed_count": (i64, [vp]),
        "rlp_mfma_pack": (i32, [vp, vp, vp, vp]),
        "rlp_policy_sample": (i32, [vp, i32, i32, vp, vp, vp, vp, u64, u64, u64, vp, vp, vp]),
        "rlp_sac_sample": (i32, [vp, i32, i32, vp, vp, vp, vp, vp, vp, i32, vp, u64, u64, u64, vp, vp,
                                 vp]),
        "rlp_rollout": (i32, [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "rlp_rollout_workspace_bytes": (i64, [i32, vp, vp, vp]),
        "rlp_mfma_forward": (i32, [vp, vp, vp, vp, i64, i32, vp]),
        "rlp_value_fixup": (i32, [vp, vp, vp, vp, vp, vp, i64, i32, vp]),
        "rlp_selftest_gemm_guard": (i32, [i32]),
        "rlp_set_rollout_sub": (i32, [i32]),
        "rlp_set_rollout_physics": (i32, [i32]),
        "rlp_set_mlp_precision": (i32, [i32]),
        "rlp_get_mlp_precision": (i32, []),
        "rlp_reward_norm": (i32, [vp, i32, i32, vp, vp, vp, vp]),
        "rlp_reward_norm_workspace": (i64, [i32, i32]),
        "rlp_gae": (i32, [vp, vp, vp, vp, vp, dbl, dbl, i32, i32, vp, vp, vp, vp]),
        "rlp_adv_normalize": (i32, [vp, i64, vp, i32, vp]),
        "rlp_reward_norm_statistics": (i32, [vp, i32, i32, vp, vp, vp]),
        "rlp_reward_norm_apply": (i32, [vp, i32, i32, vp, vp, vp]),
        "rlp_gae_normalized": (i32, [vp, vp, vp, vp, vp, vp, dbl, dbl, i32, i32, vp, vp, vp, vp]),
        "rlp_adv_stats_parts": (i32, [i32]),
        "rlp_reward_norm_parts": (i64, [i32, i32]),
        "rlp_reward_norm_stats": (i32, [vp, i32, i32, vp, vp]),
        "rlp_reward_norm_finish": (i32, [vp, i32, i32, i32, vp, vp, vp, vp, vp]),
        "rlp_ppo2_workspace_floats": (i64, [vp, i64]),
        "rlp_ppo2_grad": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp]),
        "rlp_ppo2_dense_workspace_floats": (i64, [vp, i64]),
        "rlp_ppo2_dense_grad": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp]),
        "rlp_grad_sqnorm": (i32, [vp, i64, vp, vp]),
        "rlp_grad_clip": (i32, [vp, i64, vp, C.c_float, vp]),
        "rlp_adam_step": (i32, [vp, vp, vp, vp, i64, vp, vp, vp]),
        "rlp_replay_store": (i32, [vp, i64, vp, vp, vp, vp, vp, i64, vp]),
        "rlp_replay_sample_uniform": (i32, [i64, i64, u64, u64, vp, vp]),
        "rlp_replay_workspace_bytes": (i64, [i64]),
        "rlp_replay_sample_reward_top": (i32, [vp, i64, i64, u64, u64, vp, vp, vp, i64, vp]),
        "rlp_replay_gather": (i32, [vp, vp, i64, vp, vp, vp, vp, vp, vp]),
        "rlp_ddpg_workspace": (i64, [vp, i32]),
        "rlp_ddpg_update": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "rlp_sac_workspace": (i64, [vp, i32]),
        "rlp_sac_update": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args


def lib():
    """Load librlp.so (raises if it is absent: the HIP path has no fallback)."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RLPError(f"{path} not found: build it with `make -C "
                           f"reinforcementlearningplatform_amd/csrc` or __graft_entry__.build()")
        _lib = C.CDLL(path)
        _declare(_lib)
        if _lib.rlp_abi_version() != ABI_VERSION:
            raise RLPError(f"librlp ABI version {_lib.rlp_abi_version()} != {ABI_VERSION} (rebuild "
                           f"librlp.so: make -C reinforcementlearningplatform_amd/csrc)")
        for i, (name, size) in enumerate(_abi.check_struct_sizes().items()):
            if _lib.rlp_struct_size(i) != size:
                raise RLPError(f"struct layout mismatch for {name}: C {_lib.rlp_struct_size(i)} "
                               f"vs ctypes {size}")
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().rlp_last_error_string().decode(errors="replace")
        raise RLPError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RLPError("librlp takes device tensors only (got a CPU tensor)")
    if not t.is_contiguous():
        raise RLPError("librlp takes contiguous tensors only")
    return C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


MLP_FP32, MLP_F16X3 = 0, 1


def set_mlp_precision(mode):
    """rlp_rollout's hidden-layer arithmetic: MLP_F16X3 (default) or MLP_FP32 (include/rlp.h)."""
    check(lib().rlp_set_mlp_precision(int(mode)), "rlp_set_mlp_precision")


def get_mlp_precision():
    return int(lib().rlp_get_mlp_precision())


def set_rollout_sub(sub):
    check(lib().rlp_set_rollout_sub(int(sub)), "rlp_set_rollout_sub")


def set_rollout_physics(shared):
    """-1: auto (default: 3 when the envs fill every CU with a 256-env block, else — and always
    for the UAV — 5), 1: shared-physics rollout kernel (two 4-wave blocks per CU), 3: one 8-wave
    block of 32-env waves per CU, 5: one 4-wave block of 32-env waves per CU (1 wave per SIMD),
    0: register-resident kernel (include/rlp.h rlp_set_rollout_physics)."""
    check(lib().rlp_set_rollout_physics(int(shared)), "rlp_set_rollout_physics")
