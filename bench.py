"""bench.py — env-steps/s of the CartPole PPO2 rollout hot path on 1..8 MI355X (one process per GPU).

One bench "step" = one PPO2 rollout iteration over the config's synthetic env batch, entirely on
the GPU: T env-steps x n envs of {auto-reset, actor forward + Gaussian sample, critic V(s), RK4 env
step, buffer append} in the fused HIP kernel (rlp_rollout), then the critic on terminal s', reward
normalisation, GAE(lambda) and advantage normalisation — everything learn() consumes
(SURVEY.md §8a rows a1-a6, a14, a15, a17-a19). `value` = env-steps/s of the whole job.
With --e2e the K-epoch PPO2 update (librlp's native HIP update kernels on the same GPU) is also
timed and reported separately under "e2e".

Launch: python bench.py [--gpus N]   |   torchrun --nproc-per-node N bench.py --gpus N
With --gpus N > 1 and no torchrun environment (WORLD_SIZE unset) bench.py starts the N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, one GPU
each); the launching process makes no GPU call. Every rank checks WORLD_SIZE == --gpus.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(argv):
    """`python bench.py --gpus N` (N > 1) outside torchrun: run N rank processes of this script,
    pass rank 0's JSON line through, return the first failing exit code (0 when all succeed).
    Runs before torch is imported, so this process never touches the GPU (no exec after a HIP
    call: the ranks are children)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=None)
    n = pre.parse_known_args(argv)[0].gpus
    if n is None or n <= 1 or "WORLD_SIZE" in os.environ:
        return None
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    failed_at = None
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc, failed_at = code, time.monotonic()
        # one rank failed: the others may be waiting in a collective forever. They get a grace
        # period to fail (or finish) on their own first, so each reports its own error.
        if failed_at is not None and time.monotonic() - failed_at > 30.0:
            for q in live:
                q.terminate()
            failed_at = float("inf")
        time.sleep(0.2)
    return rc


if __name__ == "__main__":
    _rc = _self_launch(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc if _rc >= 0 else 128 - _rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from reinforcementlearningplatform_amd import _abi as A  # noqa: E402
from reinforcementlearningplatform_amd import _native  # noqa: E402
from reinforcementlearningplatform_amd import kernels as K  # noqa: E402

METRIC = "env-steps/sec (whole node), CartPole+UavRobust PPO2 @ 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense peak
PEAK_F16_MFMA_TFLOPS = 16 * PEAK_FP32_MFMA_TFLOPS   # f16/bf16 dense MFMA = 16x the f32 rate
# f16x3 split: 3 f16 MFMAs per fp32-equivalent product -> the path's fp32-equivalent ceiling
PEAK_F16X3_TFLOPS = PEAK_F16_MFMA_TFLOPS / 3
PEAK_HBM_GBS = 8000.0
# the rollout kernel each --physics mode launches (rlp_rollout.hip; the name rocprof reports)
# (template arguments as rocprof prints them: KIND, H, SUB, waves per block, waves per SIMD)
ROLLOUT_KERNEL = {"shared": "rlp::rollout_sp_kernel<KIND,256,SUB,4,2>",
                  "cu": "rlp::rollout_sp_kernel<KIND,256,2,8,2>",
                  "cu4": "rlp::rollout_sp_kernel<KIND,256,2,4,1>",
                  "lanes": "rlp::rollout_kernel<KIND,256,SUB,true>"}

TRAFFIC_SOURCE = ("looked up from profiles/pmc_traffic.json (a committed rocprofv3 FETCH_SIZE / "
                  "WRITE_SIZE pass of this workload and kernel), not measured in this run")
PHYSICS_MODES = {"auto": -1, "lanes": 0, "shared": 1, "cu": 3, "cu4": 5}


def rollout_kernel_name(physics, n, env="cartpole", sub=0):
    """The kernel rlp_rollout runs for `physics` and the --sub knob, mirroring rlp_rollout's own
    selection (rlp_rollout.hip rollout_kind): auto = one 8-wave block per CU when n fills every CU
    with a 256-env block (not the UAV), else one 4-wave block of 32-env waves per CU — both only
    for sub 0 / 2; any other sub falls back to the shared-physics kernel (mode 1)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if physics == "auto":
        if sub in (0, 2):
            physics = "cu" if env != "uav" and (n + 255) // 256 >= cus else "cu4"
        else:
            physics = "shared"
    if sub == 0:   # the library's auto sub for the modes that take it
        sub = 1 if (n + 127) // 128 < 2 * cus else 2
    return ROLLOUT_KERNEL[physics].replace("SUB", str(sub))


ENVS = {
    "cartpole": (A.RLP_ENV_CARTPOLE, lambda: A.cartpole_params("ppo2"), 3),
    "uav": (A.RLP_ENV_UAV_HOVER_OUTER_LOOP, A.uav_hover_params, 1),
    "angleonly": (A.RLP_ENV_CARTPOLE_ANGLEONLY, A.angleonly_params, 3),
    "soi": (A.RLP_ENV_SOI, lambda: A.soi_params("env"), 2),
    "ugv": (A.RLP_ENV_UGV_FORWARD, lambda: A.ugv_params(A.RLP_ENV_UGV_FORWARD, "ppo2"), 2),
}


def orthogonal_params(desc, gains, seed):
    """PPOActor_Gaussian / PPOCritic init (demonstration/PPO2/PPO2-4-CartPole/train.py:59-70):
    orthogonal weights, zero bias; flattened in nn.Module.parameters() order."""
    g = torch.Generator().manual_seed(seed)
    out = []
    ds = desc.layer_dims()
    for i in range(desc.n_layers):
        w = torch.empty(ds[i + 1], ds[i])
        torch.nn.init.orthogonal_(w, gain=gains[i], generator=g)
        out += [w.flatten(), torch.zeros(ds[i + 1])]
    return torch.cat(out)


def mlp_flops(desc):
    ds = desc.layer_dims()
    return sum(2 * ds[i] * ds[i + 1] for i in range(desc.n_layers))


def dims_flops(dims):
    """Forward FLOP per row of a Linear stack with layer widths `dims`."""
    return sum(2 * dims[i] * dims[i + 1] for i in range(len(dims) - 1))


def update_flops_per_row(dims):
    """Algorithmic FLOP per row of one optimiser step's gradient of a Linear stack (what
    loss.backward() does after the forward): forward sum 2 in out, backward data pass through every
    layer but the first (sum_{l >= 1} 2 in out), weight + bias gradients sum 2 (in + 1) out."""
    L = len(dims) - 1
    return (dims_flops(dims) + sum(2 * dims[i] * dims[i + 1] for i in range(1, L))
            + sum(2 * (dims[i] + 1) * dims[i + 1] for i in range(L)))


def _wgrad_flops(dims):
    return sum(2 * (dims[i] + 1) * dims[i + 1] for i in range(len(dims) - 1))


def ddpg_learn_flops(S=4, A=2, H=256):
    """Algorithmic FLOP per batch row of one DDPG learn() (DDPG.py:72-109) with the SOI driver's
    nets (actor [S,H,H,A], critic cat(s,a) [S+A,H,H,1]): target actor + target critic forward; the
    critic's forward, backward data pass (layers >= 1) and weight gradients; the actor's forward,
    the updated critic's forward on (s, mu(s)), its backward data pass down to the action columns,
    the actor's backward data pass (layers >= 1) and weight gradients."""
    da, dc = [S, H, H, A], [S + A, H, H, 1]
    fa, fc = dims_flops(da), dims_flops(dc)
    critic = fc + (fc - 2 * dc[0] * H) + _wgrad_flops(dc)
    actor = fa + fc + (fc - 2 * dc[0] * H + 2 * A * H) + (fa - 2 * S * H) + _wgrad_flops(da)
    return fa + fc + critic + actor


def sac_learn_flops(S=41, A=2, h=(128, 64)):
    """Algorithmic FLOP per batch row of one SAC learn() (Soft_Actor_Critic.py:70-129) with the SAC
    demo nets (actor trunk [S,128,64] + mean / log_std heads [64 -> A]; twin critics
    cat(s,a) [S+A,128,64,1]): the actor on s' and the twin target critics; the twin critics'
    forward, backward data (layers >= 1) and weight gradients; the actor on s, the twin critics on
    (s, a~pi(s)) and their backward data pass down to the action columns, the actor's backward data
    pass (layers >= 1) and weight gradients (trunk and both heads)."""
    dt, dc = [S, *h], [S + A, *h, 1]
    fa = dims_flops(dt) + 2 * (2 * h[-1] * A)
    wa = _wgrad_flops(dt) + 2 * 2 * (h[-1] + 1) * A
    fc = dims_flops(dc)
    target = fa + 2 * fc
    critic = 2 * fc + 2 * (fc - 2 * dc[0] * h[0]) + 2 * _wgrad_flops(dc)
    actor = fa + 2 * fc + 2 * (fc - 2 * dc[0] * h[0] + 2 * A * h[0]) + (fa - 2 * S * h[0]) + wa
    return target + critic + actor


def learn_roofline(flop_per_row, batch, learn_ms):
    ach = flop_per_row * batch / (learn_ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": ach, "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / PEAK_FP32_MFMA_TFLOPS, "flop_per_learn": flop_per_row * batch,
            "peak_basis": "f32 MFMA dense (the update's v_mfma_f32_16x16x4_f32 GEMMs)",
            "note": "one learn() of `batch` rows is a chain of small dependent launches in one HIP "
                    "graph: latency-bound at this batch, far from the roof"}


def offpolicy_reuse(make_loop, n, ref_rows, flop_per_row,
                    configs=((4096, 64), (16384, 16), (65536, 4), (131072, 2)), steps=3, warmup=1):
    """The off-policy loop at the reference driver's sample reuse or near it: per vector step of n
    transitions, `iters` learn() iterations of `batch` rows (one captured graph replayed iters
    times), so sampled rows per transition = batch * iters / n against the reference's
    `ref_rows` per transition (one ref_rows-row learn() per env step). The configurations give
    ratio 1/16 at the bench's n; each takes 4x fewer, 4x fatter updates than the one before."""
    out = []
    for batch, iters in configs:
        loop, agent = make_loop(batch, iters)
        # enough warm-up steps to hold `batch` rows: learn() skips while the replay has fewer
        for _ in range(max(warmup, -(-batch // n))):
            loop.step(learn=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            loop.step(learn=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        agent.learn(iter=iters)
        ev[1].record()
        torch.cuda.synchronize()
        lms = ev[0].elapsed_time(ev[1]) / iters
        out.append({"value": n * steps / dt, "unit": "env-steps/s", "batch": batch,
                    "learn_iters_per_step": iters, "learn_ms": lms,
                    "step_ms": dt / steps * 1e3,
                    "sampled_rows_per_transition": batch * iters / n,
                    "ratio_vs_reference": batch * iters / n / ref_rows,
                    "learn_roofline": learn_roofline(flop_per_row, batch, lms)})
        del loop, agent
    return out


def _net_dims(module):
    lin = [m for m in module.modules() if isinstance(m, torch.nn.Linear)]
    return [lin[0].in_features] + [l.out_features for l in lin]


def update_roofline(learner, rows, k_epochs, update_ms):
    """achieved TFLOP/s of the K-epoch update of one PPO2 iteration (both nets, full batch),
    priced against the arithmetic the update runs: the f16x3 kernels' 838.9 TF ceiling
    (rlp_ppo2_grad) or the f32 MFMA peak (rlp_ppo2_dense_grad, torch)."""
    dims = [_net_dims(learner.actor), _net_dims(learner.critic)]
    per_row = sum(update_flops_per_row(d) for d in dims)
    flop = per_row * rows * k_epochs
    nets = [getattr(learner, k, None) for k in ("net_a", "net_c")]
    dense = [getattr(m, "dense", True) for m in nets]
    f16x3 = type(learner).__name__ == "NativePPO2Learner" and not any(dense)
    ext = f16x3 and any(getattr(m, "ext", False) for m in nets)
    ach = flop / (update_ms * 1e-3) / 1e12
    out = {"bound": "mfma", "achieved": ach, "unit": "TFLOP/s", "flop_per_iteration": flop,
           "update_ms": update_ms,
           "flop_basis": "K x rows x (forward + backward data + weight gradients) of both nets"}
    if ext:
        # the lidar nets' layer 1 (41 inputs: h1 forward and dW1) runs on exact-f32 MFMA and is
        # HBM-bound; the rest on the f16x3 kernels: each share priced against its own arithmetic's
        # peak (the time both would take at their peaks, combined)
        flop1 = sum(2 * d[0] * d[1] + 2 * (d[0] + 1) * d[1] for d in dims) * rows * k_epochs
        peak = flop / (flop1 / PEAK_FP32_MFMA_TFLOPS + (flop - flop1) / PEAK_F16X3_TFLOPS)
        out.update(peak=peak, frac=ach / peak, layer1_flop_share=flop1 / flop,
                   peak_basis="mixed: layer 1 (f32 MFMA, HBM-bound) at the f32 MFMA peak, the "
                              "rest at the f16x3 ceiling (f16 MFMA / 3)",
                   frac_vs_f16x3_ceiling=ach / PEAK_F16X3_TFLOPS)
    else:
        peak = PEAK_F16X3_TFLOPS if f16x3 else PEAK_FP32_MFMA_TFLOPS
        out.update(peak=peak, frac=ach / peak,
                   peak_basis="f16x3 ceiling (f16 MFMA / 3)" if f16x3 else "f32 MFMA dense")
    return out


def _template_args(name):
    return [a.strip() for a in name[name.find("<") + 1:name.rfind(">")].split(",")][1:]


def pmc_traffic(workload, n, T, kernel=None):
    """HBM bytes per rollout launch from the committed rocprofv3 PMC pass of this workload
    (profiles/pmc_traffic.json: FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM + WRITE_SIZE);
    None when that pass profiled another kernel variant than `kernel` (the one this run launches)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    e = d.get(workload)
    if not e or e.get("envs_per_gpu") != n or e.get("T") != T:
        return None
    if kernel is not None and e.get("kernel"):
        want, have = _template_args(kernel), _template_args(e["kernel"])
        if all(a.isdigit() for a in want) and want != have[:len(want)]:
            return None
    return e["hbm_bytes_per_launch"]


def pmc_kernel_traffic(name, kernel):
    """HBM bytes per launch of an hbm_legs kernel from the committed PMC pass
    (profiles/pmc_traffic.json "hbm_kernels"), or None — also when that pass profiled other
    kernels than `kernel` (the leg's label, launches joined by " + ")."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        e = json.load(f).get("hbm_kernels", {}).get(name)
    if e is None:
        return None
    parts = kernel.split(" + ")
    if len(parts) != len(e["kernels"]) or not all(p.startswith(k) for p, k in zip(parts, e["kernels"])):
        return None
    return e.get("hbm_bytes_per_launch")


class Segment:
    """Device-resident state + buffers of one rank's env batch."""

    def __init__(self, env, n, T, seed, env_id0, H=256):
        kind, pf, timeout_flag = ENVS[env]
        self.env = env
        self.kind, self.params = kind, pf()
        D, S, Ad = A.ENV_DIMS[kind]
        self.S, self.Ad, self.n, self.T = S, Ad, n, T
        self.ad = A.MLPDesc.make([S, H, H, Ad], [A.RLP_ACT_TANH] * 3)
        self.cd = A.MLPDesc.make([S, H, H, 1], [A.RLP_ACT_TANH, A.RLP_ACT_TANH, A.RLP_ACT_NONE])
        self.actor = orthogonal_params(self.ad, [1.0, 1.0, 0.01], seed).cuda()
        self.critic = orthogonal_params(self.cd, [1.0, 1.0, 1.0], seed + 1).cuda()
        self.apk = K.mfma_pack(self.ad, self.actor)
        self.cpk = K.mfma_pack(self.cd, self.critic)
        lo, hi = A.action_bounds(kind, self.params)
        self.std = [(h - l) / 2 / 3 for l, h in zip(lo, hi)]   # init_std = fm/3 (train.py:169)
        self.lo, self.hi = lo, hi
        self.seed, self.env_id0 = seed, env_id0
        self.rule, self.flag = A.RLP_SUCCESS_DONE_AND_FLAG_NE, timeout_flag
        self.state = K.new_state(kind, n)
        self.need = torch.ones(n, dtype=torch.uint8, device="cuda")
        self.bufs = K.rollout_buffers(kind, T, n)
        self.rms = torch.zeros(4, dtype=torch.float64, device="cuda")
        self.work = K.reward_norm_workspace(T, n, "cuda")
        self.rnorm = torch.empty((T, n), dtype=torch.float32, device="cuda")
        self.adv = torch.empty((T, n), dtype=torch.float32, device="cuda")
        self.vt = torch.empty((T, n), dtype=torch.float32, device="cuda")
        self.stats = K.adv_stats_buffer(n, device="cuda")
        self.step0 = 0

    def rollout(self):
        cfg = K.make_rollout_cfg(self.T, self.n, self.seed, self.step0, self.env_id0, self.std,
                                 self.lo, self.hi, self.rule, self.flag)
        K.rollout(self.kind, self.params, self.state, self.need, self.ad, self.apk, self.cd,
                  self.cpk, cfg, self.bufs)
        self.step0 += self.T

    def learn_side(self):
        b = self.bufs
        # V(s'_t) of terminal transitions (non-terminal ones were written by the rollout)
        K.value_fixup(self.cd, self.cpk, b["obs_next"], b["done"], b["success"], b["value_next"])
        # one rank's learn side as VecPPO2.advantages runs it: the reward statistics, GAE over
        # the raw rewards normalised on load (the normalised rewards are not stored), the
        # advantage normalisation
        K.reward_norm_statistics(b["reward"], self.rms, self.work)
        K.gae_normalized(b["reward"], self.work, b["value"], b["value_next"], b["done"],
                         b["success"], 0.999, 0.95, adv=self.adv, v_target=self.vt,
                         stats=self.stats)
        K.adv_normalize(self.adv, self.stats)

    def iteration(self):
        self.rollout()
        self.learn_side()


E2E_ENVS = {"cartpole": ("CartPole", "CartPole"), "uav": ("UavRobust", "uav_hover_outer_loop")}


def e2e_iterations(seg, iters, k_epochs=6, learner="native"):
    """Whole PPO2 iterations through the product driver class VecPPO2 (the Distributed_PPO2
    Worker): rollout + value fix-up + reward normalisation + GAE + advantage normalisation + K
    full-batch epochs of the clipped-surrogate / MSE update (librlp's native update, or torch
    autograd + Adam, on this GPU). Under torch.distributed this is the data-parallel Worker with
    norm_scope='global' (the Distributed_PPO2 default): every optimiser step all-reduces the
    actor+critic gradients and every iteration gathers the reward / advantage statistics.
    k_epochs: the DPPO2 CartPole drivers' k_epo = 6 (demonstration/DPPO2/DPPO2-4-CartPole/
    train.py:161) or the PPO2 demo's K = 30 (PPO2-4-CartPole/train.py:146).
    Returns env-steps/s of this rank, s per iteration, and the rollout launch time inside the
    training loop (HIP events on the launch stream)."""
    import importlib
    from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import (DEFAULT_PPO_MSG,
                                                                                   VecPPO2)
    from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic
    pkg, cls_name = E2E_ENVS[seg.env]
    uevs = []
    env_cls = getattr(importlib.import_module(
        f"reinforcementlearningplatform_amd.environment.{pkg}.{cls_name}"), cls_name)
    env = env_cls(n_envs=seg.n, seed=seg.seed, env_id0=seg.env_id0)
    actor = PPOActor_Gaussian(seg.S, seg.Ad, np.array(seg.lo), np.array(seg.hi), init_std=seg.std[0])
    critic = PPOCritic(seg.S)
    with torch.no_grad():   # start from the bench nets
        for m, flat in ((actor, seg.actor), (critic, seg.critic)):
            off = 0
            for p in m.parameters():
                p.copy_(flat[off:off + p.numel()].view_as(p).cpu())
                off += p.numel()
    msg = dict(DEFAULT_PPO_MSG, K_epochs=k_epochs, norm_scope="global")
    vec = VecPPO2(env, actor, critic, msg, T=seg.T, seed=seg.seed, learner=learner,
                  success_rule=(seg.rule, seg.flag))
    evs = []

    def one(ev=None):
        if ev is not None:
            ev[0].record()
        vec.rollout()
        if ev is not None:
            ev[1].record()
        vec.advantages()
        if ev is not None:
            ev[2].record()
        vec.update()
        if ev is not None:
            ev[3].record()
    one()
    dist_on = torch.distributed.is_available() and torch.distributed.is_initialized()
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        evs.append(tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)))
        one(evs[-1])
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist_on:   # the slowest rank's clock
        t = torch.tensor([dt], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    rollout_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    update_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in evs]))
    info = {"rollout_ms": rollout_ms, "update_ms": update_ms, "learner": type(vec.learner).__name__,
            "norm_scope": "global" if vec.global_norm else "rank",
            "update_roofline": update_roofline(vec.learner, seg.n * seg.T, k_epochs, update_ms)}
    if dist_on:
        info["allreduce"] = allreduce_probe(vec)
    del vec, env
    return seg.n * seg.T * iters / dt, dt / iters, info


def allreduce_probe(vec, reps=30):
    """The per-optimiser-step RCCL all-reduce of the learner (one flat buffer of the actor+critic
    gradients, native_ppo2.NativePPO2Learner._allreduce_grads), timed alone on this rank with HIP
    events, and the collectives one PPO2 iteration issues."""
    lrn = vec.learner
    numel = sum(p.numel() for p in lrn.params())
    buf = torch.zeros(numel, dtype=torch.float32, device="cuda")
    for _ in range(3):
        torch.distributed.all_reduce(buf, group=lrn.pg)
    torch.distributed.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.distributed.all_reduce(buf, group=lrn.pg)
    e1.record()
    torch.cuda.synchronize()
    per_iter = vec.msg['K_epochs'] + (2 if vec.global_norm else 0)
    return {"bytes": numel * 4, "ms_per_allreduce": e0.elapsed_time(e1) / reps,
            "allreduces_per_iteration": per_iter,
            "note": "K gradient all-reduces (one per optimiser step) + the reward-chunk and "
                    "advantage-partial gathers of norm_scope='global'"}


def _demo_nets(S, A, lo, hi, actor_widths, critic_widths, seed):
    """The demo drivers' PPOActor_Gaussian / PPOCritic with their own hidden widths (tanh hidden
    layers, tanh(mean) * gain + off; orthogonal init, demonstration/PPO2/*/train.py)."""
    import torch.nn as nn

    class DemoActor(nn.Module):
        def __init__(self):
            super().__init__()
            d = (S,) + tuple(actor_widths)
            self.hidden = nn.ModuleList([nn.Linear(d[i], d[i + 1]) for i in range(len(actor_widths))])
            self.mean_layer = nn.Linear(d[-1], A)
            self.a_min, self.a_max = torch.tensor(lo, dtype=torch.float), torch.tensor(hi, dtype=torch.float)
            self.off = (self.a_min + self.a_max) / 2.0
            self.gain = self.a_max - self.off
            self.std = torch.tensor(float((hi[0] - lo[0]) / 6), dtype=torch.float)
            for l in self.hidden:
                nn.init.orthogonal_(l.weight)
                nn.init.constant_(l.bias, 0)
            nn.init.orthogonal_(self.mean_layer.weight, gain=0.01)
            nn.init.constant_(self.mean_layer.bias, 0)

        def forward(self, s):
            for l in self.hidden:
                s = torch.tanh(l(s))
            return torch.tanh(self.mean_layer(s)) * self.gain + self.off

    class DemoCritic(nn.Module):
        def __init__(self):
            super().__init__()
            d = (S,) + tuple(critic_widths) + (1,)
            self.layers = nn.ModuleList([nn.Linear(d[i], d[i + 1]) for i in range(len(d) - 1)])
            for l in self.layers:
                nn.init.orthogonal_(l.weight)
                nn.init.constant_(l.bias, 0)

        def forward(self, s):
            for l in self.layers[:-1]:
                s = torch.tanh(l(s))
            return self.layers[-1](s)

    torch.manual_seed(seed)
    return DemoActor(), DemoCritic()


DEMO_E2E = {
    # demonstration/PPO2/PPO2-4-SecondOrderIntegration/train.py:37-125,146 (K = 30)
    "soi": dict(actor=(128, 64, 32), critic=(64, 64), K=30, n=65536, T=64),
    # demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/train.py:48-50,95-97,146 (K = 25)
    "ugvoa": dict(actor=(256, 256), critic=(256, 256), K=25, n=16384, T=64),
}


def demo_nets_e2e_leg(rank, which, iters=2, seed=19):
    """Whole PPO2 iterations (VecPPO2) for the PPO2 drivers whose nets the fused f16x3 kernels do
    not take: the rollout through rlp_rollout's plain-layout path (SOI) or its per-step lidar path
    (UGV-OA), the K-epoch update through rlp_ppo2_dense_grad (exact f32 MFMA: the fused per-row
    kernel for the SOI nets) or, for the 41-input nets, rlp_ppo2_grad (f16x3) + Adam."""
    from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import VecPPO2
    c = DEMO_E2E[which]
    n, T = c["n"], c["T"]
    if which == "soi":
        from reinforcementlearningplatform_amd.environment.SecondOrderIntegration.SecondOrderIntegration \
            import SecondOrderIntegration
        env = SecondOrderIntegration(n_envs=n, seed=seed, env_id0=rank * n)
    else:
        from reinforcementlearningplatform_amd.environment.UGVForwardObstacleAvoidance import \
            UGVForwardObstacleAvoidance
        env = UGVForwardObstacleAvoidance(n_envs=n, variant="ppo2", seed=seed, env_id0=rank * n)
    env.reset(random=True)
    ar = np.array(env.action_range, dtype=np.float64)
    actor, critic = _demo_nets(env.state_dim, env.action_dim, ar[:, 0], ar[:, 1], c["actor"],
                               c["critic"], seed)
    vec = VecPPO2(env, actor, critic, {'K_epochs': c["K"], 'gamma': 0.99}, T=T)
    evs = []

    def one(ev=None):
        if ev is not None:
            ev[0].record()
        vec.rollout()
        if ev is not None:
            ev[1].record()
        vec.advantages()
        if ev is not None:
            ev[2].record()
        vec.update()
        if ev is not None:
            ev[3].record()
    one()
    dist_on = torch.distributed.is_available() and torch.distributed.is_initialized()
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        evs.append(tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)))
        one(evs[-1])
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([dt], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    lr = vec.learner
    update_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in evs]))
    nets = [getattr(lr, k, None) for k in ("net_a", "net_c")]
    kinds = [("rlp_ppo2_dense_grad (exact f32 MFMA, fused per-row kernel)" if m.fused else
              "rlp_ppo2_dense_grad (exact f32 MFMA GEMMs)") if m.dense else "rlp_ppo2_grad (f16x3 FD + wgrad)"
             for m in nets if m is not None]
    out = {"value": n * T * iters / dt, "unit": "env-steps/s", "s_per_iteration": dt / iters,
           "rollout_ms": float(np.mean([e[0].elapsed_time(e[1]) for e in evs])),
           "update_ms": update_ms, "envs_per_gpu": n,
           "T": T, "K_epochs": c["K"], "learner": type(lr).__name__,
           "update": (" / ".join(dict.fromkeys(kinds)) + " + rlp_adam_step") if kinds else "torch",
           "update_roofline": update_roofline(lr, n * T, c["K"], update_ms),
           "rollout": "plain-layout nets (per-step rlp_mlp_forward + sample/step kernel)"
                      if vec.plain else "fused / lidar per-step path",
           "config": f"{env.name} PPO2, actor {[env.state_dim, *c['actor'], env.action_dim]} / "
                     f"critic {[env.state_dim, *c['critic'], 1]} tanh (the demo driver's nets)"}
    del vec, env
    return out


def soi_ddpg_leg(rank, n=65536, steps=20, warmup=3, batch=4096, capacity=1 << 20, seed=11,
                 reuse_legs=True):
    """BASELINE config 3: SecondOrderIntegration DDPG (DDPG copy), n envs, replay buffer in HBM.
    One step = actor forward (librlp MLP, ReLU) + exploration noise + env step + n transitions
    into the replay ring + auto-reset, then one DDPG update on `batch` rows sampled from HBM
    (the driver's one learn() per env step, train.py:240, with the batch scaled from 64)."""
    import torch.nn as nn
    import torch.nn.functional as func
    from reinforcementlearningplatform_amd.algorithm.actor_critic.DDPG import DDPG
    from reinforcementlearningplatform_amd.algorithm.actor_critic.vec_ddpg import VecDDPG
    from reinforcementlearningplatform_amd.environment.SecondOrderIntegration.SecondOrderIntegration \
        import SecondOrderIntegration

    class Critic(nn.Module):   # train.py:26-60
        def __init__(self, beta, S, A):
            super().__init__()
            self.fc1, self.fc2 = nn.Linear(S + A, 256), nn.Linear(256, 256)
            self.action_value, self.q = nn.Linear(A, 256), nn.Linear(256, 1)
            self.optimizer = torch.optim.Adam(self.parameters(), lr=beta)

        def forward(self, s, a):
            return self.q(func.relu(self.fc2(func.relu(self.fc1(torch.cat([s, a], 1))))))

    class Actor(nn.Module):    # train.py:63-100
        def __init__(self, alpha, S, A, lo, hi):
            super().__init__()
            self.a_min, self.a_max = torch.tensor(lo, dtype=torch.float), torch.tensor(hi, dtype=torch.float)
            self.off = (self.a_min + self.a_max) / 2.0
            self.gain = self.a_max - self.off
            self.fc1, self.fc2, self.mu = nn.Linear(S, 256), nn.Linear(256, 256), nn.Linear(256, A)
            self.optimizer = torch.optim.Adam(self.parameters(), lr=alpha)

        def forward(self, s):
            return self.gain * torch.tanh(self.mu(func.relu(self.fc2(func.relu(self.fc1(s)))))) + self.off

    torch.manual_seed(seed)
    env = SecondOrderIntegration(n_envs=n, variant="ddpg", seed=seed, env_id0=rank * n)
    env.reset(random=True)
    lo, hi = env.action_range[:, 0], env.action_range[:, 1]
    msg = {'state_dim': 4, 'action_dim': 2, 'action_range': env.action_range, 'name': env.name}
    out = {}
    for native in (True, False):
        torch.manual_seed(seed)
        nets = [Actor(1e-4, 4, 2, lo, hi), Actor(1e-4, 4, 2, lo, hi), Critic(3e-4, 4, 2),
                Critic(3e-4, 4, 2)]
        agent = DDPG(msg, 0.99, 0.005, 0.005, capacity, batch, *nets, device="cuda", seed=seed,
                     graph=True, native=native)
        assert (agent._native is not None) == native
        loop = VecDDPG(env, agent, learn_iters=1)
        for learn in ((False, True) if native else (True,)):
            for _ in range(warmup):
                loop.step(learn=learn)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                loop.step(learn=learn)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            key = "env_only" if not learn else "with_learn" if native else "with_learn_torch_update"
            out[key] = n * steps / dt
        if native:   # the update alone: one captured learn() (gather + rlp_ddpg_update + refresh)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(steps):
                agent.learn(is_reward_ascent=False)
            ev[1].record()
            torch.cuda.synchronize()
            out["learn_ms"] = ev[0].elapsed_time(ev[1]) / steps
    def make_loop(b, iters):
        torch.manual_seed(seed)
        nets = [Actor(1e-4, 4, 2, lo, hi), Actor(1e-4, 4, 2, lo, hi), Critic(3e-4, 4, 2),
                Critic(3e-4, 4, 2)]
        ag = DDPG(msg, 0.99, 0.005, 0.005, capacity, b, *nets, device="cuda", seed=seed,
                  graph=True, native=True)
        return VecDDPG(env, ag, learn_iters=iters), ag
    reuse = offpolicy_reuse(make_loop, n, 64, ddpg_learn_flops()) if reuse_legs else []
    return {"value": out["with_learn"], "unit": "env-steps/s", "env_only": out["env_only"],
            "with_learn_torch_update": out["with_learn_torch_update"], "learn_ms": out["learn_ms"],
            "learn_roofline": learn_roofline(ddpg_learn_flops(), batch, out["learn_ms"]),
            "reference_reuse": reuse,
            "envs_per_gpu": n, "replay_capacity": capacity, "batch": batch, "learn_iters_per_step": 1,
            "update_to_data": {"sampled_rows_per_transition": batch / n, "reference": 64,
                               "reference_basis": "DDPG-4-SecondOrderIntegration/train.py:180,237: "
                                                  "one 64-row learn() per env step",
                               "ratio_vs_reference": batch / n / 64,
                               "note": "throughput at a lower sample reuse than the reference driver"},
            "config": "SecondOrderIntegration (DDPG copy) DDPG, replay in HBM, nets [4,256,256,2] "
                      "relu / Q [6,256,256,1] relu; native DDPG update (rlp_ddpg_update, f32 MFMA) "
                      "in one HIP graph per learn(); with_learn_torch_update = the same loop with "
                      "the reference's torch update"}


def ugvoa_leg(rank, n=16384, steps=30, warmup=3, seed=5):
    """SURVEY §8(f) f3 / BASELINE config 5 shard: UGVForwardObstacleAvoidance (env-dir copy) env
    steps at n envs per GPU (131 072 / 8): f64 RK4 + the 37-beam fake lidar against the env's
    obstacles + reward/terminal + auto-reset of finished envs (map generator on the GPU), actions
    uniform over the action box. One lidar scan per env-step (obs_cur of a step is the previous
    obs_next, as in the drivers)."""
    from reinforcementlearningplatform_amd.environment.UGVForwardObstacleAvoidance import \
        UGVForwardObstacleAvoidance
    env = UGVForwardObstacleAvoidance(n_envs=n, seed=seed, env_id0=rank * n)
    kind, p = env.KIND, env.params
    lo = torch.tensor(env.action_range[:, 0], device="cuda", dtype=torch.float32)
    hi = torch.tensor(env.action_range[:, 1], device="cuda", dtype=torch.float32)
    g = torch.Generator(device="cuda").manual_seed(seed)
    acts = [lo + (hi - lo) * torch.rand(n, 2, device="cuda", generator=g) for _ in range(8)]
    counter = [1]

    def one(i, ev=None):
        if ev is not None:
            ev[0].record()
        _, on, r, f, d = K.env_step(kind, p, env.state, acts[i % 8], want_obs_cur=False)
        if ev is not None:
            ev[1].record()
        K.env_reset(kind, p, env.state, mask=d, seed=seed, counter=counter[0], env_id0=rank * n)
        counter[0] += 1
        return d

    dsum = torch.zeros((), device="cuda", dtype=torch.int64)
    for i in range(warmup):   # (also loads torch's reduction kernels before the timed region)
        dsum += one(i).sum()
    torch.cuda.synchronize()
    dsum.zero_()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        dsum += one(i, evs[i]).sum()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    step_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    return {"value": n * steps / dt, "unit": "env-steps/s", "envs_per_gpu": n,
            "env_step_kernel_ms": step_ms, "resets_per_step": float(dsum) / steps,
            "config": "UGVForwardObstacleAvoidance env-dir copy: f64 RK4 + 37-beam lidar vs 10 "
                      "circles + GPU map generator on reset, random actions"}


def ugvoa_ppo2_leg(rank, n=16384, T=64, iters=3, seed=17):
    """UGVForwardObstacleAvoidance PPO2 rollout (the PPO2 demo's 41 -> 256 -> 256 -> 2 / -> 1 tanh
    nets, demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/train.py:48-50,95-97) through
    rlp_rollout: two launches per step (round 6: oa_policy2_kernel — actor + critic with layer 1
    on 11 K-steps of exact f32 MFMA and the 256 x 256 hidden layer on the f16x3 split, the Philox
    sample — and oa_step_kernel<64> — the lidar env step, the 37-beam scans and the map-generator
    resets of the ended envs), or one launch per segment under RLP_OA_ONE_LAUNCH=1
    (oa_rollout_kernel, opt-in: DESIGN.md §4 round 6); n envs per GPU (config 5: 131 072 / 8)."""
    one_launch = os.environ.get("RLP_OA_ONE_LAUNCH", "") == "1"
    kind = A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE
    p = A.default_params(kind, "ppo2")
    D, S, Ad = A.ENV_DIMS[kind]
    ad = A.MLPDesc.make([S, 256, 256, Ad], [A.RLP_ACT_TANH] * 3)
    cd = A.MLPDesc.make([S, 256, 256, 1], [A.RLP_ACT_TANH, A.RLP_ACT_TANH, A.RLP_ACT_NONE])
    apk = K.mfma_pack(ad, orthogonal_params(ad, [1.0, 1.0, 0.01], seed).cuda())
    cpk = K.mfma_pack(cd, orthogonal_params(cd, [1.0, 1.0, 1.0], seed + 1).cuda())
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 6 for l, h in zip(lo, hi)]
    st = K.new_state(kind, n)
    need = torch.ones(n, dtype=torch.uint8, device="cuda")
    bufs = K.rollout_buffers(kind, T, n)
    step0 = [0]
    ws = [None]   # the lidar path's scratch, allocated once (rlp_rollout_workspace_bytes)

    def seg():
        cfg = K.make_rollout_cfg(T, n, seed, step0[0], rank * n, std, lo, hi,
                                 A.RLP_SUCCESS_DONE_AND_FLAG_NE, A.timeout_flag(kind))
        ws[0] = K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs, workspace=ws[0])
        step0[0] += T
    seg()
    torch.cuda.synchronize()
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(iters)]
    t0 = time.perf_counter()
    for i in range(iters):
        evs[i][0].record()
        seg()
        evs[i][1].record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    seg_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    rows = n * T + n   # actor + critic per env-step, the bootstrap critic per env
    flop = n * T * (mlp_flops(ad) + mlp_flops(cd)) + n * mlp_flops(cd)
    hid = 2 * 256 * 256                     # the hidden layer's FLOP per row and net
    f_hidden = (2 * n * T + n) * hid        # on the f16x3 split (the default arithmetic)
    f_exact = flop - f_hidden               # layers 1 and 3: exact f32 MFMA / VALU
    ideal_s = (f_exact / PEAK_FP32_MFMA_TFLOPS + f_hidden / PEAK_F16X3_TFLOPS) / 1e12
    peak_mixed = flop / ideal_s / 1e12      # the FLOP-weighted ceiling of that arithmetic mix
    ach = flop / (seg_ms * 1e-3) / 1e12
    return {"value": n * T * iters / dt, "unit": "env-steps/s", "envs_per_gpu": n, "T": T,
            "ms_per_segment": dt / iters * 1e3, "episodes_per_segment": int(bufs["done"].sum()),
            "roofline": {"bound": "mfma", "achieved": ach, "peak": peak_mixed,
                         "unit": "TFLOP/s", "frac": ach / peak_mixed,
                         "flop_per_segment": flop, "segment_ms": seg_ms, "rows": rows,
                         "peak_basis": "mixed: layers 1 and 3 (%.3g FLOP) at the f32 MFMA peak "
                                       "%.1f TF, the hidden layer (%.3g FLOP) at the f16x3 ceiling "
                                       "%.1f TF" % (f_exact, PEAK_FP32_MFMA_TFLOPS, f_hidden,
                                                    PEAK_F16X3_TFLOPS),
                         "frac_vs_f32_peak": ach / PEAK_FP32_MFMA_TFLOPS,
                         "kernel": ("rlp::oa_rollout_kernel(rlp::OaSegArgs const*)" if one_launch
                                    else "rlp::oa_policy2_kernel + rlp::oa_step_kernel<64> per step"),
                         "note": "whole segment (the segment-start reset and observation, the T "
                                 "steps + the bootstrap critic), the lidar env's f64 work "
                                 "included, against the nets' FLOPs"},
            "config": "UGVForwardObstacleAvoidance (PPO2 copy, 37-beam lidar, 10 circles) PPO2 "
                      "rollout, nets [41,256,256,2] / [41,256,256,1] tanh (rlp_rollout)"}


def ugvoa_sac_leg(rank, n=16384, steps=20, warmup=3, batch=4096, capacity=1 << 20, seed=13,
                  reuse_legs=True):
    """BASELINE config 5 shard: UGVForwardObstacleAvoidance SAC, n envs per GPU (131 072 / 8),
    replay in HBM. One step = actor trunk + squashed-Gaussian sample (librlp) + env step with the
    lidar kernel + n transitions into the replay ring + auto-reset (GPU map generator), then one
    SAC update on `batch` rows sampled from HBM (the driver's learn() per env step, batch scaled
    from 256). Nets: the SAC demo drivers' SACActor [41,128,64,2+2] / twin SACCritic [43,128,64,1]."""
    from reinforcementlearningplatform_amd.algorithm.actor_critic.Soft_Actor_Critic import SAC
    from reinforcementlearningplatform_amd.algorithm.actor_critic.vec_sac import VecSAC
    from reinforcementlearningplatform_amd.environment.UGVForwardObstacleAvoidance import \
        UGVForwardObstacleAvoidance
    from reinforcementlearningplatform_amd.utils.classes import SACActor, SACCritic
    torch.manual_seed(seed)
    env = UGVForwardObstacleAvoidance(n_envs=n, seed=seed, env_id0=rank * n)
    S, Ad = env.state_dim, env.action_dim
    lo, hi = env.action_range[:, 0], env.action_range[:, 1]
    msg = {'state_dim': S, 'action_dim': Ad, 'action_range': env.action_range, 'name': env.name}
    out = {}
    for native in (True, False):
        torch.manual_seed(seed)
        agent = SAC(msg, 0.99, 0.005, capacity, batch,
                    SACActor(S, Ad, lo, hi, std_min=0.05, std_scale=1.), SACCritic(S, Ad),
                    SACCritic(S, Ad), 1e-4, 1e-4, 1e-4, True, device="cuda", seed=seed, graph=True,
                    native=native)
        assert (agent._native is not None) == native
        loop = VecSAC(env, agent)
        for learn in ((False, True) if native else (True,)):
            for _ in range(warmup):
                loop.step(learn=learn)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                loop.step(learn=learn)
            torch.cuda.synchronize()
            key = "env_only" if not learn else "with_learn" if native else "with_learn_torch_update"
            out[key] = n * steps / (time.perf_counter() - t0)
        if native:   # the update alone: one captured learn()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(steps):
                agent.learn()
            ev[1].record()
            torch.cuda.synchronize()
            out["learn_ms"] = ev[0].elapsed_time(ev[1]) / steps
    def make_loop(b, iters):
        torch.manual_seed(seed)
        ag = SAC(msg, 0.99, 0.005, capacity, b,
                 SACActor(S, Ad, lo, hi, std_min=0.05, std_scale=1.), SACCritic(S, Ad),
                 SACCritic(S, Ad), 1e-4, 1e-4, 1e-4, True, device="cuda", seed=seed, graph=True,
                 native=True)
        return VecSAC(env, ag, learn_iters=iters), ag
    reuse = offpolicy_reuse(make_loop, n, 256, sac_learn_flops(S, Ad)) if reuse_legs else []
    return {"value": out["with_learn"], "unit": "env-steps/s", "env_only": out["env_only"],
            "with_learn_torch_update": out["with_learn_torch_update"], "learn_ms": out["learn_ms"],
            "learn_roofline": learn_roofline(sac_learn_flops(S, Ad), batch, out["learn_ms"]),
            "reference_reuse": reuse,
            "envs_per_gpu": n, "replay_capacity": capacity, "batch": batch,
            "learn_iters_per_step": 1,
            "update_to_data": {"sampled_rows_per_transition": batch / n, "reference": 256,
                               "reference_basis": "SAC-4-UGVForward/train.py:206,263: one 256-row "
                                                  "learn() per env step",
                               "ratio_vs_reference": batch / n / 256,
                               "note": "throughput at a lower sample reuse than the reference driver"},
            "config": "UGVForwardObstacleAvoidance (env-dir copy, 37-beam lidar, 10 circles) SAC, "
                      "replay in HBM, demo nets; native SAC update (rlp_sac_update, f32 MFMA) in one "
                      "HIP graph per learn() (sample, gather, update, actor refresh); "
                      "with_learn_torch_update = the same loop with the reference's torch update"}


def hbm_legs(seg, n_env=1 << 22, iters=10, warmup=2):
    """BASELINE.md §3 / SURVEY §8(d): the HBM-bound kernels priced against the HBM roof (8 TB/s),
    with algorithmic bytes per launch (the minimal reads + writes of the kernel's contract):
      gae_kernel           r, V, V' f32 + done, success u8 read; adv, v_target f32 written
      reward_norm          stats pass reads r; apply reads r and writes the normalised reward
      adv_normalize        reads and writes adv
      env_step_kernel<K>   f64 state read (D) and written (DW, the components step() changes) +
                           f32 action read; f32 obs_next, f64 reward, i32 flag, u8 done written
    GAE / normaliser on the bench segment (n x T); env steps at n_env envs (SOI, UGV, UAV kinds)."""
    out = {}

    def timed(fn):
        for _ in range(warmup):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(iters)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in ev]))

    def put(name, kernel, nbytes, ms, extra=None):
        gbs = nbytes / (ms * 1e-3) / 1e9
        # "effective": algorithmic bytes / time. Part of a small kernel's reads can come from the
        # L2 / Infinity Cache (PMC HBM bytes below the algorithmic ones), so this is not HBM
        # utilisation; hbm_frac_pmc beside it prices the PMC-measured HBM bytes instead
        out[name] = dict({"kernel": kernel, "bytes_per_launch": int(nbytes), "avg_launch_ms": ms,
                          "bandwidth": "effective", "achieved": gbs, "peak": PEAK_HBM_GBS,
                          "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS}, **(extra or {}))

    b, smp = seg.bufs, seg.n * seg.T
    rms = torch.zeros(4, dtype=torch.float64, device="cuda")
    # the learn side's calls (Segment.learn_side), each priced alone
    ms = timed(lambda: K.reward_norm_statistics(b["reward"], rms, seg.work))
    put("reward_norm", "rlp::reward_stats_kernel<true> + rlp::reward_merge_kernel", smp * 4, ms,
        {"samples": smp, "note": "the running statistics (chunk statistics, then one block: the "
                                 "per-step merges and the scan); the rewards are normalised inside "
                                 "gae_kernel's load"})
    ms = timed(lambda: K.gae_normalized(b["reward"], seg.work, b["value"], b["value_next"],
                                        b["done"], b["success"], 0.999, 0.95, adv=seg.adv,
                                        v_target=seg.vt, stats=seg.stats))
    put("gae", "rlp::gae_kernel<1>", smp * (3 * 4 + 2 + 2 * 4), ms,
        {"samples": smp, "note": "the raw reward normalised on load"})
    ms = timed(lambda: K.adv_normalize(seg.adv, seg.stats))
    put("adv_normalize", "rlp::adv_stats_merge_kernel + rlp::adv_norm_kernel<true>", smp * 8, ms,
        {"samples": smp})
    # the form that stores the normalised rewards (rlp_reward_norm: statistics + apply), which
    # GAE then re-reads — the learn side before round 6
    ms = timed(lambda: K.reward_norm(b["reward"], rms, seg.work, out=seg.rnorm))
    put("reward_norm_stored",
        "rlp::reward_stats_kernel<true> + rlp::reward_merge_kernel + rlp::reward_apply_kernel<true>",
        smp * 12, ms, {"samples": smp})
    for env, kind, pf, dw in (("soi", A.RLP_ENV_SOI, lambda: A.soi_params("env"), 5),
                              ("ugv", A.RLP_ENV_UGV_FORWARD,
                               lambda: A.ugv_params(A.RLP_ENV_UGV_FORWARD, "ppo2"), 6),
                              ("uav", A.RLP_ENV_UAV_HOVER_OUTER_LOOP, A.uav_hover_params, 22)):
        D, S, Ad = A.ENV_DIMS[kind]
        p = pf()
        st = K.new_state(kind, n_env)
        K.env_reset(kind, p, st, seed=7, counter=1)
        lo, hi = A.action_bounds(kind, p)
        g = torch.Generator(device="cuda").manual_seed(3)
        act = (torch.tensor(lo, device="cuda") + (torch.tensor(hi, device="cuda") - torch.tensor(lo, device="cuda"))
               * torch.rand(n_env, Ad, device="cuda", generator=g)).float().contiguous()
        on = torch.empty((n_env, S), dtype=torch.float32, device="cuda")
        r = torch.empty(n_env, dtype=torch.float64, device="cuda")
        f = torch.empty(n_env, dtype=torch.int32, device="cuda")
        d = torch.empty(n_env, dtype=torch.uint8, device="cuda")
        lib = _native.lib()

        def step():
            K.check(lib.rlp_env_step(kind, K.C.byref(p), K.ptr(st), n_env, K.ptr(act), None,
                                     K.ptr(on), K.ptr(r), K.ptr(f), K.ptr(d), K.stream_ptr()),
                    "rlp_env_step")
        ms = timed(step)
        nbytes = n_env * (D * 8 + Ad * 4 + dw * 8 + S * 4 + 8 + 4 + 1)
        put(f"env_step_{env}", f"rlp::env_step_kernel<{kind}>", nbytes, ms, {"envs": n_env})
        del st, act, on, r, f, d
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(env, seconds=10.0):
    """Oracle (plain-C port of the reference driver loop: actor + critic forward, sampling and env
    step per env-step) on a bounded sample of the same workload, timed on 1 host thread and on
    P threads (OpenMP over independent envs; P = OMP_NUM_THREADS or the process's CPU set — the
    DPPO-style fan-out of BASELINE.md §3). `value`/`cores` are the P-thread run."""
    from oracle import oracle
    kind, pf, tflag = ENVS[env]
    p = pf()
    D, S, Ad = A.ENV_DIMS[kind]
    ad = A.MLPDesc.make([S, 256, 256, Ad], [1, 1, 1])
    cd = A.MLPDesc.make([S, 256, 256, 1], [1, 1, 0])
    ap = orthogonal_params(ad, [1.0, 1.0, 0.01], 1).numpy()
    cp = orthogonal_params(cd, [1.0, 1.0, 1.0], 2).numpy()
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 6 for l, h in zip(lo, hi)]

    def run(n, T):
        cfg = K.make_rollout_cfg(T, n, 3407, 0, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE, tflag)
        st = np.zeros((D, n))
        need = np.ones(n, np.uint8)
        t0 = time.perf_counter()
        oracle.rollout(kind, p, st, need, ad, ap, cd, cp, cfg, want_buffers=True)
        return time.perf_counter() - t0

    def sample(threads, secs):
        oracle.set_threads(threads)
        dt = run(16 * threads, 8)
        T = 64
        n = max(16 * threads, int(16 * threads * 8 * secs / max(dt, 1e-6) / T))
        dt = run(n, T)
        return n * T / dt, n, T, dt

    def env_only(threads, secs):   # the env step alone, random actions
        oracle.set_threads(threads)
        n = 4096 * threads
        st = np.zeros((D, n))
        oracle.env_reset(kind, p, st, seed=3, counter=1)
        act = np.random.default_rng(0).uniform(lo, hi, (n, Ad)).astype(np.float32)
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.env_step(kind, p, st, act, want_obs_cur=False)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= secs:
                return n * reps / dt, n * reps, dt

    def learn(threads, B=1000, K=30):
        """the PPO2-CartPole driver's update (K=30 full-batch epochs on its
        1000-row buffer, Proximal_Policy_Optimization2.py:102-163) with the reference's own
        arithmetic: torch-autograd + Adam on the CPU (vec_ppo2.PPO2Learner, pinned to the
        reference's learn() by tests/test_learn_golden.py)."""
        from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import (
            DEFAULT_PPO_MSG, PPO2Learner)
        from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic
        old = torch.get_num_threads()
        torch.set_num_threads(threads)
        torch.manual_seed(0)
        actor = PPOActor_Gaussian(S, Ad, np.array(lo), np.array(hi), init_std=std[0])
        lrn = PPO2Learner(actor, PPOCritic(S), dict(DEFAULT_PPO_MSG, K_epochs=K), device="cpu")
        g = torch.Generator().manual_seed(1)
        x = [torch.randn(B, S, generator=g), torch.randn(B, Ad, generator=g),
             -torch.rand(B, Ad, generator=g), torch.randn(B, 1, generator=g),
             torch.randn(B, 1, generator=g)]
        lrn.update(*x)   # warm-up
        t0 = time.perf_counter()
        lrn.update(*x)
        dt = time.perf_counter() - t0
        torch.set_num_threads(old)
        return B / dt, dt

    P = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    v1, n1, T1, dt1 = sample(1, seconds / 2)
    vp, n_p, Tp, dtp = sample(P, seconds / 2)
    e1, en1, edt1 = env_only(1, 1.5)
    ep, enp, edtp = env_only(P, 1.5)
    l1, ldt1 = learn(1)
    lp, ldtp = learn(P)
    oracle.set_threads(P)
    return {"value": vp, "unit": "env-steps/s", "cores": P, "kind": "port",
            "cpu_model": _cpu_model(), "cpus_visible": os.cpu_count(),
            "cores_note": "the GPU box grants one GPU's job 16 host CPUs (OMP_NUM_THREADS=16); the "
                          "other visible CPUs serve the other GPUs' jobs",
            "single_thread": {"value": v1, "cores": 1, "env_steps": n1 * T1, "seconds": dt1},
            "sample": f"oracle/rlp_oracle.c rollout (actor+critic 256x256 fp32 MLP with double "
                      f"accumulation, Philox sample, f64 RK4 {env} step): {n_p} envs x {Tp} steps = "
                      f"{n_p * Tp} env-steps in {dtp:.1f} s on {P} host threads (OpenMP over envs); "
                      f"1 thread: {n1} x {T1} in {dt1:.1f} s",
            "env_only": {"value": ep, "unit": "env-steps/s", "cores": P,
                         "single_thread": e1, "env_steps": enp, "seconds": edtp,
                         "sample": f"oracle env_step ({env}, f64 RK4, uniform actions): "
                                   f"{4096 * P} envs x repeats on {P} threads, {4096} on 1"},
            "learn": {"value": lp, "unit": "rows/s (K=30 epochs each)", "cores": P,
                      "single_thread": l1, "seconds": ldtp, "single_thread_seconds": ldt1,
                      "sample": "torch CPU autograd + Adam (the reference's learn() arithmetic), "
                                "K=30 full-batch epochs on a 1000-row buffer, [S,256,256,A] nets"},
            "e2e": {"value": 1.0 / (1.0 / vp + 1.0 / lp), "unit": "env-steps/s", "cores": P,
                    "single_thread": 1.0 / (1.0 / v1 + 1.0 / l1),
                    "note": "rollout + K=30 update per collected row (the PPO2-CartPole driver's "
                            "learn() after each 1000-row buffer)"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each); default WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--env", default="cartpole", choices=sorted(ENVS))
    ap.add_argument("--envs-per-gpu", type=int, default=65536)
    ap.add_argument("--T", type=int, default=128, help="rollout segment length (steps per env)")
    ap.add_argument("--sub", type=int, default=0, help="16-env sub-blocks per wave (2|4; 0=lib default)")
    ap.add_argument("--seed", type=int, default=3407)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--e2e", type=int, default=2, help="PPO2 iterations incl. the K-epoch update to time (0: skip)")
    ap.add_argument("--e2e-k30", type=int, default=1, help="also time e2e at the PPO2 demo's K=30")
    ap.add_argument("--demo-e2e", type=int, default=1, help="also time whole PPO2 iterations of the "
                    "SOI (4-128-64-32) and UGV-OA (41-256-256) demo nets (dense native update)")
    ap.add_argument("--uav", type=int, default=1, help="also time the UavRobust rollout (32768 envs/GPU)")
    ap.add_argument("--fp32-leg", type=int, default=1, help="also time the exact-f32 MLP path")
    ap.add_argument("--ddpg", type=int, default=1, help="also time SOI DDPG with the HBM replay (config 3)")
    ap.add_argument("--oa", type=int, default=1, help="also time UGVForwardObstacleAvoidance env steps (lidar)")
    ap.add_argument("--sac", type=int, default=1, help="also time UGVForwardObstacleAvoidance SAC (config 5 shard)")
    ap.add_argument("--offpolicy-steps", type=int, default=20,
                    help="timed vector steps of the DDPG / SAC legs (short runs for counter passes)")
    ap.add_argument("--physics", default="auto", choices=list(PHYSICS_MODES),
                    help="rollout kernel: env state in LDS + full-lane physics waves (two 4-wave "
                         "blocks per CU, one 8-wave block per CU, or one 4-wave block per CU; auto: "
                         "cu when the envs fill every CU, else cu4), or per-wave registers")
    ap.add_argument("--uav-envs", type=int, default=32768, help="UavRobust leg's envs per GPU (config 4: 262144 / 8)")
    ap.add_argument("--uav-physics", default=None, choices=list(PHYSICS_MODES),
                    help="rollout kernel of the UavRobust leg (default: --physics)")
    ap.add_argument("--hbm", type=int, default=1, help="also time the HBM-bound kernels (GAE, reward / "
                    "advantage normalisation, SOI / UGV / UAV env steps) against the HBM roof")
    ap.add_argument("--learner", default="native", choices=["native", "torch"],
                    help="e2e leg's K-epoch update: librlp kernels or torch autograd + Adam")
    ap.add_argument("--precision", default="f16x3", choices=["f16x3", "fp32"],
                    help="rollout hidden-layer arithmetic (include/rlp.h rlp_set_mlp_precision)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch with torchrun "
                 f"--nproc-per-node {args.gpus}, or without WORLD_SIZE set so bench.py starts the "
                 f"ranks itself)")
    # one process per GPU; RLP_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks folded
    # onto the visible devices) — the driver's runs use RCCL ("nccl") with one GPU per rank
    backend = os.environ.get("RLP_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()   # counting devices does not initialise HIP
    if world > 1 and backend == "nccl" and ndev < world:
        sys.exit(f"bench.py: --gpus {world} needs {world} visible GPUs, this node has {ndev} "
                 f"(RLP_BENCH_BACKEND=gloo folds the ranks onto the visible GPUs for a rehearsal)")
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if args.sub:
        _native.set_rollout_sub(args.sub)
    _native.set_rollout_physics(PHYSICS_MODES[args.physics])
    prec = _native.MLP_F16X3 if args.precision == "f16x3" else _native.MLP_FP32
    _native.set_mlp_precision(prec)

    n, T = args.envs_per_gpu, args.T
    seg = Segment(args.env, n, T, args.seed, env_id0=rank * n)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(steps):
        barrier()
        t0 = time.perf_counter()
        ev = []
        for _ in range(steps):
            # HIP events on the stream the rollout kernel is launched on (torch's current stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            seg.rollout()
            e1.record()
            seg.learn_side()
            ev.append((e0, e1))
        barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, float(np.mean([a.elapsed_time(b) for a, b in ev]))

    for _ in range(args.warmup):
        seg.iteration()
    elapsed, rollout_ms = timed(args.steps)

    env_steps = n * T * world * args.steps
    value = env_steps / elapsed
    flop_launch = n * T * (mlp_flops(seg.ad) + mlp_flops(seg.cd)) + n * mlp_flops(seg.cd)
    achieved = flop_launch / (rollout_ms * 1e-3) / 1e12
    if prec == _native.MLP_F16X3:
        peak, basis = PEAK_F16X3_TFLOPS, ("f16 dense MFMA %.1f TF / 3 (f16x3 split: 3 f16 MFMAs per "
                                          "fp32-equivalent product)" % PEAK_F16_MFMA_TFLOPS)
        dtype, mlp = "fp32 (f16x3 split MFMA)", "f16x3 split MFMA, f32 accumulate (fp32-class error)"
    else:
        peak, basis = PEAK_FP32_MFMA_TFLOPS, "f32 MFMA dense (v_mfma_f32_16x16x4_f32)"
        dtype, mlp = "fp32", "fp32 MFMA (exact f32)"
    out = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
        "data": "synthetic",
        "config": {"workload": f"{args.env}_ppo2_rollout", "envs_per_gpu": n, "global_envs": n * world,
                   "T": T, "env_steps_per_iteration": n * T * world,
                   "nets": "actor [S,256,256,A] tanh, critic [S,256,256,1]",
                   "parallelism": f"dp{world} (env shards, no data-path collective)",
                   "physics": "f64", "mlp": mlp},
        "roofline": {"bound": "mfma", "kernel": (rollout_kernel_name(args.physics, n, args.env, args.sub) if args.precision == "f16x3"
                                                else "rlp::rollout_kernel<KIND,256,SUB,false>"), "achieved": achieved,
                     "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
                     "traffic_source": TRAFFIC_SOURCE,
                     "peak_basis": basis, "avg_launch_ms": rollout_ms, "flop_per_launch": flop_launch},
    }
    if prec == _native.MLP_F16X3 and args.fp32_leg:
        # the exact-f32 MFMA path on the same workload, for reference (include/rlp.h)
        _native.set_mlp_precision(_native.MLP_FP32)
        seg.iteration()
        el32, ms32 = timed(max(2, args.steps // 2))
        _native.set_mlp_precision(prec)
        ach32 = flop_launch / (ms32 * 1e-3) / 1e12
        out["fp32_mfma_path"] = {"value": n * T * world * max(2, args.steps // 2) / el32,
                                 "unit": "env-steps/s", "avg_launch_ms": ms32, "achieved": ach32,
                                 "peak": PEAK_FP32_MFMA_TFLOPS, "frac": ach32 / PEAK_FP32_MFMA_TFLOPS}
    traffic = pmc_traffic(out["config"]["workload"], n, T, out["roofline"]["kernel"])
    if traffic is not None:
        out["roofline"]["traffic"] = traffic
    if args.uav and args.env == "cartpole":
        un, uT, usteps = args.uav_envs, 64, 5
        uphys = args.uav_physics or args.physics
        _native.set_rollout_physics(PHYSICS_MODES[uphys])
        useg = Segment("uav", un, uT, args.seed + 1, env_id0=rank * un)
        for _ in range(2):
            useg.iteration()
        barrier()
        t1 = time.perf_counter()
        uev = []
        for _ in range(usteps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            useg.rollout()
            e1.record()
            useg.learn_side()
            uev.append((e0, e1))
        barrier()
        uel = time.perf_counter() - t1
        if dist is not None:
            t = torch.tensor([uel], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            uel = float(t.item())
        ums = float(np.mean([a.elapsed_time(b) for a, b in uev]))
        uflop = un * uT * (mlp_flops(useg.ad) + mlp_flops(useg.cd)) + un * mlp_flops(useg.cd)
        uach = uflop / (ums * 1e-3) / 1e12
        upeak = PEAK_F16X3_TFLOPS if prec == _native.MLP_F16X3 else PEAK_FP32_MFMA_TFLOPS
        out["uav_ppo2_rollout"] = {
            "value": un * uT * usteps * world / uel, "unit": "env-steps/s", "envs_per_gpu": un,
            "global_envs": un * world, "T": uT,
            "config": "UavRobust hover outer loop (6-DoF + FNTSMC), PPO2 [6,256,256,3]",
            "roofline": {"bound": "mfma", "kernel": (rollout_kernel_name(uphys, un, "uav", args.sub)
                                                     if args.precision == "f16x3"
                                                     else "rlp::rollout_kernel<KIND,256,SUB,false>"),
                         "achieved": uach, "peak": upeak, "unit": "TFLOP/s", "frac": uach / upeak,
                         "traffic": pmc_traffic("uav_ppo2_rollout", un, uT,
                                                rollout_kernel_name(uphys, un, "uav", args.sub)),
                         "traffic_source": TRAFFIC_SOURCE,
                         "avg_launch_ms": ums, "flop_per_launch": uflop}}
        del useg
        _native.set_rollout_physics(PHYSICS_MODES[args.physics])
    if args.hbm:
        out["hbm_kernels"] = hbm_legs(seg)
        for k, v in out["hbm_kernels"].items():
            v["traffic"] = pmc_kernel_traffic(k, v["kernel"])
            v["hbm_frac_pmc"] = (None if v["traffic"] is None else
                                 v["traffic"] / (v["avg_launch_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS)
    if args.ddpg and args.env == "cartpole":
        d = soi_ddpg_leg(rank, steps=args.offpolicy_steps, warmup=min(3, args.offpolicy_steps))
        if dist is not None:
            t = torch.tensor([d["value"], d["env_only"]], device="cuda", dtype=torch.float64)
            dist.all_reduce(t)   # independent replicas: sum of the ranks' rates
            d["value"], d["env_only"] = float(t[0]), float(t[1])
        out["soi_ddpg"] = d
    if args.oa and args.env == "cartpole":
        d = ugvoa_leg(rank)
        if dist is not None:
            t = torch.tensor([d["value"]], device="cuda", dtype=torch.float64)
            dist.all_reduce(t)
            d["value"] = float(t[0])
        out["ugvoa_lidar"] = d
    if args.oa and args.env == "cartpole":
        d = ugvoa_ppo2_leg(rank)
        if dist is not None:
            t = torch.tensor([d["value"]], device="cuda", dtype=torch.float64)
            dist.all_reduce(t)
            d["value"] = float(t[0])
        out["ugvoa_ppo2_rollout"] = d
    if args.sac and args.env == "cartpole":
        d = ugvoa_sac_leg(rank, steps=args.offpolicy_steps, warmup=min(3, args.offpolicy_steps))
        if dist is not None:
            t = torch.tensor([d["value"], d["env_only"]], device="cuda", dtype=torch.float64)
            dist.all_reduce(t)   # independent env shards / replicas: sum of the ranks' rates
            d["value"], d["env_only"] = float(t[0]), float(t[1])
        out["ugvoa_sac"] = d
    if args.demo_e2e and args.env == "cartpole":
        for which in ("soi", "ugvoa"):
            d = demo_nets_e2e_leg(rank, which)
            d["value"] *= world
            out[f"{which}_ppo2_e2e"] = d
    if args.e2e and args.env in E2E_ENVS:
        upd = ("librlp rlp_ppo2_grad + rlp_adam_step" if args.learner == "native"
               else "torch autograd + Adam (fp32)")
        v, it_s, info = e2e_iterations(seg, args.e2e, learner=args.learner)
        out["e2e"] = dict({"value": v * world, "unit": "env-steps/s", "s_per_iteration": it_s,
                           "update": f"K=6 full-batch epochs per iteration (DPPO2 drivers' k_epo), {upd}",
                           "note": "VecPPO2 iterations (rollout + value fix-up + reward / advantage "
                                   "normalisation + GAE + PPO update); `value` above is the rollout "
                                   "hot path"}, **info)
        out["e2e"]["rollout_frac"] = flop_launch / (info["rollout_ms"] * 1e-3) / 1e12 / peak
        if args.e2e_k30:
            v30, it30, info30 = e2e_iterations(seg, max(1, args.e2e // 2), k_epochs=30,
                                               learner=args.learner)
            out["e2e"]["k30"] = dict({
                "value": v30 * world, "unit": "env-steps/s", "s_per_iteration": it30,
                "update": f"K=30 full-batch epochs per iteration (PPO2-4-CartPole/train.py:146), {upd}"},
                **info30)
            out["e2e"]["k30"]["rollout_frac"] = (flop_launch / (info30["rollout_ms"] * 1e-3) / 1e12
                                                 / peak)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.env, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
