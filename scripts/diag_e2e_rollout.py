"""Why is the CartPole rollout slower inside the PPO2 training loop than back to back?
 Times the same rollout launch (65 536 envs x 128, HIP events on the launch
stream) in five settings, 5 launches each, in this order:
  A  back to back                          (the bench's timed region)
  B  after 0.3 s of an idle GPU            (clock ramp-down)
  C  after a 0.5 s f16 GEMM burst          (power / clock state after heavy MFMA work)
  D  after a K=30 native PPO2 update       (exactly the e2e loop's pattern)
  E  after re-packing perturbed weights    (packed W2 fresh in HBM, not in L2 / MALL)
Run under `rocprofv3 --pmc GRBM_GUI_ACTIVE ...` the rollout dispatches come in the same order,
so the per-dispatch cycle counts separate a clock effect (same cycles, longer time) from a
memory / cache effect (more cycles)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from reinforcementlearningplatform_amd import kernels as K  # noqa: E402
from reinforcementlearningplatform_amd.algorithm.policy_base.native_ppo2 import NativePPO2Learner  # noqa: E402
from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import DEFAULT_PPO_MSG  # noqa: E402
from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic  # noqa: E402


def main():
    torch.cuda.set_device(0)
    seg = bench.Segment("cartpole", 65536, 128, 3407, 0)
    actor = PPOActor_Gaussian(4, 1, np.array([-8.]), np.array([8.]), init_std=seg.std[0])
    critic = PPOCritic(4)
    lrn = NativePPO2Learner(actor, critic, dict(DEFAULT_PPO_MSG, K_epochs=30), device="cuda")
    b = seg.bufs
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.float16)

    def timed_rollout():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        seg.rollout()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    def burst(seconds):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(10):
                a @ a
            torch.cuda.synchronize()

    def update():
        seg.learn_side()
        lrn.update(b["obs"].view(-1, 4), b["action"].view(-1, 1), b["logp"].view(-1, 1),
                   seg.adv.view(-1, 1), seg.vt.view(-1, 1))
        torch.cuda.synchronize()

    def repack():
        seg.actor.add_(1e-7 * torch.randn_like(seg.actor))
        K.mfma_pack(seg.ad, seg.actor, out=seg.apk)
        K.mfma_pack(seg.cd, seg.critic, out=seg.cpk)
        torch.cuda.synchronize()

    for _ in range(3):
        timed_rollout()
    out = {}
    out["A_back_to_back"] = [timed_rollout() for _ in range(5)]
    res = []
    for _ in range(5):
        time.sleep(0.3)
        res.append(timed_rollout())
    out["B_after_idle_0.3s"] = res
    res = []
    for _ in range(5):
        burst(0.5)
        res.append(timed_rollout())
    out["C_after_f16_gemm_burst_0.5s"] = res
    res = []
    for _ in range(5):
        update()
        res.append(timed_rollout())
    out["D_after_k30_update"] = res
    res = []
    for _ in range(5):
        repack()
        res.append(timed_rollout())
    out["E_after_repack"] = res
    res = []
    for _ in range(5):
        update()
        burst(0.05)
        res.append(timed_rollout())
    out["F_after_update_then_50ms_gemm"] = res
    for k, v in out.items():
        print(f"{k:32s} mean {np.mean(v):.3f} ms  {['%.3f' % x for x in v]}")
    print(json.dumps({k: float(np.mean(v)) for k, v in out.items()}))


if __name__ == "__main__":
    main()
