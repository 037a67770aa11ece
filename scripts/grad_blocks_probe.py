"""Per-parameter-block error of the native PPO2 gradients against torch float64 (debug aid for
tests/test_gpu_update.py::test_ppo2_grads_vs_torch; not a test). Run on the GPU box."""
import copy
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_update import make_case, torch_grads, split  # noqa: E402
from reinforcementlearningplatform_amd.algorithm.policy_base.native_ppo2 import NativePPO2Learner  # noqa: E402
from reinforcementlearningplatform_amd.algorithm.policy_base.vec_ppo2 import DEFAULT_PPO_MSG  # noqa: E402

for S, A, N in ((4, 1, 3037), (4, 1, 1)):
    msg = dict(DEFAULT_PPO_MSG)
    actor, critic, s, a, lp, adv, vt = make_case(S, A, N, seed=S * 10 + A)
    ga64, gc64, _, _ = torch_grads(actor, critic, s, a, lp, adv, vt, msg, torch.float64)
    ra, rc = copy.deepcopy(actor), copy.deepcopy(critic)
    nl = NativePPO2Learner(actor, critic, msg, device="cuda")
    dev = lambda t: t.cuda().contiguous()
    nl.grads(dev(s), dev(a), dev(lp), dev(adv), dev(vt))
    gan, gcn = nl.net_a.grad.double().cpu(), nl.net_c.grad.double().cpu()
    for name, gn, g64, mod in (("actor", gan, ga64, ra), ("critic", gcn, gc64, rc)):
        for i, (tn, t64) in enumerate(zip(split(gn, mod), split(g64, mod))):
            err = (tn - t64).abs()
            print(f"S{S} N{N} {name} block {i} n={t64.numel()} max|ref| {t64.abs().max():.3e} "
                  f"max err {err.max():.3e} argmax {int(err.argmax())} got {float(tn.flatten()[int(err.argmax())]):.4e} "
                  f"want {float(t64.flatten()[int(err.argmax())]):.4e}")
        if name == "actor":
            w = split(gn, mod)[0].view(256, S)
            r = split(g64, mod)[0].view(256, S)
            print("  dW1 rows 0..3 got", w[:4].numpy().round(5).tolist())
            print("  dW1 rows 0..3 want", r[:4].numpy().round(5).tolist())
            b = split(gn, mod)[1]; rb = split(g64, mod)[1]
            print("  db1[0:8] got", b[:8].numpy().round(5).tolist(), "want", rb[:8].numpy().round(5).tolist())
