"""Which PPO2 update a net gets (CPU only: the checks are torch forwards on a probe batch, no
kernel runs). librlp's update kernels differentiate tanh hidden layers with the actor head
tanh(z) * gain + off (the CartPole driver's PPOActor_Gaussian, demonstration/PPO2/PPO2-4-CartPole/
train.py:39-76) or the critic's linear head; a net with the right Linear shapes and any other
arithmetic (ReLU hidden layers, a linear actor head) must get the torch learner, and
learner='native' must refuse it instead of applying tanh' to it."""
import pytest
import torch
import torch.nn as nn

from reinforcementlearningplatform_amd.algorithm.policy_base.native_ppo2 import (
    NativePPO2Learner, dense_fits, native_fits)
from reinforcementlearningplatform_amd.utils.classes import PPOActor_Gaussian, PPOCritic

MSG = dict(a_lr=3e-4, c_lr=1e-3, set_adam_eps=True)


class ReluActor(nn.Module):
    def __init__(self, S=4, A=1, head="tanh"):
        super().__init__()
        self.fc1, self.fc2, self.mean_layer = nn.Linear(S, 256), nn.Linear(256, 256), nn.Linear(256, A)
        self.a_min, self.a_max = torch.full((A,), -1.0), torch.full((A,), 1.0)
        self.off = (self.a_min + self.a_max) / 2.0
        self.gain = self.a_max - self.off
        self.std = torch.tensor(0.5)
        self.head = head

    def forward(self, s):
        h = torch.relu(self.fc2(torch.relu(self.fc1(s))))
        z = self.mean_layer(h)
        return torch.tanh(z) * self.gain + self.off if self.head == "tanh" else z


class ReluCritic(nn.Module):
    def __init__(self, S=4):
        super().__init__()
        self.fc1, self.fc2, self.fc3 = nn.Linear(S, 256), nn.Linear(256, 256), nn.Linear(256, 1)

    def forward(self, s):
        return self.fc3(torch.relu(self.fc2(torch.relu(self.fc1(s)))))


class TanhActorLinearHead(ReluActor):
    def forward(self, s):
        return self.mean_layer(torch.tanh(self.fc2(torch.tanh(self.fc1(s)))))


def test_tanh_nets_take_the_f16x3_update():
    actor, critic = PPOActor_Gaussian(4, 1, [-1.0], [1.0]), PPOCritic(4)
    assert native_fits(actor, True) and native_fits(critic, False)


@pytest.mark.parametrize("make,is_actor", [(lambda: ReluActor(), True), (lambda: ReluCritic(), False),
                                           (lambda: TanhActorLinearHead(), True)])
def test_other_arithmetic_is_not_native(make, is_actor):
    m = make()
    assert not native_fits(m, is_actor) and not dense_fits(m, is_actor)


def test_native_learner_refuses_relu_nets():
    with pytest.raises(ValueError, match="Linear/Tanh"):
        NativePPO2Learner(ReluActor(), PPOCritic(4), MSG, device="cpu")
    with pytest.raises(ValueError, match="Linear/Tanh"):
        NativePPO2Learner(PPOActor_Gaussian(4, 1, [-1.0], [1.0]), ReluCritic(), MSG, device="cpu")


class TanhStackActor(nn.Module):  # the PPO2-SOI demo's actor shape (train.py:37-88), any widths
    def __init__(self, widths=(128, 64, 32), S=4, A=2):
        super().__init__()
        dims = (S,) + tuple(widths)
        self.hidden = nn.ModuleList([nn.Linear(dims[i], dims[i + 1]) for i in range(len(widths))])
        self.mean_layer = nn.Linear(dims[-1], A)
        self.a_min, self.a_max = torch.full((A,), -3.0), torch.full((A,), 3.0)
        self.off = (self.a_min + self.a_max) / 2.0
        self.gain = self.a_max - self.off
        self.std = torch.tensor(1.0)

    def forward(self, s):
        for l in self.hidden:
            s = torch.tanh(l(s))
        return torch.tanh(self.mean_layer(s)) * self.gain + self.off


class TanhStackCritic(nn.Module):
    def __init__(self, widths=(64, 64), S=4):
        super().__init__()
        dims = (S,) + tuple(widths)
        self.hidden = nn.ModuleList([nn.Linear(dims[i], dims[i + 1]) for i in range(len(widths))])
        self.out = nn.Linear(dims[-1], 1)

    def forward(self, s):
        for l in self.hidden:
            s = torch.tanh(l(s))
        return self.out(s)


@pytest.mark.parametrize("actor_w,critic_w,fused", [((128, 64, 32), (64, 64), True),
                                                    ((96, 96), (96, 96), False)])
def test_dense_nets_fused_only_for_the_soi_shapes(actor_w, critic_w, fused):
    """rlp_ppo2_dense_grad runs the SOI demo's two shapes as one fused per-row launch
    (rlp_dense.hip ppo2_fused_kind); _Net.fused mirrors that test and the bench labels by it."""
    from reinforcementlearningplatform_amd.algorithm.policy_base.native_ppo2 import _Net
    a, c = _Net(TanhStackActor(actor_w), True, "cpu"), _Net(TanhStackCritic(critic_w), False, "cpu")
    assert a.dense and c.dense and not a.ext and not c.ext
    assert a.fused == fused and c.fused == fused
