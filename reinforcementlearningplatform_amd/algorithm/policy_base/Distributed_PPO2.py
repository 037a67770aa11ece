"""Distributed_PPO2 — drop-in for demonstration/DPPO2/*/Distributed_PPO2.py, re-designed for one
node of MI355X: the reference's `num_of_pro` CPU worker processes (each one env, Hogwild updates of
shared-memory global nets, Distributed_PPO2.py:13-172) become one process per GPU, each owning a
shard of n envs stepped by the fused rollout kernel, with synchronous data-parallel PPO2 updates
(gradients averaged by one RCCL all-reduce per optimiser step). Env i of rank r has global id
r * n + i and draws from the Philox stream keyed by that id, so the union of all ranks'
trajectories is the same for any world size.

Launch one process per GPU (torchrun --nproc-per-node N ...); with WORLD_SIZE unset it runs on a
single GPU. The class keeps the reference's surface: constructor (env, actor_lr, critic_lr,
num_of_pro, path), global_actor / global_critic / eval_actor, save_ac, global_evaluate, evaluate,
start_multi_process, DPPO2_info; `Worker` is the per-rank VecPPO2 learner.

Worker semantics follow the DPPO2 demo copy of the env's kind (DPPO2_COPY below, overridable
through ppo_msg): the Worker.learn() update (update_rule 'dppo2': frozen local nets, gradients
accumulated in never-zeroed local buffers and clipped in place, SharedAdam betas (0.9, 0.99)), the
copy's clip norm and success rule, no lr decay (the Worker stores use_lr_decay and never applies
it, Distributed_PPO2.py:50), and the copy's exploration-std schedule after every learn().
"""
import os
import warnings

import numpy as np

import torch

from ... import _abi
from ...utils.classes import PPOActor_Gaussian, PPOCritic
from .vec_ppo2 import VecPPO2

Worker = VecPPO2

# Per-kind DPPO2 demo-copy semantics: clip_grad_norm_ max_norm, the buffer's success rule
# (rlp_success_rule, flag) and the std schedule (kind, period, step, floor):
#   "reset": std = std0 * max(1 - t / period * step, floor), std0 = (a_max - a_min) / 6
#   "scale": std *= max(1 - t / period * step, floor)
# applied when t % period == 0 and t > 0, t = this worker's learn() count.
_CP_SOI = dict(clip=0.2, rule=(_abi.RLP_SUCCESS_FLAG_NE, 1), std=("reset", 250, 0.05, 0.05))
_OTHERS = dict(clip=0.5, rule=(_abi.RLP_SUCCESS_DONE_AND_FLAG_NE, 2), std=("scale", 1000, 0.05, 0.2))
DPPO2_COPY = {
    # demonstration/DPPO2/DPPO2-4-CartPole/Distributed_PPO2.py:88-102 (0.2), :138, :160-165
    _abi.RLP_ENV_CARTPOLE: _CP_SOI,
    # demonstration/DPPO2/DPPO2-4-SecondOrderIntegration/Distributed_PPO2.py: same as CartPole
    _abi.RLP_ENV_SOI: _CP_SOI,
    # demonstration/DPPO2/DPPO2-4-{CartPoleAngleOnly,UGVForward,UGVBidirectional,
    # UGVForwardObstacleAvoidance}/Distributed_PPO2.py:89,100 (0.5), :135-141, :163-168
    _abi.RLP_ENV_CARTPOLE_ANGLEONLY: _OTHERS,
    _abi.RLP_ENV_UGV_FORWARD: _OTHERS,
    _abi.RLP_ENV_UGV_BIDIRECTIONAL: _OTHERS,
    _abi.RLP_ENV_UGV_OBSTACLE_AVOIDANCE: _OTHERS,
    # no DPPO2 copy for the UAV: the PPO2 convention (terminal && flag != 1, the UAV time-out)
    _abi.RLP_ENV_UAV_HOVER_OUTER_LOOP: dict(clip=0.5, rule=(_abi.RLP_SUCCESS_DONE_AND_FLAG_NE, 1),
                                            std=("scale", 1000, 0.05, 0.2)),
}


def dppo2_std_schedule(copy, action_range):
    """The Worker.run() std schedule of a DPPO2 copy as a callable (t_epoch, actor) -> None."""
    kind, period, step, floor = copy["std"]
    ar = np.asarray(action_range, dtype=np.float64)
    std0 = torch.tensor((ar[:, 1] - ar[:, 0]) / 2 / 3, dtype=torch.float)

    def schedule(t, actor):
        if t % period == 0 and t > 0:
            ratio = max(1 - t / period * step, floor)
            if kind == "reset":
                actor.std = (std0 * ratio).to(torch.as_tensor(actor.std).device)
            else:
                actor.std = actor.std * ratio
    return schedule


def init_distributed(backend=None):
    """torch.distributed from the torchrun environment (RCCL on ROCm GPUs, gloo on CPU)."""
    if not torch.distributed.is_available() or int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    if not torch.distributed.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            torch.distributed.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    return torch.distributed.group.WORLD


class Distributed_PPO2:
    def __init__(self, env, actor_lr: float = 3e-4, critic_lr: float = 1e-3, num_of_pro: int = 5,
                 path: str = '', ppo_msg: dict = None, T: int = 128, actor=None, critic=None,
                 seed: int = 3407, eval_env=None, device=None):
        """env: this rank's batched env (a VecEnv with n_envs > 0, built with env_id0 = rank * n).
        num_of_pro is informational: the parallelism is the torch.distributed world size."""
        self.group = init_distributed()
        self.rank = torch.distributed.get_rank() if self.group is not None else 0
        self.world = torch.distributed.get_world_size() if self.group is not None else 1
        self.env = env
        self.eval_env = eval_env
        self.state_dim_nn, self.action_dim_nn = env.state_dim, env.action_dim
        self.action_range = env.action_range
        self.actor_lr, self.critic_lr = actor_lr, critic_lr
        self.num_of_pro = num_of_pro
        self.path = path
        ar = np.array(env.action_range)
        self.global_actor = actor if actor is not None else PPOActor_Gaussian(
            state_dim=env.state_dim, action_dim=env.action_dim, a_min=ar[:, 0], a_max=ar[:, 1],
            init_std=0.8, use_orthogonal_init=True)
        self.global_critic = critic if critic is not None else PPOCritic(
            state_dim=env.state_dim, use_orthogonal_init=True)
        self.eval_actor = self.global_actor
        self.copy = DPPO2_COPY[env.KIND]
        if env.KIND == _abi.RLP_ENV_CARTPOLE_ANGLEONLY and getattr(env, "variant", "dppo2") == "env":
            warnings.warn("Distributed_PPO2: CartPoleAngleOnly(variant='env') is the env-dir file; "
                          "the DPPO2 demos train the demo copy, CartPoleAngleOnly(variant='dppo2')",
                          stacklevel=2)
        msg = dict(ppo_msg or {})
        msg.setdefault('a_lr', actor_lr)
        msg.setdefault('c_lr', critic_lr)
        msg.setdefault('update_rule', 'dppo2')
        msg.setdefault('grad_clip_norm', self.copy["clip"])
        msg.setdefault('adam_betas', (0.9, 0.99))        # SharedAdam (utils/classes.py:677)
        msg.setdefault('use_grad_clip', True)
        self.msg = msg
        self.worker = Worker(env, self.global_actor, self.global_critic, msg, T=T, seed=seed,
                             success_rule=msg.get('success_rule', self.copy["rule"]),
                             process_group=self.group, device=device)
        self.global_actor, self.global_critic = self.worker.actor, self.worker.critic
        self.eval_actor = self.global_actor
        self.global_training_num = 0
        self.training_record = []
        self.evaluate_record = []

    def save_ac(self, msg, path):
        torch.save(self.global_actor.state_dict(), path + 'actor' + msg)
        torch.save(self.global_critic.state_dict(), path + 'critic' + msg)

    def evaluate(self, state):
        return self.worker.gpu_actor(torch.as_tensor(np.asarray(state, np.float32)).view(1, -1)
                                     ).cpu().numpy().flatten()

    def global_evaluate(self, eval_num: int = 10, save: bool = True):
        """Rank 0: checkpoint the global nets and run deterministic test episodes
        (Distributed_PPO2.py:236-269, rendering left out)."""
        if self.rank != 0:
            return []
        if save and self.path:
            temp = self.path + 'trainNum_{}/'.format(self.global_training_num)
            os.makedirs(temp, exist_ok=True)
            self.save_ac(msg='', path=temp)
        rs = []
        if self.eval_env is not None:
            for _ in range(eval_num):
                self.eval_env.reset(True)
                r = 0.0
                while not self.eval_env.is_terminal:
                    self.eval_env.current_state = self.eval_env.next_state.copy()
                    self.eval_env.step_update(self.evaluate(self.eval_env.current_state))
                    r += self.eval_env.reward
                rs.append(r)
        self.evaluate_record.append(rs)
        return rs

    def start_multi_process(self, iterations: int = 1, eval_every: int = 500, std_schedule=None):
        """Run `iterations` synchronous PPO2 iterations on every rank (the reference loops
        forever). After each learn() the exploration std follows the copy's schedule
        (Worker.run :160-165), or std_schedule(t_epoch, actor) if given (False: none). Checkpoint
        + evaluation whenever global_training_num crosses a multiple of eval_every (the reference
        evaluator tests `% 500 == 0` on a counter every worker bumps by one)."""
        if std_schedule is None:
            std_schedule = dppo2_std_schedule(self.copy, self.env.action_range)
        if not hasattr(self, "t_epoch"):
            self.t_epoch = 0
        for _ in range(iterations):
            self.worker.iteration(learn=True)
            before = self.global_training_num
            self.global_training_num += self.world
            self.training_record.append(self.worker.episode_stats())
            if std_schedule:
                std_schedule(self.t_epoch, self.global_actor)
            self.t_epoch += 1
            if eval_every and before // eval_every != self.global_training_num // eval_every:
                self.global_evaluate()
        return self.training_record

    def DPPO2_info(self):
        print('number of process:', self.world)
        print('agent name：', self.env.name)
        print('state_dim:', self.state_dim_nn)
        print('action_dim:', self.action_dim_nn)
        print('action_range:', self.action_range)
