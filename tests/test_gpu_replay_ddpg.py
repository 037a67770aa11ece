"""GPU parity of the HBM replay buffer (rlp_replay_*) and the DDPG agent / VecDDPG loop against the
reference ReplayBuffer (utils/classes.py:189-247) and DDPG.learn (algorithm/actor_critic/
DDPG.py:72-109), pinned by tests/golden/replay.npz and ddpg_soi_learn.npz (made by running the
reference, tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as func

from reinforcementlearningplatform_amd import kernels as K
from reinforcementlearningplatform_amd.algorithm.actor_critic.DDPG import DDPG
from reinforcementlearningplatform_amd.algorithm.actor_critic.vec_ddpg import VecDDPG
from reinforcementlearningplatform_amd.environment.SecondOrderIntegration.SecondOrderIntegration \
    import SecondOrderIntegration
from reinforcementlearningplatform_amd.utils.classes import GPUNet, ReplayBuffer

pytestmark = pytest.mark.gpu


def test_replay_store_and_sort_match_reference(golden):
    g = golden("replay")
    for batched in (False, True):
        rb = ReplayBuffer(10, 4, 2, 1, device="cuda", seed=1)
        if batched:   # n = 23 > capacity in one call: only the last 10 can survive, as sequentially
            rb.store_transition(g["s"], g["a"], g["r"], g["s2"], g["d"])
        else:
            for i in range(len(g["r"])):
                rb.store_transition(g["s"][i], g["a"][i], g["r"][i], g["s2"][i], g["d"][i])
        assert rb.mem_counter == int(g["mem_counter"])
        for ours, ref in ((rb.s_mem, g["s_mem"]), (rb.a_mem, g["a_mem"]), (rb.r_mem, g["r_mem"]),
                          (rb._s_mem, g["s2_mem"]), (rb.end_mem, g["end_mem"])):
            np.testing.assert_array_equal(ours.cpu().numpy(), np.asarray(ref, np.float32))
        rb.get_reward_sort()
        np.testing.assert_array_equal(rb.sorted_index.cpu().numpy(), g["sorted_index"])
        # sample_buffer(is_reward_ascent=True): random.sample(sorted_index[-q:], min(q, batch))
        q = int(0.25 * 10)
        idx = rb.sample_index(is_reward_ascent=True).cpu().numpy()
        assert len(idx) == min(q, 4) and set(idx) == set(g["sorted_index"][-q:])


def test_replay_uniform_sampling():
    max_mem, B = 1000, 200_000
    i1 = K.replay_sample_uniform(max_mem, B, seed=5, counter=1).cpu().numpy()
    i2 = K.replay_sample_uniform(max_mem, B, seed=5, counter=1).cpu().numpy()
    i3 = K.replay_sample_uniform(max_mem, B, seed=5, counter=2).cpu().numpy()
    assert i1.min() >= 0 and i1.max() < max_mem
    np.testing.assert_array_equal(i1, i2)
    assert (i1 != i3).mean() > 0.99
    counts = np.bincount(i1, minlength=max_mem)
    exp = B / max_mem
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < max_mem + 6 * np.sqrt(2 * max_mem)     # ~6 sigma of a chi2(999)


def test_replay_reward_top_large():
    cap = 100_000
    rng = np.random.default_rng(0)
    rb = ReplayBuffer(cap, 20_000, 3, 2, device="cuda", seed=3)
    n = 77_777   # partially filled
    r = np.round(rng.normal(size=n), 2)
    rb.store_transition(rng.normal(size=(n, 3)), rng.normal(size=(n, 2)), r,
                        rng.normal(size=(n, 3)), np.zeros(n))
    idx = rb.sample_index(is_reward_ascent=True).cpu().numpy()
    q = int(0.25 * n)
    order = np.argsort(r.astype(np.float32), kind="stable")
    assert len(idx) == min(q, 20_000) and len(set(idx)) == len(idx)
    assert set(idx) <= set(order[-q:])
    s, a, rr, s2, end = rb.sample_buffer(is_reward_ascent=False)
    assert s.shape == (20_000, 3) and a.shape == (20_000, 2) and (end == 1).all()


# the DDPG-SOI driver's nets (demonstration/DDPG/DDPG-4-SecondOrderIntegration/train.py:26-100)
class Critic(nn.Module):
    def __init__(self, beta, state_dim, action_dim):
        super().__init__()
        self.fc1 = nn.Linear(state_dim + action_dim, 256)
        self.fc2 = nn.Linear(256, 256)
        self.action_value = nn.Linear(action_dim, 256)
        self.q = nn.Linear(256, 1)
        self.optimizer = torch.optim.Adam(self.parameters(), lr=beta)

    def forward(self, s, a):
        sav = func.relu(self.fc1(torch.cat([s, a], 1)))
        sav = func.relu(self.fc2(sav))
        return self.q(sav)


class Actor(nn.Module):
    def __init__(self, alpha, state_dim, action_dim, a_min, a_max):
        super().__init__()
        self.a_min = torch.tensor(a_min, dtype=torch.float)
        self.a_max = torch.tensor(a_max, dtype=torch.float)
        self.off = (self.a_min + self.a_max) / 2.0
        self.gain = self.a_max - self.off
        self.fc1 = nn.Linear(state_dim, 256)
        self.fc2 = nn.Linear(256, 256)
        self.mu = nn.Linear(256, action_dim)
        self.optimizer = torch.optim.Adam(self.parameters(), lr=alpha)

    def forward(self, s):
        s = func.relu(self.fc1(s))
        s = func.relu(self.fc2(s))
        return self.gain * torch.tanh(self.mu(s)) + self.off


def load_flat(m, flat):
    off = 0
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.from_numpy(np.asarray(flat[off:off + p.numel()])).view_as(p))
            off += p.numel()


def make_agent(g=None, memory=10000, batch=64, seed=0, graph=False, native="auto"):
    lo, hi = np.array([-3., -3.]), np.array([3., 3.])
    nets = [Actor(1e-4, 4, 2, lo, hi), Actor(1e-4, 4, 2, lo, hi), Critic(3e-4, 4, 2),
            Critic(3e-4, 4, 2)]
    if g is not None:
        for m, k in zip(nets, ("actor", "target_actor", "critic", "target_critic")):
            load_flat(m, g[f"before_{k}"])
    env_msg = {'state_dim': 4, 'action_dim': 2, 'action_range': np.stack([lo, hi], 1),
               'name': 'SecondOrderIntegration'}
    return DDPG(env_msg, gamma=0.99, actor_soft_update=0.005, critic_soft_update=0.005,
                memory_capacity=memory, batch_size=batch, actor=nets[0], target_actor=nets[1],
                critic=nets[2], target_critic=nets[3], device="cuda", seed=seed, graph=graph,
                native=native)


@pytest.mark.parametrize("native", [True, False])
def test_ddpg_update_matches_reference(golden, native):
    """One learn() iteration from the reference's before-weights on its sampled batch: the
    after-weights of all four nets (native rlp_ddpg_update and the torch path)."""
    g = golden("ddpg_soi_learn")
    agent = make_agent(g, native=native)
    assert (agent._native is not None) == native
    dev = lambda k: torch.as_tensor(np.asarray(g[k]), dtype=torch.float32, device="cuda")
    agent.update(dev("s"), dev("a"), dev("r"), dev("s2"), dev("end"))
    for k, m in (("actor", agent.actor), ("target_actor", agent.target_actor),
                 ("critic", agent.critic), ("target_critic", agent.target_critic)):
        got = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        np.testing.assert_allclose(got, g[f"after_{k}"], rtol=1e-5, atol=1e-7, err_msg=k)


def test_batched_actor_and_noise():
    agent = make_agent()
    for n in (40_001, 5000):   # the fused inference chain with two / one 16-row tiles per block
        s = torch.rand(n, 4, device="cuda") * 4 - 2
        a0 = agent.choose_action(s, is_optimal=True)
        with torch.no_grad():
            ref = agent.actor(s)
        torch.testing.assert_close(a0, ref, rtol=1e-5, atol=2e-6)   # ReLU net through librlp
    sig = np.array([0.5, 0.5], np.float32)
    a1 = agent.choose_action(s, sigma=sig)
    z = ((a1 - ref) / 0.5)[(a1.abs() < 2.9).all(1)]             # unclipped rows
    assert abs(float(z.mean())) < 0.05 and abs(float(z.std()) - 1) < 0.05
    assert float(a1.abs().max()) <= 3.0


@pytest.mark.parametrize("graph", [False, True])
def test_vecddpg_loop_fills_replay_and_learns(graph):
    n = 4096
    env = SecondOrderIntegration(n_envs=n, variant="ddpg", seed=2)
    env.reset(random=True)
    agent = make_agent(memory=200_000, batch=512, seed=4, graph=graph)
    loop = VecDDPG(env, agent, learn_iters=1)
    p0 = torch.cat([p.detach().reshape(-1) for p in agent.actor.parameters()]).clone()
    dones = 0
    for t in range(30):
        r, d, out = loop.step()
        dones += int(d.sum())
        assert torch.isfinite(r).all()
    assert agent.memory.mem_counter == 30 * n
    p1 = torch.cat([p.detach().reshape(-1) for p in agent.actor.parameters()])
    assert torch.isfinite(p1).all() and not torch.equal(p0, p1)
    assert out is not None and all(torch.isfinite(x) for x in out)
    # the ring holds what the envs produced: end = 1 - done and obs bounded by the DDPG copy
    m = agent.memory
    assert set(torch.unique(m.end_mem[:30 * n]).tolist()) <= {0.0, 1.0}
    assert float(m.s_mem[:30 * n].abs().max()) < 10


def test_ddpg_graphed_update_is_one_adam_step():
    """graph=True: the captured learn moves every parameter by one Adam step (<= ~lr) from the
    same start as an eager agent, and the GPU actor is refreshed inside the graph."""
    e_agent, g_agent = make_agent(seed=1), make_agent(seed=1, graph=True)
    for m_e, m_g in ((e_agent.actor, g_agent.actor), (e_agent.critic, g_agent.critic),
                     (e_agent.target_actor, g_agent.target_actor),
                     (e_agent.target_critic, g_agent.target_critic)):
        m_g.load_state_dict(m_e.state_dict())
    rng = np.random.default_rng(0)
    n = 5000
    g_agent.memory.store_transition(rng.uniform(-2, 2, (n, 4)), rng.uniform(-3, 3, (n, 2)),
                                    rng.normal(size=n), rng.uniform(-2, 2, (n, 4)),
                                    (rng.uniform(size=n) < 0.1).astype(float))
    g_agent.choose_action(torch.zeros(8, 4, device="cuda"), True)   # builds the GPU actor
    g_agent.learn(is_reward_ascent=False)
    torch.cuda.synchronize()
    for lr, m_e, m_g in ((1e-4, e_agent.actor, g_agent.actor), (3e-4, e_agent.critic, g_agent.critic)):
        pe = torch.cat([p.detach().reshape(-1) for p in m_e.parameters()])
        pg = torch.cat([p.detach().reshape(-1) for p in m_g.parameters()])
        assert torch.isfinite(pg).all() and not torch.equal(pe, pg)
        assert float((pe - pg).abs().max()) <= 1.5 * lr
    # the GPU actor aliases the native update's actor parameters: no copy launch in the graph
    assert g_agent._native is not None
    assert g_agent.gpu_actor.flat.data_ptr() == g_agent._native.nets["actor"].flat.data_ptr()
    flat = g_agent.gpu_actor.flat.clone()
    g_agent.gpu_actor.refresh()
    assert g_agent.gpu_actor.flat.data_ptr() == g_agent._native.nets["actor"].flat.data_ptr()
    torch.testing.assert_close(flat, g_agent.gpu_actor.flat, rtol=0, atol=0)
    for _ in range(5):
        g_agent.learn(is_reward_ascent=False, iter=2)
    assert all(torch.isfinite(p).all() for p in g_agent.actor.parameters())


def _flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def _batch(B, seed):
    rng = np.random.default_rng(seed)
    dev = lambda x: torch.as_tensor(x, dtype=torch.float32, device="cuda")
    return (dev(rng.uniform(-2, 2, (B, 4))), dev(rng.uniform(-3, 3, (B, 2))), dev(rng.normal(size=B)),
            dev(rng.uniform(-2, 2, (B, 4))), dev((rng.uniform(size=B) > 0.1).astype(np.float32)))


def ddpg_f64_grads(before, critic_after, batch, gamma=0.99):
    """DDPG.learn's gradients (DDPG.py:83-104) in float64 on the CPU: `before` = deep copies of
    (actor, target_actor, critic, target_critic) at the step's start; the critic's gradient at the
    before-weights, the actor's through `critic_after` (the critic after its own Adam step)."""
    import copy
    dbl = lambda m: copy.deepcopy(m).cpu().double()
    actor, t_actor, critic, t_critic = (dbl(m) for m in before)
    for m in (actor, t_actor):   # (non-parameter tensors: .cpu() / .double() do not move them)
        m.gain, m.off = m.gain.detach().cpu().double(), m.off.detach().cpu().double()
    s, a, r, s_, end = (x.detach().cpu().double() for x in batch)
    with torch.no_grad():
        target = r.unsqueeze(1) + gamma * end.unsqueeze(1) * t_critic(s_, t_actor(s_))
    func.mse_loss(target, critic(s, a)).backward()
    gc = torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros(p.numel(), dtype=torch.float64)
                    for p in critic.parameters()])
    ca = dbl(critic_after)
    for p in ca.parameters():
        p.requires_grad_(False)
    (-ca(s, actor(s)).mean()).backward()
    ga = torch.cat([p.grad.reshape(-1) for p in actor.parameters()])
    return {"critic": gc.numpy(), "actor": ga.numpy()}


def assert_f32_class(name, native, torch32, truth_n, truth_t, floor_rel=2e-7):
    """|native - f64| <= 4 |torch f32 - f64| + 2e-7 max|g| (each against the float64 gradient of
    the inputs it used): the f32-class bound tests/test_learn_golden.py puts on the PPO2 update."""
    native, torch32 = (np.asarray(x, np.float64) for x in (native, torch32))
    e32 = np.abs(torch32 - truth_t).max()
    en = np.abs(native - truth_n).max()
    floor = floor_rel * np.abs(truth_n).max()
    assert en <= 4 * e32 + floor, (name, en, e32, floor)


ADAM_LR = {"actor": 1e-4, "critic": 3e-4}   # make_agent's Actor / Critic learning rates
ADAM_EPS = 1e-8                              # torch.optim.Adam's default eps (DDPG.py's optimisers)


def assert_adam_tracks(name, native, torch32, gmin, lr, steps, rtol=1e-4, atol=2e-6):
    """Parameters after `steps` Adam steps agree to rtol / atol, except where a gradient sat in
    Adam's eps regime: the step is lr m / (sqrt(v_hat) + eps) with sqrt(v_hat) ~ |g|, so for
    |g| ~ eps it is a steep function of g and two f32 summation orders of a gradient that
    cancels to ~1e-7 of max|g| move the element apart by a fraction of lr (the one element of the
    critic's 68 609 that does so at batch 1000: |g| = 6e-9, steps 0.37 / 0.39 lr). Such elements
    (min over the steps of the torch |g| below 10 eps) may differ by at most 2 lr per step, and
    there may be only a few."""
    d = (native - torch32).abs()
    bad = d > atol + rtol * torch32.abs()
    nbad = int(bad.sum())
    if nbad == 0:
        return
    assert nbad <= max(2, native.numel() // 10000), (name, nbad)
    assert bool((gmin[bad] < 10 * ADAM_EPS).all()), (name, "outside Adam's eps regime",
                                                     gmin[bad].max().item(), d.max().item())
    assert float(d[bad].max()) <= 2 * lr * steps, (name, d.max().item())


@pytest.mark.parametrize("B", [4096, 1000])
def test_native_ddpg_tracks_torch_update(B):
    """rlp_ddpg_update against the torch autograd + Adam path from the same weights over 5
    updates on fresh batches (bench batch 4096, and a batch that is not a multiple of the
    256-row weight-gradient split): per-step losses and all four nets agree to f32 GEMM noise;
    the drivers' unused critic.action_value stays put (no gradient), its target copy is blended."""
    torch.manual_seed(3)
    t_agent, n_agent = make_agent(native=False), make_agent(native=True)
    for k in ("actor", "target_actor", "critic", "target_critic"):
        getattr(n_agent, k).load_state_dict(getattr(t_agent, k).state_dict())
    av0 = n_agent.critic.action_value.weight.detach().clone()
    tav0 = n_agent.target_critic.action_value.weight.detach().clone()
    import copy
    gmin = {}
    for it in range(5):
        batch = _batch(B, it)
        before = [copy.deepcopy(getattr(t_agent, k)) for k in
                  ("actor", "target_actor", "critic", "target_critic")]
        lt = t_agent.update(*batch)
        ln = n_agent.update(*batch)
        for x, y in zip(lt, ln):
            torch.testing.assert_close(y, x, rtol=2e-4, atol=1e-6)
        if it == 0:   # the same start: both gradients against float64, f32-class bound
            tn = ddpg_f64_grads(before, n_agent.critic, batch)
            tt = ddpg_f64_grads(before, t_agent.critic, batch)
        for k in ("critic", "actor"):
            gt = torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros_like(p).reshape(-1)
                            for p in getattr(t_agent, k).parameters()])
            gmin[k] = gt.abs() if it == 0 else torch.minimum(gmin[k], gt.abs())
            if it == 0:
                assert_f32_class(k, n_agent._native.grad[k].cpu(), gt.cpu(), tn[k], tt[k])
    for k in ("actor", "target_actor", "critic", "target_critic"):
        a, b = _flat(getattr(n_agent, k)), _flat(getattr(t_agent, k))
        if k in ADAM_LR:
            assert_adam_tracks(k, a, b, gmin[k], ADAM_LR[k], 5)
        else:
            torch.testing.assert_close(a, b, rtol=1e-4, atol=2e-6, msg=lambda m, k=k: f"{k}: {m}")
    assert torch.equal(n_agent.critic.action_value.weight, av0)
    tav = n_agent.target_critic.action_value.weight
    assert not torch.equal(tav, tav0)
    torch.testing.assert_close(tav, t_agent.target_critic.action_value.weight, rtol=0, atol=1e-7)


def test_native_ddpg_deterministic_and_state_dict_views():
    """Two runs from the same weights on the same batches are bit-identical (fixed-order weight
    gradient reduction, no atomics), and the modules' state_dict() sees the native steps."""
    out = []
    for _ in range(2):
        torch.manual_seed(5)
        agent = make_agent(native=True)
        sd0 = {k: v.clone() for k, v in agent.actor.state_dict().items()}
        for it in range(3):
            agent.update(*_batch(4096, 10 + it))
        sd = agent.actor.state_dict()
        assert any(not torch.equal(sd[k], sd0[k]) for k in sd)
        out.append(torch.cat([_flat(getattr(agent, k)) for k in
                              ("actor", "target_actor", "critic", "target_critic")]))
    assert torch.equal(out[0], out[1])


def test_native_ddpg_rejects_other_nets():
    """A critic whose forward is not relu(Linear(cat(s, a))) ... Linear stays on the torch path
    under native='auto' and is refused under native=True."""
    class TanhCritic(Critic):
        def forward(self, s, a):
            return self.q(torch.tanh(self.fc2(torch.tanh(self.fc1(torch.cat([s, a], 1))))))

    lo, hi = np.array([-3., -3.]), np.array([3., 3.])
    env_msg = {'state_dim': 4, 'action_dim': 2, 'action_range': np.stack([lo, hi], 1), 'name': 'x'}
    mk = lambda native: DDPG(env_msg, actor=Actor(1e-4, 4, 2, lo, hi), target_actor=Actor(1e-4, 4, 2, lo, hi),
                             critic=TanhCritic(3e-4, 4, 2), target_critic=TanhCritic(3e-4, 4, 2),
                             device="cuda", native=native)
    assert mk("auto")._native is None
    with pytest.raises(ValueError):
        mk(True)


def test_native_ddpg_odd_shapes_track_torch():
    """Shapes that take the dense GEMM's generic staging paths: 3 states, 1 action, hidden widths
    48 / 20 (not multiples of 4 or of the 64-wide tiles), batch 777 (not a multiple of the
    256-row weight-gradient slices): native vs torch update from the same weights, 3 steps."""
    class C(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1, self.fc2, self.q = nn.Linear(4, 48), nn.Linear(48, 20), nn.Linear(20, 1)
            self.optimizer = torch.optim.Adam(self.parameters(), lr=3e-4)

        def forward(self, s, a):
            return self.q(func.relu(self.fc2(func.relu(self.fc1(torch.cat([s, a], 1))))))

    class Ac(nn.Module):
        def __init__(self):
            super().__init__()
            self.a_min, self.a_max = torch.tensor([-2.]), torch.tensor([2.])
            self.off = (self.a_min + self.a_max) / 2.0
            self.gain = self.a_max - self.off
            self.fc1, self.fc2, self.mu = nn.Linear(3, 48), nn.Linear(48, 20), nn.Linear(20, 1)
            self.optimizer = torch.optim.Adam(self.parameters(), lr=1e-4)

        def forward(self, s):
            return self.gain * torch.tanh(self.mu(func.relu(self.fc2(func.relu(self.fc1(s)))))) + self.off

    msg = {'state_dim': 3, 'action_dim': 1, 'action_range': np.array([[-2., 2.]]), 'name': 'x'}
    torch.manual_seed(9)
    nets = [Ac(), Ac(), C(), C()]
    agents = []
    for native in (False, True):
        ns = [type(m)() for m in nets]
        for m, src in zip(ns, nets):
            m.load_state_dict(src.state_dict())
        agents.append(DDPG(msg, 0.99, 0.005, 0.005, 10000, 777, *ns, device="cuda", native=native))
    assert agents[0]._native is None and agents[1]._native is not None
    rng = np.random.default_rng(4)
    B = 777
    d = lambda x: torch.as_tensor(x, dtype=torch.float32, device="cuda")
    import copy
    for it in range(3):
        batch = (d(rng.uniform(-2, 2, (B, 3))), d(rng.uniform(-2, 2, (B, 1))), d(rng.normal(size=B)),
                 d(rng.uniform(-2, 2, (B, 3))), d((rng.uniform(size=B) > 0.1).astype(np.float32)))
        before = [copy.deepcopy(getattr(agents[0], k)) for k in
                  ("actor", "target_actor", "critic", "target_critic")]
        lt = agents[0].update(*batch)
        ln = agents[1].update(*batch)
        for x, y in zip(lt, ln):
            torch.testing.assert_close(y, x, rtol=2e-4, atol=1e-6)
        if it == 0:   # the same start: both gradients against float64, f32-class bound
            tn = ddpg_f64_grads(before, agents[1].critic, batch)
            tt = ddpg_f64_grads(before, agents[0].critic, batch)
            for k in ("actor", "critic"):
                gt = torch.cat([p.grad.reshape(-1) for p in getattr(agents[0], k).parameters()])
                assert_f32_class(k, agents[1]._native.grad[k].cpu(), gt.cpu(), tn[k], tt[k])
    for k in ("actor", "target_actor", "critic", "target_critic"):
        a = _flat(getattr(agents[1], k))
        b = _flat(getattr(agents[0], k))
        assert float((a - b).abs().max()) <= 3e-5, (k, float((a - b).abs().max()))


@pytest.mark.parametrize("opt", ["sgd", "nadam", "adamw_wd"])
def test_native_ddpg_needs_plain_adam(opt):
    """The native update implements torch.optim.Adam only: an SGD, NAdam or weight-decayed AdamW
    optimizer keeps the torch update path under native='auto' (and trains with that optimizer),
    and native=True refuses it."""
    lo, hi = np.array([-3., -3.]), np.array([3., 3.])
    env_msg = {'state_dim': 4, 'action_dim': 2, 'action_range': np.stack([lo, hi], 1), 'name': 'x'}

    def mk(native):
        torch.manual_seed(2)
        nets = [Actor(1e-4, 4, 2, lo, hi), Actor(1e-4, 4, 2, lo, hi), Critic(3e-4, 4, 2),
                Critic(3e-4, 4, 2)]
        for m in (nets[0], nets[2]):
            m.optimizer = {"sgd": lambda p: torch.optim.SGD(p, lr=1e-3),
                           "nadam": lambda p: torch.optim.NAdam(p, lr=1e-3),
                           "adamw_wd": lambda p: torch.optim.AdamW(p, lr=1e-3, weight_decay=0.01),
                           }[opt](m.parameters())
        return DDPG(env_msg, actor=nets[0], target_actor=nets[1], critic=nets[2],
                    target_critic=nets[3], device="cuda", native=native)
    ag = mk("auto")
    assert ag._native is None
    p0 = _flat(ag.actor).clone()
    ag.update(*_batch(256, 0))
    assert not torch.equal(p0, _flat(ag.actor))
    with pytest.raises(ValueError):
        mk(True)
