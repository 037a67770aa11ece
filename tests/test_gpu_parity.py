"""GPU parity: librlp.so's HIP kernels against the CPU oracle and the reference's golden vectors.

Tolerances: physics is float64 on both sides, so env outputs must match the
reference numpy step() to ~1 ulp of libm (checked at rtol 1e-9); float32 observations to 1 ulp;
MLP outputs (fp32 MFMA vs the reference's fp32 torch) at rtol 1e-5 + atol 1e-6-ish; GAE is
bit-exact; Philox resets are bit-exact."""
import numpy as np
import pytest
import torch

from oracle import oracle
from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd import kernels as K

pytestmark = pytest.mark.gpu

from test_oracle_golden import ENV_CASES  # noqa: E402


def dev(x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def host(t):
    return t.detach().cpu().numpy()


def close(a, b, rtol, atol, what):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    bad = np.abs(a - b) > atol + rtol * np.abs(b)
    assert not bad.any(), f"{what}: {bad.sum()} mismatches, max abs err {np.max(np.abs(a - b))}"


@pytest.mark.parametrize("name,kind,pf", ENV_CASES, ids=[c[0] for c in ENV_CASES])
def test_env_step_vs_reference_golden(golden, name, kind, pf):
    g = golden(name)
    p = pf()
    st = dev(g["state"].T)
    oc, on, r, f, d = K.env_step(kind, p, st, dev(g["action"]))
    torch.cuda.synchronize()
    close(host(st).T, g["state_next"], 1e-9, 1e-12, "state_next")
    close(host(oc), g["obs_cur"].astype(np.float32), 1e-6, 1e-7, "obs_cur")
    close(host(on), g["obs_next"].astype(np.float32), 1e-6, 1e-7, "obs_next")
    close(host(r), g["reward"], 1e-7, 1e-9, "reward")
    np.testing.assert_array_equal(host(f), g["flag"])
    np.testing.assert_array_equal(host(d), g["done"])


def _random_states(kind, n, rng):
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind)
    st = np.zeros((D, n))
    oracle.env_reset(kind, p, st, seed=123, counter=7)
    # spread the states, incl. out-of-bounds neighbourhoods
    if kind in (A.RLP_ENV_CARTPOLE, A.RLP_ENV_CARTPOLE_ANGLEONLY):
        st[0] = rng.uniform(-0.85, 0.85, n); st[1] = rng.uniform(-3, 3, n)
        st[2] = rng.uniform(-1.6, 1.6, n); st[3] = rng.uniform(-3, 3, n)
        st[4] = rng.integers(0, 250, n) * 0.02
    elif kind == A.RLP_ENV_SOI:
        st[0:2] = rng.uniform(-0.1, 5.1, (2, n)); st[2:4] = rng.uniform(-3, 3, (2, n))
        st[4] = rng.integers(0, 250, n) * 0.02
    elif kind in (A.RLP_ENV_UGV_FORWARD, A.RLP_ENV_UGV_BIDIRECTIONAL):
        st[0:2] = rng.uniform(-0.1, 5.1, (2, n)); st[2] = rng.uniform(-0.5, 3, n)
        st[3] = rng.uniform(-np.pi, np.pi, n); st[4] = rng.uniform(-3, 3, n)
        st[5] = rng.integers(0, 500, n) * 0.02
    elif kind == A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE:   # the reset maps, any pose in/near them
        st[0:2] = rng.uniform(-0.1, 5.1, (2, n)); st[2] = rng.uniform(-0.5, 3, n)
        st[3] = rng.uniform(-np.pi, np.pi, n); st[4] = rng.uniform(-3, 3, n)
        st[5] = rng.integers(0, 152, n) * 0.1
        st[3, ::7] = rng.choice([0.0, np.pi / 2, -np.pi / 2, np.pi, -np.pi], st[3, ::7].shape)
    else:
        st[0:3] = rng.uniform(-4.9, 4.9, (3, n)); st[2] = rng.uniform(0.05, 4.9, n)
        st[3:6] = rng.uniform(-2, 2, (3, n)); st[6:9] = rng.uniform(-0.6, 0.6, (3, n))
        st[9:12] = rng.uniform(-2, 2, (3, n)); st[12] = rng.integers(0, 999, n) * 0.01
        st[16:22] = rng.uniform(-0.3, 0.3, (6, n))
    lo, hi = A.action_bounds(kind, p)
    act = rng.uniform(lo, hi, (n, Ad)).astype(np.float32)
    return p, st, act


@pytest.mark.parametrize("kind", sorted(A.ENV_DIMS))
def test_env_step_vs_oracle_large(kind):
    rng = np.random.default_rng(kind)
    n = 1 << 16
    p, st, act = _random_states(kind, n, rng)
    st0 = st.copy()
    g = dev(st)
    oc, on, r, f, d = K.env_step(kind, p, g, dev(act))
    o_oc, o_on, o_r, o_f, o_d = oracle.env_step(kind, p, st, act)
    torch.cuda.synchronize()
    close(host(g), st, 1e-9, 1e-12, "state")
    close(host(oc), o_oc, 1e-6, 1e-7, "obs_cur")
    close(host(on), o_on, 1e-6, 1e-7, "obs_next")
    close(host(r), o_r, 1e-8, 1e-9, "reward")
    # flags and done exact; a row is exempt only when the oracle's own flag flips under a 1e-12
    # relative perturbation of its input state (a threshold straddled within float64 rounding of
    # libm ulps), and such rows are listed
    hf, hd = host(f), host(d)
    bad = np.nonzero((hf != o_f) | (hd != o_d))[0]
    exempt = []
    for i in bad:
        flips = set()
        for eps in (-2e-12, -1e-12, 1e-12, 2e-12):
            sp = np.ascontiguousarray(st0[:, i:i + 1] * (1 + eps))
            _, _, _, pf_, pd_ = oracle.env_step(kind, p, sp, act[i:i + 1])
            flips.add((int(pf_[0]), int(pd_[0])))
        assert (int(hf[i]), int(hd[i])) in flips, \
            f"env {i}: flag/done {hf[i]}/{hd[i]} vs oracle {o_f[i]}/{o_d[i]} with margin > 1e-12"
        exempt.append(int(i))
    if exempt:
        print(f"kind {kind}: rows within 1e-12 of a threshold (exempt): {exempt}")
    assert len(exempt) <= 2, exempt


@pytest.mark.parametrize("kind", sorted(A.ENV_DIMS))
def test_reset_bit_exact_and_observe(kind):
    D, S, _ = A.ENV_DIMS[kind]
    p = A.default_params(kind)
    n = 100_003
    rng = np.random.default_rng(5)
    mask = (rng.uniform(0, 1, n) < 0.7).astype(np.uint8)
    st0 = rng.uniform(-1, 1, (D, n))
    g = dev(st0)
    K.env_reset(kind, p, g, mask=dev(mask), seed=3407, counter=11, env_id0=1000)
    o = st0.copy()
    oracle.env_reset(kind, p, o, mask=mask, seed=3407, counter=11, env_id0=1000)
    np.testing.assert_array_equal(host(g), o)
    obs = K.env_observe(kind, p, g)
    close(host(obs), oracle.env_observe(kind, p, o), 1e-6, 1e-7, "observe")


def test_mlp_forward_shipped_nets(golden):
    g = golden("ppo2_cartpole_nets")
    ad = A.MLPDesc.make([4, 256, 256, 1], [1, 1, 1])
    cd = A.MLPDesc.make([4, 256, 256, 1], [1, 1, 0])
    x = dev(g["x"])
    mean = host(K.mlp_forward(ad, dev(g["actor_params"]), x)) * np.float32(8)
    v = host(K.mlp_forward(cd, dev(g["critic_params"]), x))
    close(mean, g["actor_mean"], 1e-5, 2e-6, "actor mean vs torch")
    close(v, g["critic_v"], 1e-5, 2e-5, "critic v vs torch")


@pytest.mark.parametrize("dims,acts", [
    ([4, 128, 64, 32, 2], [1, 1, 1, 1]),      # PPO2-4-SecondOrderIntegration actor
    ([6, 128, 64, 3], [1, 1, 1]),             # PPO-4-UavHoverOuterLoop actor
    ([2, 256, 256, 1], [1, 1, 0]),            # AngleOnly critic
    ([41, 256, 256, 2], [1, 1, 1]),           # UGV obstacle-avoidance actor (41 inputs)
    ([5, 33, 17, 1], [2, 1, 0]),              # ragged widths, relu
])
def test_mlp_forward_generic_vs_oracle(dims, acts):
    rng = np.random.default_rng(len(dims) * 100 + dims[0])
    d = A.MLPDesc.make(dims, acts)
    prm = (rng.normal(0, 1, d.param_count()) / 8).astype(np.float32)
    n = 3001
    x = rng.uniform(-2, 2, (n, dims[0])).astype(np.float32)
    mask = (rng.uniform(0, 1, n) < 0.5).astype(np.uint8)
    y = K.mlp_forward(d, dev(prm), dev(x), mask=dev(mask), out=torch.full((n, dims[-1]), 7.0,
                                                                           device="cuda"))
    ref = oracle.mlp_forward(d, prm, x)
    yh = host(y)
    close(yh[mask == 1], ref[mask == 1], 1e-5, 2e-6, "masked rows")
    assert (yh[mask == 0] == 7.0).all()


def test_policy_sample_philox_and_noise(golden):
    rng = np.random.default_rng(2)
    n, Ad = 70_000, 3
    mean = rng.uniform(-9, 9, (n, Ad)).astype(np.float32)
    std, lo, hi = [2.6, 1.0, 0.5], [-8, -8, -8], [8, 8, 8]
    a, lp = K.policy_sample(dev(mean), std, lo, hi, seed=3407, counter=99, env_id0=5)
    oa, olp = oracle.policy_sample(mean, std, lo, hi, seed=3407, counter=99, env_id0=5)
    close(host(a), oa, 1e-6, 2e-6, "philox action")
    close(host(lp), olp, 1e-6, 2e-6, "philox logp")
    eps = rng.normal(0, 1, (n, Ad)).astype(np.float32)
    a, lp = K.policy_sample(dev(mean), std, lo, hi, noise=dev(eps))
    oa, olp = oracle.policy_sample(mean, std, lo, hi, noise=eps)
    close(host(a), oa, 0, 1e-6, "noise action")
    close(host(lp), olp, 1e-6, 1e-6, "noise logp")
    # reference log_prob semantics on the shipped-net samples
    g = golden("ppo2_cartpole_nets")
    m = g["actor_mean"][:256]
    e = (g["sample_a"].astype(np.float64) - m) / float(g["std"])
    cl = np.abs(g["sample_a"]) >= 8
    e[cl] = np.sign(g["sample_a"][cl]) * (np.abs(e[cl]) + 1)
    a, lp = K.policy_sample(dev(m), float(g["std"]), [-8], [8], noise=dev(e.astype(np.float32)))
    close(host(a), g["sample_a"], 0, 2e-6, "sample a vs torch")
    close(host(lp), g["sample_logp"], 0, 2e-6, "sample logp vs torch")


def test_gae_bit_exact_vs_reference(golden):
    g = golden("gae")
    for c in range(4):
        k = lambda s: g[f"c{c}_{s}"]
        T = len(k("r"))
        col = lambda x, dt: dev(x.reshape(T, 1), dt)
        stats = K.adv_stats_buffer(1, device="cuda")
        adv, vt = K.gae(col(k("r"), torch.float32), col(k("v"), torch.float32),
                        col(k("vn"), torch.float32), col(k("done"), torch.uint8),
                        col(k("success"), torch.uint8), float(g["gamma"]), float(g["lmd"]),
                        stats=stats)
        np.testing.assert_array_equal(host(adv).ravel(), k("adv"))
        np.testing.assert_array_equal(host(vt).ravel(), k("v_target"))
        K.adv_normalize(adv, stats)
        close(host(adv).ravel(), k("adv_norm"), 2e-5, 2e-6, "adv_norm")


def test_gae_batched_bit_exact_vs_oracle():
    rng = np.random.default_rng(9)
    T, n = 200, 40_000
    r = rng.normal(0, 1, (T, n)).astype(np.float32)
    v = rng.normal(30, 5, (T, n)).astype(np.float32)
    vn = rng.normal(30, 5, (T, n)).astype(np.float32)
    done = (rng.uniform(0, 1, (T, n)) < 0.01).astype(np.uint8)
    succ = (done * (rng.uniform(0, 1, (T, n)) < 0.6)).astype(np.uint8)
    adv, vt = K.gae(dev(r), dev(v), dev(vn), dev(done), dev(succ), 0.999, 0.95)
    oadv, ovt = oracle.gae(r, v, vn, done, succ, 0.999, 0.95)
    np.testing.assert_array_equal(host(adv), oadv)
    np.testing.assert_array_equal(host(vt), ovt)


@pytest.mark.parametrize("T,n", [(1000, 1), (64, 10_000), (3, 65_536)])
def test_reward_norm_vs_oracle(golden, T, n):
    rng = np.random.default_rng(T)
    r = rng.normal(-2, 3, (T, n)).astype(np.float32)
    rms = torch.zeros(4, dtype=torch.float64, device="cuda")
    out = host(K.reward_norm(dev(r), rms))
    o, orms = oracle.reward_norm(r)
    close(out, o, 1e-6, 1e-6, "normalised reward")
    close(host(rms), orms, 1e-9, 1e-9, "running stats")
    if n == 1:
        gg = golden("reward_norm")
        rms = torch.zeros(4, dtype=torch.float64, device="cuda")
        out = host(K.reward_norm(dev(gg["x"].astype(np.float32).reshape(-1, 1)), rms)).ravel()
        close(out, gg["y"], 1e-5, 1e-6, "vs reference Normalization")


@pytest.mark.parametrize("T,n", [(64, 8192), (5, 4096 * 3)])
def test_reward_norm_cross_rank_merge_bit_exact(T, n):
    """SURVEY §8e's Welford/Chan merge across ranks: W "ranks" of n envs (chunk statistics
    gathered rank-major, merged in global env order) reproduce one rank of W*n envs bit for bit,
    and every rank ends with the same running statistics."""
    rng = np.random.default_rng(n)
    W = 2
    r = rng.normal(-1, 2, (T, W * n)).astype(np.float32)
    rms1 = torch.zeros(4, dtype=torch.float64, device="cuda")
    whole = host(K.reward_norm(dev(r), rms1))
    parts, halves = [], []
    for k in range(W):
        rk = dev(r[:, k * n:(k + 1) * n])
        work = K.reward_norm_workspace(T, n, "cuda")
        parts.append(K.reward_norm_stats(rk, work).clone())
        halves.append((rk, work))
    allp = torch.cat(parts)
    for k, (rk, work) in enumerate(halves):
        rms = torch.zeros(4, dtype=torch.float64, device="cuda")
        out = host(K.reward_norm_finish(rk, rms, work, allp, W))
        np.testing.assert_array_equal(out, whole[:, k * n:(k + 1) * n])
        np.testing.assert_array_equal(host(rms), host(rms1))


@pytest.mark.parametrize("T,n", [(128, 65536), (7, 1000), (300, 4097), (50, 1), (3, 65_536)])
def test_gae_normalized_bit_exact_vs_stored_rewards(T, n):
    """GAE over the raw rewards normalised as they are loaded (rlp_reward_norm_statistics ->
    rlp_gae_normalized) gives the same bits as rlp_reward_norm (normalised rewards stored) ->
    rlp_gae: advantages, v_target, the advantage partials and the normalised advantages, the
    running statistics, over three chained segments; reward_norm_apply reproduces the stored
    normalised rewards from the statistics."""
    rng = np.random.default_rng(T * 7 + n)
    rms_a = torch.zeros(4, dtype=torch.float64, device="cuda")
    rms_b = torch.zeros(4, dtype=torch.float64, device="cuda")
    work_a = K.reward_norm_workspace(T, n, "cuda")
    work_b = K.reward_norm_workspace(T, n, "cuda")
    st_a, st_b = K.adv_stats_buffer(n, device="cuda"), K.adv_stats_buffer(n, device="cuda")
    for seg in range(3):
        r = dev(rng.normal(-1 + seg, 2, (T, n)).astype(np.float32))
        v = dev(rng.normal(30, 5, (T, n)).astype(np.float32))
        vn = dev(rng.normal(30, 5, (T, n)).astype(np.float32))
        done = (rng.uniform(0, 1, (T, n)) < 0.02).astype(np.uint8)
        succ = dev((done * (rng.uniform(0, 1, (T, n)) < 0.5)).astype(np.uint8))
        done = dev(done)
        rn = K.reward_norm(r, rms_a, work_a)
        adv_a, vt_a = K.gae(rn, v, vn, done, succ, 0.999, 0.95, stats=st_a)
        K.reward_norm_statistics(r, rms_b, work_b)
        adv_b, vt_b = K.gae_normalized(r, work_b, v, vn, done, succ, 0.999, 0.95, stats=st_b)
        np.testing.assert_array_equal(host(K.reward_norm_apply(r, work_b)), host(rn))
        np.testing.assert_array_equal(host(st_b), host(st_a))
        K.adv_normalize(adv_a, st_a)
        K.adv_normalize(adv_b, st_b)
        np.testing.assert_array_equal(host(rms_b), host(rms_a))
        np.testing.assert_array_equal(host(vt_b), host(vt_a))
        np.testing.assert_array_equal(host(adv_b), host(adv_a))


@pytest.mark.parametrize("T,n", [(128, 65536), (7, 1000)])
def test_adv_stats_deterministic_two_pass_and_cross_rank(T, n):
    """rlp_gae's advantage partials: run-to-run identical (no atomics), the normalised advantages
    match a float64 two-pass mean / unbiased std (torch .std()), and the partials of two half
    batches, gathered, give the whole batch's normalisation bit for bit (n a multiple of 256)."""
    rng = np.random.default_rng(T)
    r = rng.normal(0, 1, (T, n)).astype(np.float32)
    v = rng.normal(30, 5, (T, n)).astype(np.float32)
    vn = rng.normal(30, 5, (T, n)).astype(np.float32)
    done = (rng.uniform(0, 1, (T, n)) < 0.01).astype(np.uint8)
    succ = (done * (rng.uniform(0, 1, (T, n)) < 0.6)).astype(np.uint8)
    outs = []
    for _ in range(2):
        st = K.adv_stats_buffer(n, device="cuda")
        adv, _ = K.gae(dev(r), dev(v), dev(vn), dev(done), dev(succ), 0.999, 0.95, stats=st)
        raw = host(adv).astype(np.float64)
        K.adv_normalize(adv, st)
        outs.append((host(adv), host(st)))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    m, sd = raw.mean(), raw.std(ddof=1)
    P = K.adv_stats_parts(n)
    assert abs(outs[0][1][3 * P] - m) <= 1e-12 * (abs(m) + sd)
    assert abs(outs[0][1][3 * P + 1] - sd) <= 1e-12 * sd
    ref = (raw.astype(np.float32) - np.float32(m)) / (np.float32(sd) + np.float32(1e-5))
    close(outs[0][0], ref, 1e-6, 1e-6, "normalised advantages")
    if n % 512 == 0:
        h = n // 2
        stp = []
        advs = []
        for k in range(2):
            sl = slice(k * h, (k + 1) * h)
            st = K.adv_stats_buffer(h, device="cuda")
            a, _ = K.gae(dev(r[:, sl]), dev(v[:, sl]), dev(vn[:, sl]), dev(done[:, sl]),
                         dev(succ[:, sl]), 0.999, 0.95, stats=st)
            stp.append(st[:3 * K.adv_stats_parts(h)])
            advs.append(a)
        allp = torch.cat(stp + [torch.zeros(2, dtype=torch.float64, device="cuda")])
        for k in range(2):
            K.adv_normalize(advs[k], allp, 2 * K.adv_stats_parts(h))
            np.testing.assert_array_equal(host(advs[k]), outs[0][0][:, k * h:(k + 1) * h])
