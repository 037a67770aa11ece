"""GPU parity of the fused rollout kernel (rlp_rollout) — the bench's hot path.

(1) Teacher-forced parity against the oracle and the reference's shipped nets lives in
    test_gpu_rollout_parity.py.
(2) Size-independent invariants at the bench size (65 536 envs): s'_t == s_{t+1} and
    V(s'_t) == V(s_{t+1}) where not done; teacher-forced critic / actor log-prob recomputation.
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from reinforcementlearningplatform_amd import _abi as A
from reinforcementlearningplatform_amd import _native
from reinforcementlearningplatform_amd import kernels as K

pytestmark = pytest.mark.gpu


def dev(x):
    return torch.as_tensor(np.ascontiguousarray(x)).cuda()


def host(t):
    return t.detach().cpu().numpy()


def nets(S, Ad, seed, H=256):
    rng = np.random.default_rng(seed)
    ad = A.MLPDesc.make([S, H, H, Ad], [1, 1, 1])
    cd = A.MLPDesc.make([S, H, H, 1], [1, 1, 0])

    def init(d, last_gain):
        out = []
        ds = d.layer_dims()
        for i in range(d.n_layers):
            gain = last_gain if i == d.n_layers - 1 else 1.0
            w = rng.normal(0, gain / np.sqrt(ds[i]), (ds[i + 1], ds[i]))
            b = rng.normal(0, 0.05, ds[i + 1])
            out += [w.ravel(), b]
        return np.concatenate(out).astype(np.float32)
    return ad, init(ad, 1.0), cd, init(cd, 1.0)


def test_lidar_env_nets_pack_forward_and_update():
    """41-input nets (the lidar env's PPO2 demos) pack for the MFMA forward (layer 1 on 11
    K-steps), which matches the oracle's double-accumulated MLP; the native f16x3 update takes
    them with contiguous rows (layer 1 on the exact-f32 GEMM; precision: test_gpu_plain_nets.py)
    and refuses a gather index or a too-small workspace with a clean error before any launch."""
    from oracle import oracle
    kind = A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE
    D, S, Ad = A.ENV_DIMS[kind]
    ad, ap, cd, cp = nets(S, Ad, seed=1)
    x = np.random.default_rng(3).uniform(-1, 1, (3001, S)).astype(np.float32)
    for d, prm in ((ad, ap), (cd, cp)):
        pk = K.mfma_pack(d, dev(prm))
        y = K.mfma_forward(d, pk, dev(x)).cpu().numpy()
        ref = oracle.mlp_forward(d, prm, x)
        np.testing.assert_allclose(y, ref, rtol=1e-5, atol=2e-6)
    pk = K.mfma_pack(cd, dev(cp))
    cfg, vt = K.ppo2_loss_cfg(A.RLP_LOSS_CRITIC), dev(x[:, 0].copy())
    with pytest.raises(_native.RLPError, match="workspace"):
        K.ppo2_grad(cd, pk, cfg, dev(x), v_target=vt, workspace=torch.empty(1 << 20, device="cuda"))
    with pytest.raises(_native.RLPError, match="contiguous rows"):
        K.ppo2_grad(cd, pk, cfg, dev(x), v_target=vt, index=torch.arange(100, device="cuda"))
    g = K.ppo2_grad(cd, pk, cfg, dev(x), v_target=vt)
    assert torch.isfinite(g).all() and float(g.abs().max()) > 0


def test_rollout_invariants_at_bench_size():
    kind = A.RLP_ENV_CARTPOLE
    n, T = 65536, 48
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.cartpole_params()
    ad, ap, cd, cp = nets(S, Ad, seed=1)
    cfg = K.make_rollout_cfg(T, n, 3407, 0, 0, [8 / 3], [-8], [8], A.RLP_SUCCESS_DONE_AND_FLAG_NE, 3)
    st = K.new_state(kind, n)
    need = torch.ones(n, dtype=torch.uint8, device="cuda")
    bufs = K.rollout_buffers(kind, T, n)
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
    done = bufs["done"].bool()
    nd = ~done[:-1]
    # s'_t == s_{t+1} and V(s'_t) == V(s_{t+1}) where the env did not reset in between
    assert torch.equal(bufs["obs_next"][:-1][nd], bufs["obs"][1:][nd])
    assert torch.equal(bufs["value_next"][:-1][nd], bufs["value"][1:][nd])
    # teacher-forced critic: generic MFMA forward on the stored observations
    v = K.mlp_forward(cd, dev(cp), bufs["obs"].reshape(-1, S)).reshape(T, n)
    assert torch.allclose(v, bufs["value"], rtol=1e-5, atol=2e-5)
    # teacher-forced log-prob of the stored action under Normal(actor(s), std)
    m = K.mlp_forward(ad, dev(ap), bufs["obs"].reshape(-1, S)).reshape(T, n, 1) * 8
    lp = torch.distributions.Normal(m, torch.tensor(8 / 3, device="cuda")).log_prob(bufs["action"])
    assert torch.allclose(lp, bufs["logp"], rtol=1e-4, atol=1e-4)
    # episodes: every env starts at t=0 from the reset law, timeouts only at step 237
    assert bufs["action"].abs().max() <= 8
    f = bufs["flag"]
    assert set(torch.unique(f).tolist()) <= {0, 1, 2, 3, 4}
    obs0 = bufs["obs"][0]
    th0 = obs0[:, 0] / 2 * (np.pi / 4)
    assert th0.abs().max() <= np.pi / 8 + 1e-6 and obs0[:, 1].abs().max() == 0


@pytest.mark.parametrize("kind", [A.RLP_ENV_CARTPOLE, A.RLP_ENV_CARTPOLE_ANGLEONLY, A.RLP_ENV_SOI,
                                  A.RLP_ENV_UGV_FORWARD, A.RLP_ENV_UAV_HOVER_OUTER_LOOP])
def test_shared_physics_kernel_equals_register_kernel(kind):
    """rlp_rollout's shared-physics kernel (state in LDS, full-lane physics waves, resets right
    after the terminal step) and the register-resident kernel give identical buffers, state and
    need_reset flags, including envs that terminate and reset inside the segment."""
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind)
    ad, ap, cd, cp = nets(S, Ad, seed=kind + 20)
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 3 for l, h in zip(lo, hi)]
    n, T = 16384 + 37, 96
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    runs = []
    for phys in (1, 0, 3, 5):   # per-call selection (rlp_rollout_cfg.physics)
        cfg = K.make_rollout_cfg(T, n, 99, 5, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE,
                                 A.timeout_flag(kind), physics=phys)
        st = K.new_state(kind, n)
        need = torch.ones(n, dtype=torch.uint8, device="cuda")
        bufs = K.rollout_buffers(kind, T, n)
        for seg in range(2):  # a second segment starts from the first's state / need_reset
            K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
        runs.append(({k: v.clone() for k, v in bufs.items()}, st.clone(), need.clone()))
    (b1, s1, n1), *others = runs
    assert b1["done"][:-1].any(), "no env terminated inside the segment"
    # register kernel; 8-wave shared kernels (16-env waves; one block of 32- / 16-env waves per CU);
    # one 4-wave block of 32- / 64-env waves per CU (1 wave per SIMD)
    for bx, sx, nx in others:
        for key in b1:
            assert torch.equal(b1[key], bx[key]), key
        assert torch.equal(s1, sx)
        assert torch.equal(n1, nx)


def test_rollout_segments_chain():
    """Two T/2 segments == one T segment (state, need_reset and Philox counters carry over)."""
    kind = A.RLP_ENV_UAV_HOVER_OUTER_LOOP
    n, T = 4096, 16
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.uav_hover_params()
    ad, ap, cd, cp = nets(S, Ad, seed=3)
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    outs = []
    for split in (False, True):
        st = K.new_state(kind, n)
        need = torch.ones(n, dtype=torch.uint8, device="cuda")
        chunks = [(0, T // 2), (T // 2, T)] if split else [(0, T)]
        acts = []
        for a, b in chunks:
            cfg = K.make_rollout_cfg(b - a, n, 7, a, 0, [8 / 3] * 3, [-8] * 3, [8] * 3,
                                     A.RLP_SUCCESS_DONE_AND_FLAG_NE, 1)
            bufs = K.rollout_buffers(kind, b - a, n)
            K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
            acts.append(bufs["action"])
        outs.append((torch.cat(acts), st.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("kind", [A.RLP_ENV_CARTPOLE, A.RLP_ENV_UAV_HOVER_OUTER_LOOP,
                                  A.RLP_ENV_CARTPOLE_ANGLEONLY])
def test_mfma_forward_and_value_fixup(kind):
    D, S, Ad = A.ENV_DIMS[kind]
    ad, ap, cd, cp = nets(S, Ad, seed=11)
    rng = np.random.default_rng(kind)
    rows = 50_000 + 7
    x = rng.uniform(-2, 2, (rows, S)).astype(np.float32)
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    m = host(K.mfma_forward(ad, apk, dev(x)))
    v = host(K.mfma_forward(cd, cpk, dev(x)))
    np.testing.assert_allclose(m, oracle.mlp_forward(ad, ap, x), rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(v, oracle.mlp_forward(cd, cp, x), rtol=1e-5, atol=2e-5)
    done = (rng.uniform(0, 1, rows) < 0.05).astype(np.uint8)
    succ = (done * (rng.uniform(0, 1, rows) < 0.5)).astype(np.uint8)
    vn = torch.full((rows,), -123.0, device="cuda")
    K.value_fixup(cd, cpk, dev(x), dev(done), dev(succ), vn)
    vn = host(vn)
    need = (done == 1) & (succ == 0)
    np.testing.assert_allclose(vn[need], v[need, 0], rtol=1e-6, atol=1e-6)
    assert (vn[~need] == -123.0).all()


@pytest.mark.parametrize("kind", [A.RLP_ENV_CARTPOLE, A.RLP_ENV_UAV_HOVER_OUTER_LOOP,
                                  A.RLP_ENV_UGV_OBSTACLE_AVOIDANCE])
def test_mfma_forward_f16x3_per_call(kind):
    """rlp_mfma_forward / rlp_value_fixup with the f16x3 hidden layer chosen per call (ABI 3):
    against the oracle's double-accumulated nets at the exact path's bounds (rtol 1e-5, atol 2e-6),
    at a row count that takes the 32-row-wave launch, and a value fix-up on a masked subset."""
    D, S, Ad = A.ENV_DIMS[kind]
    ad, ap, cd, cp = nets(S, Ad, seed=12)
    rng = np.random.default_rng(kind + 100)
    rows = 140_001
    x = rng.uniform(-2, 2, (rows, S)).astype(np.float32)
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    for d, pk, prm in ((ad, apk, ap), (cd, cpk, cp)):
        y = host(K.mfma_forward(d, pk, dev(x), precision="f16x3"))
        ref = oracle.mlp_forward(d, prm, x)
        np.testing.assert_allclose(y, ref, rtol=1e-5, atol=2e-6)
        y32 = host(K.mfma_forward(d, pk, dev(x), precision="fp32"))
        assert not np.array_equal(y, y32)   # the two arithmetics really differ
    v = host(K.mfma_forward(cd, cpk, dev(x), precision="f16x3"))
    done = (rng.uniform(0, 1, rows) < 0.05).astype(np.uint8)
    succ = (done * (rng.uniform(0, 1, rows) < 0.5)).astype(np.uint8)
    vn = torch.full((rows,), -123.0, device="cuda")
    K.value_fixup(cd, cpk, dev(x), dev(done), dev(succ), vn, precision="f16x3")
    vn = host(vn)
    need = (done == 1) & (succ == 0)
    np.testing.assert_array_equal(vn[need], v[need, 0])   # same kernel arithmetic, bit for bit
    assert (vn[~need] == -123.0).all()


def test_two_threads_choose_precision_per_call():
    """Two host threads, each on its own stream, run rlp_mfma_forward and rlp_rollout with
    different hidden-layer arithmetics concurrently (fp32 in one, f16x3 in the other) while the
    library-wide default is flipped in between: every result equals the same call made alone,
    bit for bit (no global state is read by calls that choose per call)."""
    import threading
    kind = A.RLP_ENV_CARTPOLE
    p = A.cartpole_params()
    ad, ap, cd, cp = nets(4, 1, seed=21)
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    x = dev(np.random.default_rng(5).uniform(-2, 2, (70_001, 4)).astype(np.float32))
    n, T = 8192, 16

    def work(prec):
        mode = _native.MLP_FP32 if prec == "fp32" else _native.MLP_F16X3
        y = K.mfma_forward(cd, cpk, x, precision=prec)
        cfg = K.make_rollout_cfg(T, n, 9, 0, 0, [8 / 3], [-8], [8], A.RLP_SUCCESS_DONE_AND_FLAG_NE, 3,
                                 mlp_precision=mode)
        st = K.new_state(kind, n)
        need = torch.ones(n, dtype=torch.uint8, device="cuda")
        bufs = K.rollout_buffers(kind, T, n)
        K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
        return y, bufs["value"], bufs["action"], st

    alone = {q: [t.clone() for t in work(q)] for q in ("fp32", "f16x3")}
    torch.cuda.synchronize()
    assert not torch.equal(alone["fp32"][0], alone["f16x3"][0])
    got, errs = {}, []

    def thread(q):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(4):
                    got[q] = [t.clone() for t in work(q)]
            s.synchronize()
        except Exception as e:  # surfaced below
            errs.append(e)
    old = _native.get_mlp_precision()
    try:
        th = [threading.Thread(target=thread, args=(q,)) for q in ("fp32", "f16x3")]
        for t in th:
            t.start()
        for m in (_native.MLP_FP32, _native.MLP_F16X3, _native.MLP_FP32):
            _native.set_mlp_precision(m)   # the global default must not matter
        for t in th:
            t.join()
    finally:
        _native.set_mlp_precision(old)
    assert not errs, errs
    for q in ("fp32", "f16x3"):
        for a, b in zip(got[q], alone[q]):
            assert torch.equal(a, b), q


@pytest.mark.parametrize("kind", [A.RLP_ENV_CARTPOLE, A.RLP_ENV_UAV_HOVER_OUTER_LOOP])
def test_mlp_precision_modes_vs_float64(kind):
    """rlp_rollout's two hidden-layer arithmetics against a float64 evaluation of the critic on the
    observations each run recorded: the f16x3 split (default) must stay within a small factor of
    the exact f32-MFMA path's own error, and well inside the 1e-5 parity tolerance."""
    D, S, Ad = A.ENV_DIMS[kind]
    p = A.default_params(kind)
    ad, ap, cd, cp = nets(S, Ad, seed=5)
    lo, hi = A.action_bounds(kind, p)
    std = [(h - l) / 6 for l, h in zip(lo, hi)]
    n, T = 8192, 8
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    errs = {}
    for mode in (_native.MLP_FP32, _native.MLP_F16X3):   # per call (rlp_rollout_cfg)
        cfg = K.make_rollout_cfg(T, n, 11, 0, 0, std, lo, hi, A.RLP_SUCCESS_DONE_AND_FLAG_NE,
                                 A.timeout_flag(kind), mlp_precision=mode)
        st = K.new_state(kind, n)
        need = torch.ones(n, dtype=torch.uint8, device="cuda")
        bufs = K.rollout_buffers(kind, T, n)
        K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
        obs = host(bufs["obs"]).reshape(-1, S)
        v64 = oracle.mlp_forward(cd, cp, obs)[:, 0]
        v = host(bufs["value"]).reshape(-1).astype(np.float64)
        errs[mode] = np.abs(v - v64) / (np.abs(v64) + 1.0)
    e32, ex3 = errs[_native.MLP_FP32], errs[_native.MLP_F16X3]
    assert e32.max() < 1e-5 and ex3.max() < 1e-5
    assert ex3.max() <= 4 * e32.max() + 1e-7, (ex3.max(), e32.max())
    assert ex3.mean() <= 4 * e32.mean() + 1e-8, (ex3.mean(), e32.mean())


def test_per_call_selection_overrides_library_default():
    """rlp_rollout_cfg's mlp_precision / physics / sub apply to that call only, whatever the
    library-wide rlp_set_* defaults are (a multi-threaded host needs no global knob)."""
    kind = A.RLP_ENV_CARTPOLE
    p = A.cartpole_params()
    ad, ap, cd, cp = nets(4, 1, seed=2)
    apk, cpk = K.mfma_pack(ad, dev(ap)), K.mfma_pack(cd, dev(cp))
    n, T = 4096, 16

    def run(**sel):
        cfg = K.make_rollout_cfg(T, n, 3, 0, 0, [8 / 3], [-8], [8], A.RLP_SUCCESS_DONE_AND_FLAG_NE, 3,
                                 **sel)
        st = K.new_state(kind, n)
        need = torch.ones(n, dtype=torch.uint8, device="cuda")
        bufs = K.rollout_buffers(kind, T, n)
        K.rollout(kind, p, st, need, ad, apk, cd, cpk, cfg, bufs)
        return bufs["value"].clone()
    v32 = run(mlp_precision=_native.MLP_FP32)
    vx3 = run(mlp_precision=_native.MLP_F16X3)
    assert not torch.equal(v32, vx3)
    old = _native.get_mlp_precision()
    try:
        _native.set_mlp_precision(_native.MLP_FP32)
        assert torch.equal(run(mlp_precision=_native.MLP_F16X3), vx3)
        assert torch.equal(run(), v32)
    finally:
        _native.set_mlp_precision(old)
    assert torch.equal(run(mlp_precision=_native.MLP_F16X3, physics=0, sub=4), vx3)
    # the 8-wave variants (16-env waves; one block of 32-env waves per CU): same arithmetic
    assert torch.equal(run(mlp_precision=_native.MLP_F16X3, physics=3), vx3)
    assert torch.equal(run(mlp_precision=_native.MLP_F16X3, physics=5), vx3)


@pytest.mark.parametrize("acts", ["relu", "tanh"])
def test_mlp_forward_large_batch_dense_path(acts):
    """rlp_mlp_forward on >= 2048 unmasked rows runs the tiled dense GEMM (one launch per layer):
    against torch float32 Linear stacks for the DDPG driver's relu actor [4,256,256,2] and a
    tanh net, and against the one-wave-per-16-rows kernel (masked call) on the same rows."""
    torch.manual_seed(1)
    act = A.RLP_ACT_RELU if acts == "relu" else A.RLP_ACT_TANH
    d = A.MLPDesc.make([4, 256, 256, 2], [act, act, A.RLP_ACT_NONE])
    layers = [torch.nn.Linear(4, 256), torch.nn.Linear(256, 256), torch.nn.Linear(256, 2)]
    flat = torch.cat([t.detach().reshape(-1) for l in layers for t in (l.weight, l.bias)]).cuda()
    n = 5003
    x = torch.rand(n, 4, device="cuda") * 4 - 2
    f = torch.relu if acts == "relu" else torch.tanh
    with torch.no_grad():
        h = x
        for i, l in enumerate(layers):
            h = torch.nn.functional.linear(h, l.weight.cuda(), l.bias.cuda())
            if i < 2:
                h = f(h)
    y = K.mlp_forward(d, flat, x)
    torch.testing.assert_close(y, h, rtol=1e-5, atol=2e-6)
    y_small = K.mlp_forward(d, flat, x, mask=torch.ones(n, dtype=torch.uint8, device="cuda"))
    torch.testing.assert_close(y, y_small, rtol=1e-5, atol=2e-6)
