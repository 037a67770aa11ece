"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own Python code.

Run only in the build container (the reference is mounted read-only at /root/reference and never
travels to the GPU box):    python tests/golden/make_golden.py [/root/reference]

What is recorded (inputs and expected outputs only — no reference source is copied):
  * per env copy: teacher-forced single steps (state, float32 action -> next state, obs, reward,
    terminal flag), incl. threshold-straddling states and both RK4 sub-step regimes (CartPole);
  * UAV hover outer loop: multi-step sequences incl. the carried FNTSMC controller state;
  * the PPO2-CartPole shipped actor/critic (datasave/net, loaded with weights_only=True):
    forward on random inputs, choose_action samples, and the deterministic closed-loop
    known answer;
  * Proximal_Policy_Optimization2.learn()'s GAE / v_target / advantage normalisation;
  * utils.classes.Normalization on a reward stream.
cv2 is absent here and only used for drawing: it is replaced by a no-op module.
"""
import importlib.util
import os
import signal
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_cv2_stub():
    cv2 = types.ModuleType("cv2")

    def _noop(*a, **k):
        return -1
    for name in ("imshow", "waitKey", "rectangle", "line", "circle", "putText", "destroyAllWindows",
                 "VideoWriter", "VideoWriter_fourcc", "fillPoly", "ellipse", "arrowedLine",
                 "polylines", "namedWindow", "imwrite"):
        setattr(cv2, name, _noop)
    cv2.FONT_HERSHEY_COMPLEX = 0
    cv2.FONT_HERSHEY_SIMPLEX = 0
    cv2.LINE_AA = 0
    sys.modules["cv2"] = cv2


_install_cv2_stub()
for p in (REF, os.path.join(REF, "environment/UavRobust")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402  (after the stub; seeds are set after all imports)


def load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, path))
    mod = importlib.util.module_from_spec(spec)
    sys.path.insert(0, os.path.dirname(os.path.join(REF, path)))
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.path.pop(0)
    return mod


import contextlib, io  # noqa: E402


@contextlib.contextmanager
def quiet():
    with contextlib.redirect_stdout(io.StringIO()):
        yield


# ---------------------------------------------------------------------------------------------
mods = {}
with quiet():
    mods["cp_ppo2"] = load("demonstration/PPO2/PPO2-4-CartPole/CartPole.py", "ref_cp_ppo2")
    mods["cp_dppo2"] = load("demonstration/DPPO2/DPPO2-4-CartPole/CartPole.py", "ref_cp_dppo2")
    mods["ao_ppo2"] = load("demonstration/PPO2/PPO2-4-CartPoleAngleOnly/cartpole_angleonly.py",
                           "ref_ao_ppo2")
    mods["ao_env"] = load("environment/CartPole/CartPoleAngleOnly.py", "ref_ao_env")
    mods["soi_env"] = load("environment/SecondOrderIntegration/SecondOrderIntegration.py", "ref_soi")
    mods["soi_dppo2"] = load("demonstration/DPPO2/DPPO2-4-SecondOrderIntegration/"
                             "SecondOrderIntegration.py", "ref_soi_dppo2")
    mods["ugvf_env"] = load("environment/UGV/UGVForward.py", "ref_ugvf")
    mods["ugvf_ppo2"] = load("demonstration/PPO2/PPO2-4-UGVForward/UGVForward.py", "ref_ugvf_ppo2")
    mods["ugvf_dppo2"] = load("demonstration/DPPO2/DPPO2-4-UGVForward/UGVForward.py",
                              "ref_ugvf_dppo2")
    mods["ugvb_env"] = load("environment/UGV/UGVBidirectional.py", "ref_ugvb")
    mods["ugvb_ppo2"] = load("demonstration/PPO2/PPO2-4-UGVBidirectional/UGVBidirectional.py",
                             "ref_ugvb_ppo2")
    mods["ugvoa_env"] = load("environment/UGVForwardObstacleAvoidance/UGVForwardObstacleAvoidance.py",
                             "ref_ugvoa")
    mods["ugvoa_ppo2"] = load("demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/"
                              "UGVForwardObstacleAvoidance.py", "ref_ugvoa_ppo2")
    mods["ugvoa_dppo2"] = load("demonstration/DPPO2/DPPO2-4-UGVForwardObstacleAvoidance/"
                               "UGVForwardObstacleAvoidance.py", "ref_ugvoa_dppo2")
    import environment.UavRobust.UavHoverOuterLoop as uav_mod  # noqa: E402
    from environment.UavRobust.uav import uav_param  # noqa: E402
    from environment.UavRobust.FNTSMC import fntsmc_param  # noqa: E402
    ppo2_mod = load("algorithm/policy_base/Proximal_Policy_Optimization2.py", "ref_ppo2")
    cls_mod = load("utils/classes.py", "ref_classes")
    drv = load("demonstration/PPO2/PPO2-4-CartPole/train.py", "ref_ppo2_cartpole_train")

rng = np.random.default_rng(3407)
torch.manual_seed(3407)
np.random.seed(3407)


def f32(x):
    return np.asarray(x, dtype=np.float32)


# ---------------------------------------------------------------------------------------------
# CartPole (PPO2 copy == env dir; DPPO2 copy)
# ---------------------------------------------------------------------------------------------
def cartpole_time_table(mod, steps):
    env = mod.CartPole(0., 0.)
    env.reset(False)
    times = []
    for _ in range(steps):
        times.append(env.time)
        env.rk44(np.array([np.float32(0.)]))
    return np.array(times)


def gen_cartpole(key, mod, n=600):
    env = mod.CartPole(0., 0.)
    tt = cartpole_time_table(mod, 245)
    rows = {k: [] for k in ("state", "action", "state_next", "obs_cur", "obs_next", "reward",
                            "flag", "done")}
    th_hi = env.theta_max + np.pi / 180
    th_lo = -env.dtheta_max - np.pi / 180
    for i in range(n):
        k = int(rng.integers(0, 245))
        th = rng.uniform(-0.9, 0.9)
        x = rng.uniform(-1.4, 1.4)
        dth, dx = rng.uniform(-3, 3), rng.uniform(-3, 3)
        kind = i % 8
        if kind == 1:
            th = th_hi + rng.uniform(-2e-3, 2e-3); dth = rng.uniform(-0.05, 0.05)
        elif kind == 2:
            th = th_lo + rng.uniform(-5e-3, 5e-3); dth = rng.uniform(-0.05, 0.05)
        elif kind == 3:
            x = np.sign(rng.uniform(-1, 1)) * (env.x_max + rng.uniform(-2e-3, 2e-3))
            dx = rng.uniform(-0.05, 0.05)
        elif kind == 4:
            k = int(rng.integers(230, 245))
        elif kind == 5:
            th, dth, x, dx = [rng.uniform(-2e-3, 2e-3) for _ in range(4)]
        a = np.float32(rng.uniform(-8, 8))
        if i % 13 == 0:
            a = np.float32(rng.choice([-8, 8]))
        env.reset(False)
        env.theta, env.dtheta, env.x, env.dx, env.time = th, dth, x, dx, tt[k]
        env.etheta, env.ex = 0. - th, 0. - x
        rows["state"].append([th, dth, x, dx, tt[k]])
        env.step_update(np.array([a], dtype=np.float32))
        rows["action"].append([a])
        rows["state_next"].append([env.theta, env.dtheta, env.x, env.dx, env.time])
        rows["obs_cur"].append(env.current_state)
        rows["obs_next"].append(env.next_state)
        rows["reward"].append(float(env.reward))
        rows["flag"].append(env.terminal_flag)
        rows["done"].append(int(env.is_terminal))
    out = {k: np.array(v) for k, v in rows.items()}
    out["action"] = out["action"].astype(np.float32)
    out["time_table"] = tt
    np.savez(os.path.join(OUT, f"{key}.npz"), **out)
    print(key, {k: v.shape for k, v in out.items()}, "flags", np.bincount(out["flag"]))


def gen_angleonly(key, mod, n=400):
    env = mod.CartPoleAngleOnly(0.)
    rows = {k: [] for k in ("state", "action", "state_next", "obs_cur", "obs_next", "reward",
                            "flag", "done")}
    th_hi = env.thetaMax + np.pi / 180
    for i in range(n):
        k = int(rng.integers(0, 252))
        th, dth = rng.uniform(-0.85, 0.85), rng.uniform(-4, 4)
        x, dx = rng.uniform(-2, 2), rng.uniform(-2, 2)
        if i % 6 == 1:
            th = np.sign(rng.uniform(-1, 1)) * (th_hi + rng.uniform(-2e-3, 2e-3))
            dth = rng.uniform(-0.05, 0.05)
        elif i % 6 == 2:
            k = int(rng.integers(245, 252))
        elif i % 6 == 3:
            th, dth = rng.uniform(-2e-3, 2e-3), rng.uniform(-2e-3, 2e-3)
        tm = 0.
        for _ in range(k):
            tm += env.dt
        a = np.float32(rng.uniform(-5, 5))
        with quiet():
            env.reset(False)
            env.theta, env.dtheta, env.x, env.dx, env.time = th, dth, x, dx, tm
            rows["state"].append([th, dth, x, dx, tm])
            env.step_update(np.array([a], dtype=np.float32))
        rows["action"].append([a])
        rows["state_next"].append([env.theta, env.dtheta, env.x, env.dx, env.time])
        rows["obs_cur"].append(env.current_state)
        rows["obs_next"].append(env.next_state)
        rows["reward"].append(float(env.reward))
        rows["flag"].append(env.terminal_flag)
        rows["done"].append(int(env.is_terminal))
    out = {k: np.array(v) for k, v in rows.items()}
    out["action"] = out["action"].astype(np.float32)
    np.savez(os.path.join(OUT, f"{key}.npz"), **out)
    print(key, "flags", np.bincount(out["flag"]))


def gen_angleonly_env(key="angleonly_env", n=500):
    """environment/CartPole/CartPoleAngleOnly.py: dt 0.01 in `while time < tt` sub-steps of
    dt/10 (10 or 11 by step index: the time table comes from the env's own rk44), flag 1 before
    flag 3, the angle-increment reward (incl. the `==` branch: an env at rest stays put)."""
    g = np.random.default_rng(20263)
    mod = mods["ao_env"]
    env = mod.CartPoleAngleOnly(0.)
    env.reset(False)
    tt = []
    for _ in range(606):
        tt.append(env.time)
        env.rk44(np.array([np.float32(0.)]))
    rows = {k: [] for k in ("state", "action", "state_next", "obs_cur", "obs_next", "reward",
                            "flag", "done")}
    th_hi = env.thetaMax + np.pi / 180
    for i in range(n):
        k = int(g.integers(0, 606))
        th, dth = g.uniform(-0.85, 0.85), g.uniform(-4, 4)
        x, dx = g.uniform(-2, 2), g.uniform(-2, 2)
        a = np.float32(g.uniform(-8, 8))
        j = i % 8
        if j == 1:    # angle bound straddled
            th = np.sign(g.uniform(-1, 1)) * (th_hi + g.uniform(-2e-3, 2e-3)); dth = g.uniform(-0.05, 0.05)
        elif j == 2:  # time-out regime
            k = int(g.integers(596, 606))
        elif j == 3:  # angle out AND time out: flag 1 wins here
            k = int(g.integers(598, 606)); th = np.sign(g.uniform(-1, 1)) * (th_hi + 0.05)
        elif j == 4:  # inside 0.5 deg
            th, dth = g.uniform(-0.008, 0.008), g.uniform(-0.02, 0.02)
        elif j == 5:  # at rest: theta unchanged, the `==` branch
            th, dth, x, dx, a = 0., 0., g.uniform(-1, 1), 0., np.float32(0.)
        with quiet():
            env.reset(False)
            env.theta, env.dtheta, env.x, env.dx, env.time = th, dth, x, dx, tt[k]
            rows["state"].append([th, dth, x, dx, tt[k]])
            env.step_update(np.array([a], dtype=np.float32))
        rows["action"].append([a])
        rows["state_next"].append([env.theta, env.dtheta, env.x, env.dx, env.time])
        rows["obs_cur"].append(env.current_state)
        rows["obs_next"].append(env.next_state)
        rows["reward"].append(float(env.reward))
        rows["flag"].append(env.terminal_flag)
        rows["done"].append(int(env.is_terminal))
    out = {k: np.array(v) for k, v in rows.items()}
    out["action"] = out["action"].astype(np.float32)
    out["time_table"] = np.array(tt)
    np.savez(os.path.join(OUT, f"{key}.npz"), **out)
    print(key, "flags", np.bincount(out["flag"]), "rewards", np.unique(out["reward"]))


def gen_soi(key, mod, n=400):
    env = mod.SecondOrderIntegration()
    rows = {k: [] for k in ("state", "action", "state_next", "obs_cur", "obs_next", "reward",
                            "flag", "done")}
    for i in range(n):
        k = int(rng.integers(0, 252))
        tm = 0.
        for _ in range(k):
            tm += env.dt
        pos = rng.uniform(-0.1, 5.1, 2)
        vel = rng.uniform(-3, 3, 2)
        if i % 5 == 1:
            pos = np.array([2.5, 2.5]) + rng.uniform(-0.03, 0.03, 2); vel = rng.uniform(-0.03, 0.03, 2)
        elif i % 5 == 2:
            k = int(rng.integers(245, 252))
        a = f32(rng.uniform(-3, 3, 2))
        with quiet():
            env.reset(False)
            env.pos = pos.copy(); env.vel = vel.copy(); env.time = tm
            env.target = np.array([2.5, 2.5])
            rows["state"].append([pos[0], pos[1], vel[0], vel[1], tm, 2.5, 2.5])
            env.step_update(a)
        rows["action"].append(a)
        rows["state_next"].append([env.pos[0], env.pos[1], env.vel[0], env.vel[1], env.time,
                                   env.target[0], env.target[1]])
        rows["obs_cur"].append(env.current_state)
        rows["obs_next"].append(env.next_state)
        rows["reward"].append(float(env.reward))
        rows["flag"].append(env.terminal_flag)
        rows["done"].append(int(env.is_terminal))
    out = {k: np.array(v) for k, v in rows.items()}
    out["action"] = out["action"].astype(np.float32)
    np.savez(os.path.join(OUT, f"{key}.npz"), **out)
    print(key, "flags", np.bincount(out["flag"]))


def gen_ugv(key, cls, n=400):
    env = cls()
    rows = {k: [] for k in ("state", "action", "state_next", "obs_cur", "obs_next", "reward",
                            "flag", "done")}
    for i in range(n):
        k = int(rng.integers(0, 502))
        tm = 0.
        for _ in range(k):
            tm += env.dt
        pos = rng.uniform(-0.05, 5.05, 2)
        vel = rng.uniform(-1, 3)
        phi = rng.uniform(-np.pi, np.pi)
        om = rng.uniform(-3, 3)
        if i % 6 == 1:
            pos = np.array([2.5, 2.5]) + rng.uniform(-0.04, 0.04, 2); vel = rng.uniform(-0.02, 0.02)
        elif i % 6 == 2:
            k = int(rng.integers(250, 502))
            tm = 0.
            for _ in range(k):
                tm += env.dt
        elif i % 6 == 3:
            phi = np.sign(rng.uniform(-1, 1)) * (np.pi - rng.uniform(0, 0.02)); om = 3 * np.sign(phi)
        a = f32([rng.uniform(-3, 3), rng.uniform(-2 * np.pi, 2 * np.pi)])
        with quiet():
            env.reset(False)
            env.pos = pos.copy(); env.vel = vel; env.phi = phi; env.omega = om; env.time = tm
            env.target = np.array([2.5, 2.5])
            rows["state"].append([pos[0], pos[1], vel, phi, om, tm, 2.5, 2.5])
            env.step_update(a)
        rows["action"].append(a)
        rows["state_next"].append([env.pos[0], env.pos[1], env.vel, env.phi, env.omega, env.time,
                                   env.target[0], env.target[1]])
        rows["obs_cur"].append(env.current_state)
        rows["obs_next"].append(env.next_state)
        rows["reward"].append(float(env.reward))
        rows["flag"].append(env.terminal_flag)
        rows["done"].append(int(env.is_terminal))
    out = {k: np.array(v) for k, v in rows.items()}
    out["action"] = out["action"].astype(np.float32)
    np.savez(os.path.join(OUT, f"{key}.npz"), **out)
    print(key, "flags", np.bincount(out["flag"]))


# ---------------------------------------------------------------------------------------------
# UAV hover outer loop (params of demonstration/PPO/PPO-4-UavHoverOuterLoop/train.py:24-56)
# ---------------------------------------------------------------------------------------------
def make_uav():
    up = uav_param()
    up.m = 0.8; up.g = 9.8; up.J = np.array([4.212e-3, 4.212e-3, 8.255e-3]); up.d = 0.12
    up.CT = 2.168e-6; up.CM = 2.136e-8; up.J0 = 1.01e-5; up.kr = 1e-3; up.kt = 1e-3
    up.pos0 = np.array([0, 0, 0]); up.vel0 = np.array([0, 0, 0]); up.angle0 = np.array([0, 0, 0])
    up.pqr0 = np.array([0, 0, 0]); up.dt = 0.01; up.time_max = 10
    up.pos_zone = np.atleast_2d([[-5, 5], [-5, 5], [0, 5]])
    ap = fntsmc_param()
    ap.k1 = np.array([25, 25, 40]); ap.k2 = np.array([0.1, 0.1, 0.2])
    ap.alpha = np.array([2.5, 2.5, 2.5]); ap.beta = np.array([0.99, 0.99, 0.99])
    ap.gamma = np.array([1.5, 1.5, 1.2]); ap.lmd = np.array([2.0, 2.0, 2.0]); ap.dim = 3
    ap.dt = 0.01; ap.ctrl0 = np.array([0., 0., 0.]); ap.saturation = np.array([0.3, 0.3, 0.3])
    with quiet():
        env = uav_mod.uav_hover_outer_loop(up, fntsmc_param(), ap, target0=np.array([-1, 3, 2]))
    env.msg_print_flag = False
    return env


def uav_full_state(env):
    return np.concatenate([env.uav_state_call_back(), [env.time], env.pos_ref, env.att_ctrl.s1,
                           env.att_ref])


def gen_uav(key, n_seq=24, seq_len=60):
    env = make_uav()
    seqs = {k: [] for k in ("state", "action", "state_next", "obs_cur", "obs_next", "reward",
                            "flag", "done")}
    for q in range(n_seq):
        with quiet():
            env.reset(random=True)
        # perturb the fresh episode so both calm and aggressive regimes are covered
        env.x, env.y, env.z = rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(0.5, 3)
        env.vx, env.vy, env.vz = rng.uniform(-1, 1, 3)
        env.phi, env.theta, env.psi = rng.uniform(-0.3, 0.3, 3)
        env.p, env.q, env.r = rng.uniform(-1, 1, 3)
        env.att_ctrl.s1 = rng.uniform(-0.2, 0.2, 3)
        env.att_ref = rng.uniform(-0.2, 0.2, 3)
        if q % 6 == 1:  # heading for the floor: position-out (flag 2)
            env.z, env.vz = rng.uniform(0.02, 0.2), -1.5
        elif q % 6 == 2:  # rolling hard: attitude-out (flag 3)
            env.phi, env.p = 0.7, 4.0
        elif q % 6 == 4:  # yawing past the +-120 deg zone
            env.psi, env.r = 2.05, 3.0
        env.error = env.uav_pos() - env.pos_ref
        if q % 4 == 3:
            t0 = 0.
            for _ in range(1000 - seq_len // 2):
                t0 += env.dt
            env.time = t0
        for t in range(seq_len):
            a = f32(rng.uniform(-8, 8, 3)) if q % 2 else f32(rng.uniform(-2, 2, 3))
            seqs["state"].append(uav_full_state(env))
            with quiet():
                env.step_update(a)
            seqs["action"].append(a)
            seqs["state_next"].append(uav_full_state(env))
            seqs["obs_cur"].append(env.current_state)
            seqs["obs_next"].append(env.next_state)
            seqs["reward"].append(float(env.reward))
            seqs["flag"].append(env.terminal_flag)
            seqs["done"].append(int(env.is_terminal))
            if env.is_terminal:
                break
    out = {k: np.array(v) for k, v in seqs.items()}
    out["action"] = out["action"].astype(np.float32)
    np.savez(os.path.join(OUT, f"{key}.npz"), **out)
    print(key, out["state"].shape, "flags", np.bincount(out["flag"]))


# ---------------------------------------------------------------------------------------------
# Shipped PPO2-CartPole nets: forward, choose_action, closed-loop known answer
# ---------------------------------------------------------------------------------------------
def gen_nets():
    net_dir = os.path.join(REF, "demonstration/PPO2/PPO2-4-CartPole/datasave/net")
    env = mods["cp_ppo2"].CartPole(0., 0.)
    actor = drv.PPOActor_Gaussian(state_dim=4, action_dim=1,
                                  a_min=np.array(env.action_range)[:, 0],
                                  a_max=np.array(env.action_range)[:, 1], init_std=env.fm / 3,
                                  use_orthogonal_init=True)
    critic = drv.PPOCritic(state_dim=4, use_orthogonal_init=True)
    actor.load_state_dict(torch.load(os.path.join(net_dir, "actor"), weights_only=True))
    critic.load_state_dict(torch.load(os.path.join(net_dir, "critic"), weights_only=True))
    flat = lambda m: torch.cat([p.detach().flatten() for p in m.parameters()]).numpy()
    x = f32(rng.uniform(-2.2, 2.2, (512, 4)))
    x[0] = [0.1, -0.2, 0.3, 0.05]
    with torch.no_grad():
        xa = torch.tensor(x)
        pre = actor.mean_layer(torch.tanh(actor.fc2(torch.tanh(actor.fc1(xa)))))
        mean = actor(xa).numpy()
        v = critic(xa).numpy()
    # choose_action samples (torch RNG), via the reference agent
    ppo_msg = {'gamma': 0.999, 'K_epochs': 30, 'eps_clip': 0.2, 'buffer_size': 1000,
               'state_dim': 4, 'action_dim': 1, 'a_lr': 3e-4, 'c_lr': 1e-3, 'set_adam_eps': True,
               'lmd': 0.95, 'use_adv_norm': True, 'mini_batch_size': 64, 'entropy_coef': 0.01,
               'use_grad_clip': False, 'use_lr_decay': False, 'max_train_steps': int(5e6),
               'using_mini_batch': False}
    env_msg = {'state_dim': 4, 'action_dim': 1, 'name': 'CartPole', 'action_range': env.action_range}
    agent = ppo2_mod.Proximal_Policy_Optimization2(env_msg, ppo_msg, actor=actor, critic=critic)
    torch.manual_seed(11)
    sa, slp = [], []
    for i in range(256):
        a, lp = agent.choose_action(x[i].astype(np.float64))
        sa.append(a); slp.append(lp)
    # closed loop, deterministic actor (SURVEY §4 known answers)
    loops = {}
    for name, (th0, x0) in {"a": (0.3, 0.5), "b": (-0.2, -0.6)}.items():
        e = mods["cp_ppo2"].CartPole(th0, x0)
        e.reset(False)
        obs, acts, rews, flags = [], [], [], []
        while not e.is_terminal:
            e.current_state = e.next_state.copy()
            a = agent.evaluate(e.current_state)
            obs.append(e.current_state); acts.append(a)
            e.step_update(a)
            rews.append(e.reward); flags.append(e.terminal_flag)
        loops[name] = dict(obs=np.array(obs), action=np.array(acts, np.float32),
                           reward=np.array(rews), flag=np.array(flags), init=np.array([th0, x0]))
        print("closed loop", name, len(rews), "steps, return %.6f" % np.sum(rews))
    np.savez(os.path.join(OUT, "ppo2_cartpole_nets.npz"), actor_params=flat(actor),
             critic_params=flat(critic), x=x, actor_pre=pre.numpy(), actor_mean=mean,
             critic_v=v, sample_a=np.array(sa), sample_logp=np.array(slp), std=np.float32(env.fm / 3),
             **{f"loop_{k}_{q}": v for k, d in loops.items() for q, v in d.items()})


# ---------------------------------------------------------------------------------------------
# PPO2.learn GAE / v_target / adv-norm, via the reference's own learn() with probes
# ---------------------------------------------------------------------------------------------
class _TorchProbe:
    """Stands in for the `torch` name inside the reference PPO2 module to observe learn()'s
    intermediate tensors (GAE list, normalised advantage); everything else is real torch."""

    def __init__(self, rec):
        self._rec = rec

    def __getattr__(self, name):
        return getattr(torch, name)

    def tensor(self, data, *a, **k):
        if isinstance(data, list):
            self._rec["gae_list"] = np.array([float(d) for d in data], np.float32)
        return torch.tensor(data, *a, **k)

    def min(self, a, b):
        self._rec.setdefault("adv_norm", a.detach().numpy().copy())
        return torch.min(a, b)


class _TableCritic(torch.nn.Module):
    def __init__(self, table):
        super().__init__()
        self.table = torch.tensor(table, dtype=torch.float32)
        self.w = torch.nn.Parameter(torch.zeros(1))

    def forward(self, s):
        return self.table[s[:, 0].long()].view(-1, 1) + 0 * self.w


class _ConstActor(torch.nn.Module):
    """get_dist(s).log_prob(a) returns the stored a_lp exactly => ratios == 1, surr1 == adv."""

    def __init__(self, a_lp):
        super().__init__()
        self.a_lp = torch.tensor(a_lp, dtype=torch.float32)
        self.w = torch.nn.Parameter(torch.zeros(1))

    def get_dist(self, s):
        outer = self

        class D:
            def entropy(self):
                return torch.zeros(len(s), 1) + 0 * outer.w

            def log_prob(self, a):
                return outer.a_lp + 0 * outer.w
        return D()


def gen_gae(n_cases=4, B=1000):
    cases = []
    for c in range(n_cases):
        r = rng.normal(0, 1, B)
        v = f32(rng.normal(40, 5, B))
        vn = f32(rng.normal(40, 5, B))
        done = (rng.uniform(0, 1, B) < [0.004, 0.02, 0.1, 0.3][c]).astype(np.float64)
        success = done * (rng.uniform(0, 1, B) < 0.5)
        if c == 3:
            success = (rng.uniform(0, 1, B) < 0.7).astype(np.float64)  # DPPO2 rule: also non-terminal
        rec = {}
        ppo_msg = {'gamma': 0.999, 'K_epochs': 1, 'eps_clip': 0.2, 'buffer_size': B,
                   'state_dim': 1, 'action_dim': 1, 'a_lr': 3e-4, 'c_lr': 1e-3,
                   'set_adam_eps': True, 'lmd': 0.95, 'use_adv_norm': True,
                   'mini_batch_size': 64, 'entropy_coef': 0.01, 'use_grad_clip': False,
                   'use_lr_decay': False, 'max_train_steps': int(5e6), 'using_mini_batch': False}
        env_msg = {'state_dim': 1, 'action_dim': 1, 'name': 'gae', 'action_range': [[-1, 1]]}
        a_lp = rng.normal(0, 1, (B, 1))
        table = np.concatenate([v, vn])
        agent = ppo2_mod.Proximal_Policy_Optimization2(env_msg, ppo_msg, actor=_ConstActor(a_lp),
                                                       critic=_TableCritic(table))
        for i in range(B):
            agent.buffer.append(s=np.array([i]), a=np.array([0.]), log_prob=a_lp[i], r=r[i],
                                s_=np.array([B + i]), done=done[i], success=success[i], index=i)
        real = ppo2_mod.torch
        ppo2_mod.torch = _TorchProbe(rec)
        try:
            agent.learn(0, buf_num=1)
        finally:
            ppo2_mod.torch = real
        cases.append(dict(r=f32(r), v=v, vn=vn, done=done.astype(np.uint8),
                          success=success.astype(np.uint8), adv=rec["gae_list"],
                          v_target=(torch.tensor(rec["gae_list"]) + torch.tensor(v)).numpy(),
                          adv_norm=rec["adv_norm"].reshape(-1)))
    np.savez(os.path.join(OUT, "gae.npz"), gamma=0.999, lmd=0.95,
             **{f"c{i}_{k}": v for i, c in enumerate(cases) for k, v in c.items()})
    print("gae", len(cases), "cases")


def gen_reward_norm():
    norm = cls_mod.Normalization(shape=1)
    xs = np.concatenate([[-3., -1., -2.], rng.normal(-1, 2, 2000), rng.normal(-50, 30, 300)])
    out = np.array([np.asarray(norm(x)).item() for x in xs])
    np.savez(os.path.join(OUT, "reward_norm.npz"), x=xs, y=out)
    print("reward_norm", out[:3])


def gen_replay():
    """ReplayBuffer (utils/classes.py:189-247): ring overwrite, end = 1 - done, stable ascending
    reward sort (ties included)."""
    rb = cls_mod.ReplayBuffer(10, 4, 2, 1)
    n = 23
    s = rng.normal(size=(n, 2))
    a = rng.uniform(-3, 3, size=(n, 1))
    r = np.round(rng.normal(size=n), 1)        # rounded: equal rewards exercise the stable sort
    s2 = rng.normal(size=(n, 2))
    d = (rng.uniform(size=n) < 0.3).astype(float)
    for i in range(n):
        rb.store_transition(s[i], a[i], r[i], s2[i], d[i])
    with quiet():
        rb.get_reward_sort()
    np.savez(os.path.join(OUT, "replay.npz"), s=s, a=a, r=r, s2=s2, d=d, s_mem=rb.s_mem,
             a_mem=rb.a_mem, r_mem=rb.r_mem, s2_mem=rb._s_mem, end_mem=rb.end_mem,
             mem_counter=rb.mem_counter, sorted_index=np.asarray(rb.sorted_index))
    print("replay", rb.mem_counter, rb.sorted_index[:5])


def gen_ddpg():
    """One DDPG.learn step (algorithm/actor_critic/DDPG.py:72-109) with the DDPG-SOI driver's nets
    (demonstration/DDPG/DDPG-4-SecondOrderIntegration/train.py:26-100) on a fixed batch."""
    with quiet():
        drv_d = load("demonstration/DDPG/DDPG-4-SecondOrderIntegration/train.py", "ref_ddpg_soi_train")
        ddpg_mod = load("algorithm/actor_critic/DDPG.py", "ref_ddpg")
    torch.manual_seed(11)
    lo, hi = np.array([-3., -3.]), np.array([3., 3.])
    nets = [drv_d.Actor(1e-4, 4, 2, lo, hi), drv_d.Actor(1e-4, 4, 2, lo, hi),
            drv_d.Critic(3e-4, 4, 2), drv_d.Critic(3e-4, 4, 2)]
    env_msg = {'state_dim': 4, 'action_dim': 2, 'action_range': np.stack([lo, hi], 1), 'name': 'SOI'}
    agent = ddpg_mod.DDPG(env_msg=env_msg, gamma=0.99, actor_soft_update=0.005,
                          critic_soft_update=0.005, memory_capacity=10000, batch_size=64,
                          actor=nets[0], target_actor=nets[1], critic=nets[2], target_critic=nets[3])
    flat = lambda m: torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy().copy()
    before = {k: flat(m) for k, m in zip(("actor", "target_actor", "critic", "target_critic"),
                                         (agent.actor, agent.target_actor, agent.critic,
                                          agent.target_critic))}
    B = 64
    batch = (rng.uniform(-2, 2, (B, 4)), rng.uniform(-3, 3, (B, 2)), rng.normal(size=B),
             rng.uniform(-2, 2, (B, 4)), (rng.uniform(size=B) > 0.1).astype(np.float32))
    agent.memory.mem_counter = 10000
    agent.memory.sample_buffer = lambda is_reward_ascent=True, has_log_prob=False: batch
    agent.learn(is_reward_ascent=False, iter=1)
    after = {k: flat(m) for k, m in zip(("actor", "target_actor", "critic", "target_critic"),
                                        (agent.actor, agent.target_actor, agent.critic,
                                         agent.target_critic))}
    np.savez(os.path.join(OUT, "ddpg_soi_learn.npz"), s=batch[0], a=batch[1], r=batch[2],
             s2=batch[3], end=batch[4], **{f"before_{k}": v for k, v in before.items()},
             **{f"after_{k}": v for k, v in after.items()})
    print("ddpg", {k: float(np.abs(after[k] - before[k]).max()) for k in after})


# ---------------------------------------------------------------------------------------------
# UGV forward obstacle avoidance: maps from the reference's own generator (reset(True)), then
# teacher-forced states (near obstacles, walls, the target, the time limit, axis-aligned beams)
# ---------------------------------------------------------------------------------------------
OA_NOBS = 15


def oa_full_state(env):
    st = [env.pos[0], env.pos[1], env.vel, env.phi, env.omega, env.time, env.target[0],
          env.target[1]]
    obs = [[o[1][0], o[1][1], o[2][0]] for o in env.obs]
    for k in range(len(obs), OA_NOBS):
        obs.append([-1000.0 - 10.0 * k, -1000.0, 0.2])   # parked slot (never seen, never hit)
    return st + [v for o in obs for v in o]


def _alarm(signum, frame):
    raise TimeoutError


def gen_ugvoa(key, n=400):
    signal.signal(signal.SIGALRM, _alarm)
    cls = mods[key].UGVForwardObstacleAvoidance
    env = None
    while env is None:
        try:
            signal.alarm(2)
            with quiet():
                env = cls()
        except TimeoutError:
            pass
        finally:
            signal.alarm(0)
    rows = {k: [] for k in ("state", "action", "state_next", "obs_cur", "obs_next", "reward",
                            "flag", "done")}
    maps = []
    for i in range(n):
        while True:    # the reference's rejection sampler can loop forever (obsNum 15): retry
            try:
                signal.alarm(2)
                with quiet():
                    env.reset(True)
                break
            except TimeoutError:
                continue
            finally:
                signal.alarm(0)
        obs = env.obs
        maps.append([[o[1][0], o[1][1], o[2][0]] for o in obs])
        k = int(rng.integers(0, int(env.time_max / env.dt) + 2))
        tm = 0.
        for _ in range(k):
            tm += env.dt
        pos = rng.uniform(-0.05, 5.05, 2)
        vel = rng.uniform(-0.5, 3)
        phi = rng.uniform(-np.pi, np.pi)
        om = rng.uniform(-3, 3)
        j = i % 8
        if j == 1:     # next to (or just inside) an obstacle: collision / blind beams
            c = obs[int(rng.integers(0, len(obs)))]
            ang = rng.uniform(-np.pi, np.pi)
            d = c[2][0] + env.r_vehicle + rng.uniform(-0.03, 0.05)
            pos = np.array(c[1]) + d * np.array([np.cos(ang), np.sin(ang)])
        elif j == 2:   # at the target, slow: success
            pos = env.target + rng.uniform(-0.04, 0.04, 2); vel = rng.uniform(-0.02, 0.02)
            om = rng.uniform(-0.02, 0.02)
        elif j == 3:   # beams exactly axis-aligned (tan of +-pi/2: the |m| >= 1e8 branches)
            phi = float(rng.choice([0.0, np.pi / 2, -np.pi / 2, np.pi, -np.pi]))
        elif j == 4:   # near a wall / corner, heading out
            pos = rng.choice([0.02, 4.98], 2) + rng.uniform(-0.02, 0.02, 2)
        elif j == 5:   # time limit
            k = int(rng.integers(int(env.time_max / env.dt) - 3, int(env.time_max / env.dt) + 2))
            tm = 0.
            for _ in range(k):
                tm += env.dt
        elif j == 6:   # inside the lidar range of several obstacles
            c = obs[int(rng.integers(0, len(obs)))]
            pos = np.array(c[1]) + rng.uniform(-1.2, 1.2, 2)
        a = f32([rng.uniform(-3, 3), rng.uniform(-2 * np.pi, 2 * np.pi)])
        with quiet():
            env.pos = pos.copy(); env.vel = vel; env.phi = phi; env.omega = om; env.time = tm
            rows["state"].append(oa_full_state(env))
            env.step_update(a)
        rows["action"].append(a)
        rows["state_next"].append(oa_full_state(env))
        rows["obs_cur"].append(env.current_state)
        rows["obs_next"].append(env.next_state)
        rows["reward"].append(float(env.reward))
        rows["flag"].append(env.terminal_flag)
        rows["done"].append(int(env.is_terminal))
    out = {k: np.array(v) for k, v in rows.items()}
    out["action"] = out["action"].astype(np.float32)
    out["maps"] = np.array(maps)
    np.savez_compressed(os.path.join(OUT, f"{key}.npz"), **out)
    print(key, "flags", np.bincount(out["flag"]))


# ---------------------------------------------------------------------------------------------
# SAC: the squashed-Gaussian actor head (utils/classes.py SACActor and the SAC demo copy) and two
# SAC.learn updates (algorithm/actor_critic/Soft_Actor_Critic.py:70-124), Normal.rsample's noise
# recorded so the device code can replay it
# ---------------------------------------------------------------------------------------------
class _EpsTape:
    def __init__(self, replay=None):
        self.tape, self.replay = [], replay
        self.orig = torch.distributions.Normal.rsample

    def __enter__(self):
        tape = self

        def rsample(dist, sample_shape=torch.Size()):
            shape = dist._extended_shape(sample_shape)
            eps = tape.replay.pop(0) if tape.replay is not None else torch.randn(shape)
            tape.tape.append(eps.clone())
            return dist.loc + eps * dist.scale
        torch.distributions.Normal.rsample = rsample
        return self

    def __exit__(self, *a):
        torch.distributions.Normal.rsample = self.orig


def gen_sac():
    with quiet():
        drv_s = load("demonstration/SAC/SAC-4-UGVForward/train.py", "ref_sac_ugvf_train")
        sac_mod = load("algorithm/actor_critic/Soft_Actor_Critic.py", "ref_sac")
    torch.manual_seed(13)
    S, A, B = 41, 2, 64
    lo, hi = np.array([-3., -2 * np.pi]), np.array([3., 2 * np.pi])
    out = {}
    # actor heads: utils.classes.SACActor (clamp -20, 2) and the demo copy (per-dim clamp)
    for key, actor in (("utils", cls_mod.SACActor(S, A, lo, hi)),
                       ("demo", drv_s.SACActor(S, A, lo, hi, std_scale=1.))):
        with torch.no_grad():   # spread log_std over both clamp bounds
            actor.log_std_layer.weight.mul_(4000.0)
            actor.mean_layer.weight.mul_(100.0)
        x = torch.tensor(rng.uniform(-1, 1, (512, S)), dtype=torch.float)
        with torch.no_grad(), _EpsTape() as tp:
            a, lp = actor(x)
            a_det, _ = actor(x, deterministic=True, with_logprob=False)
        out[f"{key}_params"] = torch.cat([p.detach().reshape(-1) for p in actor.parameters()]).numpy()
        out[f"{key}_x"], out[f"{key}_eps"] = x.numpy(), tp.tape[0].numpy()
        out[f"{key}_a"], out[f"{key}_logpi"], out[f"{key}_a_det"] = a.numpy(), lp.numpy(), a_det.numpy()
    # two learn() iterations with the demo nets
    actor = drv_s.SACActor(S, A, lo, hi, std_scale=1.)
    critic, target = drv_s.SACCritic(S, A), drv_s.SACCritic(S, A)
    env_msg = {'state_dim': S, 'action_dim': A, 'action_range': np.stack([lo, hi], 1), 'name': 'OA'}
    agent = sac_mod.SAC(env_msg=env_msg, gamma=0.99, critic_tau=0.005, memory_capacity=10000,
                        batch_size=B, actor=actor, critic=critic, target_critic=target, a_lr=1e-4,
                        c_lr=1e-4, alpha_lr=1e-4, adaptive_alpha=True)
    flat = lambda m: torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy().copy()
    for k, m in (("actor", agent.actor), ("critic", agent.critic), ("target_critic", agent.target_critic)):
        out[f"before_{k}"] = flat(m)
    batches = []
    for it in range(2):
        batches.append((rng.uniform(-1, 1, (B, S)), rng.uniform(lo, hi, (B, A)), rng.normal(size=B),
                        rng.uniform(-1, 1, (B, S)), (rng.uniform(size=B) < 0.1).astype(np.float32)))
    agent.memory.mem_counter = 10000
    agent.memory.sample_buffer = lambda is_reward_ascent=True, has_log_prob=False: batches.pop(0)
    keep = [tuple(np.array(x) for x in b) for b in batches]
    with _EpsTape() as tp:
        agent.learn(is_reward_ascent=False, iter=2)
    for k, m in (("actor", agent.actor), ("critic", agent.critic), ("target_critic", agent.target_critic)):
        out[f"after_{k}"] = flat(m)
    out["after_log_alpha"] = agent.log_alpha.detach().numpy().copy()
    out["learn_eps"] = np.stack([e.numpy() for e in tp.tape])
    for i, b in enumerate(keep):
        for name, v in zip(("s", "a", "r", "s2", "dw"), b):
            out[f"b{i}_{name}"] = v
    np.savez_compressed(os.path.join(OUT, "sac.npz"), **out)
    print("sac", len(tp.tape), float(out["after_log_alpha"][0]),
          {k: float(np.abs(out[f"after_{k}"] - out[f"before_{k}"]).max())
           for k in ("actor", "critic", "target_critic")})


def _grad_tap(grads, name, opt, params):
    """Record the .grad every parameter of `params` holds when `opt.step()` is first called (a
    parameter without .grad is recorded as zeros: the optimizer skips it)."""
    step = opt.step

    def wrapped(*a, **k):
        if name not in grads:
            grads[name] = np.concatenate([
                (p.grad.detach().reshape(-1).numpy().copy() if p.grad is not None
                 else np.zeros(p.numel(), np.float32)) for p in params])
        return step(*a, **k)
    opt.step = wrapped


def gen_ddpg_grad():
    """DDPG.learn (algorithm/actor_critic/DDPG.py:72-109) once on a 1000-row batch with the
    DDPG-SOI driver's nets (demonstration/DDPG/DDPG-4-SecondOrderIntegration/train.py:26-100): the
    critic's and the actor's p.grad at their optimizer.step() (the actor's is taken through the
    critic after its Adam step, as learn() does), plus before / after weights. Own RNG streams."""
    g = np.random.default_rng(20264)
    with quiet():
        drv_d = load("demonstration/DDPG/DDPG-4-SecondOrderIntegration/train.py", "ref_ddpg_soi_train")
        ddpg_mod = load("algorithm/actor_critic/DDPG.py", "ref_ddpg")
    torch.manual_seed(23)
    lo, hi = np.array([-3., -3.]), np.array([3., 3.])
    nets = [drv_d.Actor(1e-4, 4, 2, lo, hi), drv_d.Actor(1e-4, 4, 2, lo, hi),
            drv_d.Critic(3e-4, 4, 2), drv_d.Critic(3e-4, 4, 2)]
    env_msg = {'state_dim': 4, 'action_dim': 2, 'action_range': np.stack([lo, hi], 1), 'name': 'SOI'}
    B = 1000
    agent = ddpg_mod.DDPG(env_msg=env_msg, gamma=0.99, actor_soft_update=0.005,
                          critic_soft_update=0.005, memory_capacity=10000, batch_size=B,
                          actor=nets[0], target_actor=nets[1], critic=nets[2], target_critic=nets[3])
    names = ("actor", "target_actor", "critic", "target_critic")
    mods_ = (agent.actor, agent.target_actor, agent.critic, agent.target_critic)
    before = {k: _flat(m) for k, m in zip(names, mods_)}
    batch = (g.uniform(-2, 2, (B, 4)), g.uniform(-3, 3, (B, 2)), g.normal(size=B),
             g.uniform(-2, 2, (B, 4)), (g.uniform(size=B) > 0.1).astype(np.float32))
    agent.memory.mem_counter = 10000
    agent.memory.sample_buffer = lambda is_reward_ascent=True, has_log_prob=False: batch
    grads = {}
    _grad_tap(grads, "critic", agent.critic.optimizer, list(agent.critic.parameters()))
    _grad_tap(grads, "actor", agent.actor.optimizer, list(agent.actor.parameters()))
    agent.learn(is_reward_ascent=False, iter=1)
    after = {k: _flat(m) for k, m in zip(names, mods_)}
    np.savez_compressed(os.path.join(OUT, "ddpg_soi_grad.npz"), s=batch[0], a=batch[1], r=batch[2],
                        s2=batch[3], end=batch[4], **{f"before_{k}": v for k, v in before.items()},
                        **{f"after_{k}": v for k, v in after.items()},
                        **{f"grad_{k}": v for k, v in grads.items()})
    print("ddpg_grad", {k: float(np.abs(v).max()) for k, v in grads.items()})


def gen_sac_grad():
    """SAC.learn (algorithm/actor_critic/Soft_Actor_Critic.py:70-124) once on a 1000-row batch
    with the SAC-UGVForward demo's nets (demonstration/SAC/SAC-4-UGVForward/train.py:32-120, 41
    inputs), the log_std layer scaled so rows reach both clamp bounds: the actor's, critic's and
    log_alpha's p.grad at their optimizer.step(), Normal.rsample's noise (both draws), before /
    after weights. Own RNG streams."""
    g = np.random.default_rng(20265)
    with quiet():
        drv_s = load("demonstration/SAC/SAC-4-UGVForward/train.py", "ref_sac_ugvf_train")
        sac_mod = load("algorithm/actor_critic/Soft_Actor_Critic.py", "ref_sac")
    torch.manual_seed(29)
    S, A, B = 41, 2, 1000
    lo, hi = np.array([-3., -2 * np.pi]), np.array([3., 2 * np.pi])
    actor = drv_s.SACActor(S, A, lo, hi, std_scale=1.)
    with torch.no_grad():
        actor.log_std_layer.weight.mul_(1500.0)
        actor.mean_layer.weight.mul_(30.0)
    critic, target = drv_s.SACCritic(S, A), drv_s.SACCritic(S, A)
    env_msg = {'state_dim': S, 'action_dim': A, 'action_range': np.stack([lo, hi], 1), 'name': 'OA'}
    agent = sac_mod.SAC(env_msg=env_msg, gamma=0.99, critic_tau=0.005, memory_capacity=10000,
                        batch_size=B, actor=actor, critic=critic, target_critic=target, a_lr=1e-4,
                        c_lr=1e-4, alpha_lr=1e-4, adaptive_alpha=True)
    out = {f"before_{k}": _flat(m) for k, m in (("actor", agent.actor), ("critic", agent.critic),
                                                ("target_critic", agent.target_critic))}
    out["before_log_alpha"] = agent.log_alpha.detach().numpy().copy()
    batch = (g.uniform(-1, 1, (B, S)), g.uniform(lo, hi, (B, A)), g.normal(size=B),
             g.uniform(-1, 1, (B, S)), (g.uniform(size=B) < 0.1).astype(np.float32))
    agent.memory.mem_counter = 10000
    agent.memory.sample_buffer = lambda is_reward_ascent=True, has_log_prob=False: batch
    grads = {}
    _grad_tap(grads, "actor", agent.actor_optimizer, list(agent.actor.parameters()))
    _grad_tap(grads, "critic", agent.critic_optimizer, list(agent.critic.parameters()))
    _grad_tap(grads, "log_alpha", agent.alpha_optimizer, [agent.log_alpha])
    with _EpsTape() as tp:
        agent.learn(is_reward_ascent=False, iter=1)
    for k, m in (("actor", agent.actor), ("critic", agent.critic), ("target_critic", agent.target_critic)):
        out[f"after_{k}"] = _flat(m)
    out["after_log_alpha"] = agent.log_alpha.detach().numpy().copy()
    out["eps"] = np.stack([e.numpy() for e in tp.tape])
    for name, v in zip(("s", "a", "r", "s2", "dw"), batch):
        out[name] = v
    out.update({f"grad_{k}": v for k, v in grads.items()})
    np.savez_compressed(os.path.join(OUT, "sac_grad.npz"), **out)
    print("sac_grad", len(tp.tape), {k: float(np.abs(v).max()) for k, v in grads.items()})


# ---------------------------------------------------------------------------------------------
# PPO2 learn() (Proximal_Policy_Optimization2.py:78-174) on a fixed buffer, the DPPO2 Worker's
# learn() (demonstration/DPPO2/DPPO2-4-CartPole/Distributed_PPO2.py:54-103), and N=1 driver
# transcripts (demonstration/PPO2/PPO2-4-{CartPole,CartPoleAngleOnly}/train.py:184-217). Each
# generator seeds its own RNGs, so it reproduces when run alone.
# ---------------------------------------------------------------------------------------------
def _flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy().copy()


class _RandpermTape:
    """Records the permutations SubsetRandomSampler draws (torch.randperm) inside learn()."""

    def __init__(self):
        self.perms, self.orig = [], torch.randperm

    def __enter__(self):
        tape = self

        def randperm(n, *a, **k):
            out = tape.orig(n, *a, **k)
            tape.perms.append(out.clone())
            return out
        torch.randperm = randperm
        return self

    def __exit__(self, *a):
        torch.randperm = self.orig


def _learn_buffer(g, B, S, actor, lp_noise):
    s = g.uniform(-2, 2, (B, S))
    with torch.no_grad():
        mean = actor(torch.tensor(s, dtype=torch.float))
        a = torch.clamp(mean + actor.std * torch.tensor(g.normal(size=mean.shape), dtype=torch.float),
                        actor.a_min, actor.a_max)
        lp = torch.distributions.Normal(mean, actor.std).log_prob(a).numpy().astype(np.float64)
    lp = lp + lp_noise * g.normal(size=lp.shape)      # old-policy log-probs: ratios off 1
    r = g.normal(-1, 2, B)
    s2 = s + 0.05 * g.normal(size=(B, S))
    done = (g.uniform(size=B) < 0.03).astype(np.float64)
    success = done * (g.uniform(size=B) < 0.5)
    return s, a.numpy().astype(np.float64), lp, r, s2, done, success


def gen_ppo2_learn():
    """Three learn() calls (K=3) on one 1000-row buffer with the PPO2-CartPole driver's nets
    (train.py:39-125): full batch; use_grad_clip=True; mini-batch (64) with the sampler's
    permutations recorded. The GAE / v_target / normalised advantages learn() feeds the epochs
    are recorded too (probes on the reference module's torch name)."""
    g = np.random.default_rng(20261)
    out = {}
    B = 1000
    for mode, over in (("full", {}), ("clip", {'use_grad_clip': True}),
                       ("mini", {'using_mini_batch': True})):
        torch.manual_seed(17)
        actor = drv.PPOActor_Gaussian(state_dim=4, action_dim=1, a_min=np.array([-8.]),
                                      a_max=np.array([8.]), init_std=8 / 3, use_orthogonal_init=True)
        critic = drv.PPOCritic(state_dim=4, use_orthogonal_init=True)
        with torch.no_grad():   # a last layer large enough for a non-trivial tanh'(z3)
            torch.nn.init.orthogonal_(actor.mean_layer.weight, gain=1.0)
        ppo_msg = {'gamma': 0.999, 'K_epochs': 3, 'eps_clip': 0.2, 'buffer_size': B,
                   'state_dim': 4, 'action_dim': 1, 'a_lr': 3e-4, 'c_lr': 1e-3,
                   'set_adam_eps': True, 'lmd': 0.95, 'use_adv_norm': True,
                   'mini_batch_size': 64, 'entropy_coef': 0.01, 'use_grad_clip': False,
                   'use_lr_decay': False, 'max_train_steps': int(5e6), 'using_mini_batch': False}
        ppo_msg.update(over)
        env_msg = {'state_dim': 4, 'action_dim': 1, 'name': 'CartPole', 'action_range': [[-8., 8.]]}
        agent = ppo2_mod.Proximal_Policy_Optimization2(env_msg, ppo_msg, actor=actor, critic=critic)
        s, a, lp, r, s2, done, success = _learn_buffer(g, B, 4, actor, 0.3)
        for i in range(B):
            agent.buffer.append(s=s[i], a=a[i], log_prob=lp[i], r=r[i], s_=s2[i], done=done[i],
                                success=success[i], index=i)
        before_a, before_c = _flat(actor), _flat(critic)
        with torch.no_grad():
            st = torch.tensor(s, dtype=torch.float)
            vs = critic(st)
        rec = {}
        real = ppo2_mod.torch
        ppo2_mod.torch = _TorchProbe(rec)
        grads = {}

        def _tap(name, opt, params):   # the .grad each optimiser step consumes (post-clip)
            step = opt.step

            def wrapped(*a, **k):
                if name not in grads:
                    grads[name] = np.concatenate([p.grad.detach().reshape(-1).numpy().copy()
                                                  for p in params])
                return step(*a, **k)
            opt.step = wrapped
        _tap("actor", agent.optimizer_actor, list(actor.parameters()))
        _tap("critic", agent.optimizer_critic, list(critic.parameters()))
        try:
            with _RandpermTape() as tape:
                agent.learn(0, buf_num=1)
        finally:
            ppo2_mod.torch = real
        adv = torch.tensor(rec["gae_list"]).view(-1, 1)
        v_target = adv + vs
        adv_n = (adv - adv.mean()) / (adv.std() + 1e-5)
        out.update({f"{mode}_s": s, f"{mode}_a": a, f"{mode}_a_lp": lp, f"{mode}_r": r,
                    f"{mode}_s_": s2, f"{mode}_done": done, f"{mode}_success": success,
                    f"{mode}_before_actor": before_a, f"{mode}_before_critic": before_c,
                    f"{mode}_after_actor": _flat(actor), f"{mode}_after_critic": _flat(critic),
                    f"{mode}_adv_norm": adv_n.numpy()[:, 0], f"{mode}_v_target": v_target.numpy()[:, 0],
                    # the reference's own first-step gradients (first epoch; mini: first batch)
                    f"{mode}_grad_actor": grads["actor"], f"{mode}_grad_critic": grads["critic"]})
        if mode == "mini":
            out["mini_perms"] = np.stack([p.numpy() for p in tape.perms])
        print("ppo2_learn", mode, "max |dW| actor %.3e critic %.3e" % (
            np.abs(out[f"{mode}_after_actor"] - before_a).max(),
            np.abs(out[f"{mode}_after_critic"] - before_c).max()), len(tape.perms), "perms")
    np.savez_compressed(os.path.join(OUT, "ppo2_learn.npz"), std=np.float32(8 / 3), **out)


def gen_ppo2_soi_learn():
    """learn() (K = 3, full batch) with the PPO2-SecondOrderIntegration demo's nets (actor
    4 -> 128 -> 64 -> 32 -> 2, critic 4 -> 64 -> 64 -> 1; demonstration/PPO2/
    PPO2-4-SecondOrderIntegration/train.py:37-125, ppo_msg :146-160 with K_epochs 3) on a 500-row
    buffer (the demo's buffer_size = time_max / dt * 2): the reference's first-step p.grad,
    the GAE / v_target / normalised advantages learn() computed, and the after-weights."""
    g = np.random.default_rng(20266)
    with quiet():
        drv_soi = load("demonstration/PPO2/PPO2-4-SecondOrderIntegration/train.py", "ref_ppo2_soi_train")
    torch.manual_seed(31)
    lo, hi = np.array([-3., -3.]), np.array([3., 3.])
    actor = drv_soi.PPOActor_Gaussian(state_dim=4, action_dim=2, a_min=lo, a_max=hi, init_std=1.0,
                                      use_orthogonal_init=True)
    critic = drv_soi.PPOCritic(state_dim=4, use_orthogonal_init=True)
    with torch.no_grad():   # a last layer large enough for a non-trivial tanh'(z)
        torch.nn.init.orthogonal_(actor.mean_layer.weight, gain=1.0)
    B = 500
    ppo_msg = {'gamma': 0.99, 'K_epochs': 3, 'eps_clip': 0.2, 'buffer_size': B, 'state_dim': 4,
               'action_dim': 2, 'a_lr': 3e-4, 'c_lr': 1e-3, 'set_adam_eps': True, 'lmd': 0.95,
               'use_adv_norm': True, 'mini_batch_size': 64, 'entropy_coef': 0.01,
               'use_grad_clip': False, 'use_lr_decay': False, 'max_train_steps': int(5e6),
               'using_mini_batch': False}
    env_msg = {'state_dim': 4, 'action_dim': 2, 'name': 'SecondOrderIntegration',
               'action_range': [[-3., 3.], [-3., 3.]]}
    agent = ppo2_mod.Proximal_Policy_Optimization2(env_msg, ppo_msg, actor=actor, critic=critic)
    s, a, lp, r, s2, done, success = _learn_buffer(g, B, 4, actor, 0.3)
    for i in range(B):
        agent.buffer.append(s=s[i], a=a[i], log_prob=lp[i], r=r[i], s_=s2[i], done=done[i],
                            success=success[i], index=i)
    before_a, before_c = _flat(actor), _flat(critic)
    with torch.no_grad():
        vs = critic(torch.tensor(s, dtype=torch.float))
    rec, grads = {}, {}
    _grad_tap(grads, "actor", agent.optimizer_actor, list(actor.parameters()))
    _grad_tap(grads, "critic", agent.optimizer_critic, list(critic.parameters()))
    real = ppo2_mod.torch
    ppo2_mod.torch = _TorchProbe(rec)
    try:
        agent.learn(0, buf_num=1)
    finally:
        ppo2_mod.torch = real
    adv = torch.tensor(rec["gae_list"]).view(-1, 1)
    v_target = adv + vs
    adv_n = (adv - adv.mean()) / (adv.std() + 1e-5)
    np.savez_compressed(os.path.join(OUT, "ppo2_soi_learn.npz"), s=s, a=a, a_lp=lp, r=r, s_=s2,
                        done=done, success=success, before_actor=before_a, before_critic=before_c,
                        after_actor=_flat(actor), after_critic=_flat(critic),
                        adv_norm=adv_n.numpy()[:, 0], v_target=v_target.numpy()[:, 0],
                        grad_actor=grads["actor"], grad_critic=grads["critic"], std=np.float32(1.0))
    print("ppo2_soi_learn", {k: float(np.abs(v).max()) for k, v in grads.items()})


def gen_ppo2_ugvoa_learn():
    """learn() with the PPO2-UGVForwardObstacleAvoidance demo's nets and K (actor / critic
    41 -> 256 -> 256 -> 2 / -> 1 tanh, demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/
    train.py:39-125; ppo_msg :144-162: K_epochs 25, a_lr 1e-4, c_lr 1e-3, full batch; init_std
    per action dim = range / 6, :164) on a 1 200-row buffer (the demo's buffer_size =
    time_max / dt * 4 = 15 / 0.05 * 4): the reference's first-step p.grad, the GAE / v_target /
    normalised advantages learn() computed, and the after-weights of the 25 epochs. Inputs:
    4 state features in [-2, 2] and 37 lidar ranges in [0, 2] (the laser_dis range)."""
    g = np.random.default_rng(20267)
    with quiet():
        drv_oa = load("demonstration/PPO2/PPO2-4-UGVForwardObstacleAvoidance/train.py",
                      "ref_ppo2_ugvoa_train")
    torch.manual_seed(37)
    S, A = 41, 2
    lo, hi = np.array([-3., -2 * np.pi]), np.array([3., 2 * np.pi])
    std0 = (hi - lo) / 2 / 3
    actor = drv_oa.PPOActor_Gaussian(state_dim=S, action_dim=A, a_min=lo, a_max=hi, init_std=std0,
                                     use_orthogonal_init=True)
    critic = drv_oa.PPOCritic(state_dim=S, use_orthogonal_init=True)
    with torch.no_grad():   # a last layer large enough for a non-trivial tanh'(z)
        torch.nn.init.orthogonal_(actor.mean_layer.weight, gain=1.0)
    B, K = 1200, 25
    ppo_msg = {'gamma': 0.99, 'K_epochs': K, 'eps_clip': 0.2, 'buffer_size': B, 'state_dim': S,
               'action_dim': A, 'a_lr': 1e-4, 'c_lr': 1e-3, 'set_adam_eps': True, 'lmd': 0.95,
               'use_adv_norm': True, 'mini_batch_size': 64, 'entropy_coef': 0.01,
               'use_grad_clip': False, 'use_lr_decay': False, 'max_train_steps': int(5e6),
               'using_mini_batch': False}
    env_msg = {'state_dim': S, 'action_dim': A, 'name': 'UGVForwardObstacleAvoidance',
               'action_range': np.stack([lo, hi], 1)}
    agent = ppo2_mod.Proximal_Policy_Optimization2(env_msg, ppo_msg, actor=actor, critic=critic)
    s, a, lp, r, s2, done, success = _learn_buffer(g, B, S, actor, 0.3)
    s[:, 4:] = (s[:, 4:] + 2) / 2          # lidar ranges in [0, 2]
    s2[:, 4:] = np.clip((s2[:, 4:] + 2) / 2, 0, 2)
    with torch.no_grad():   # the buffer's actions / log-probs for these inputs
        mean = actor(torch.tensor(s, dtype=torch.float))
        at = torch.clamp(mean + actor.std * torch.tensor(g.normal(size=mean.shape), dtype=torch.float),
                         actor.a_min, actor.a_max)
        a = at.numpy().astype(np.float64)
        lp = torch.distributions.Normal(mean, actor.std).log_prob(at).numpy().astype(np.float64)
    lp = lp + 0.3 * g.normal(size=lp.shape)
    for i in range(B):
        agent.buffer.append(s=s[i], a=a[i], log_prob=lp[i], r=r[i], s_=s2[i], done=done[i],
                            success=success[i], index=i)
    before_a, before_c = _flat(actor), _flat(critic)
    with torch.no_grad():
        vs = critic(torch.tensor(s, dtype=torch.float))
    rec, grads = {}, {}
    _grad_tap(grads, "actor", agent.optimizer_actor, list(actor.parameters()))
    _grad_tap(grads, "critic", agent.optimizer_critic, list(critic.parameters()))
    real = ppo2_mod.torch
    ppo2_mod.torch = _TorchProbe(rec)
    try:
        agent.learn(0, buf_num=1)
    finally:
        ppo2_mod.torch = real
    adv = torch.tensor(rec["gae_list"]).view(-1, 1)
    v_target = adv + vs
    adv_n = (adv - adv.mean()) / (adv.std() + 1e-5)
    np.savez_compressed(os.path.join(OUT, "ppo2_ugvoa_learn.npz"), s=s, a=a, a_lp=lp, r=r, s_=s2,
                        done=done, success=success, before_actor=before_a, before_critic=before_c,
                        after_actor=_flat(actor), after_critic=_flat(critic),
                        adv_norm=adv_n.numpy()[:, 0], v_target=v_target.numpy()[:, 0],
                        grad_actor=grads["actor"], grad_critic=grads["critic"],
                        std=std0.astype(np.float32), a_min=lo, a_max=hi, K=np.int32(K))
    print("ppo2_ugvoa_learn", {k: float(np.abs(v).max()) for k, v in grads.items()})


def gen_dppo2_learn():
    """Two consecutive Worker.learn() iterations of the DPPO2-CartPole copy (SharedAdam with the
    driver's lr / eps, k_epo = 6, use_grad_clip=True, clip 0.2), the local nets reloaded from the
    global ones before each, as Worker.run() does (:124-125). Captures the global nets after each
    learn() — they carry the never-zeroed local gradient buffers' accumulation."""
    with quiet():
        dmod = load("demonstration/DPPO2/DPPO2-4-CartPole/Distributed_PPO2.py", "ref_dppo2_cp")
        ddrv = load("demonstration/DPPO2/DPPO2-4-CartPole/train.py", "ref_dppo2_cp_train")
    g = np.random.default_rng(20262)
    torch.manual_seed(23)
    mk_a = lambda: ddrv.PPOActor_Gaussian(state_dim=4, action_dim=1, a_min=np.array([-8.]),
                                          a_max=np.array([8.]), init_std=1.2,
                                          use_orthogonal_init=True)
    g_actor, l_actor = mk_a(), mk_a()
    g_critic = ddrv.PPOCritic(state_dim=4, use_orthogonal_init=True)
    l_critic = ddrv.PPOCritic(state_dim=4, use_orthogonal_init=True)
    with torch.no_grad():
        torch.nn.init.orthogonal_(g_actor.fc3.weight, gain=1.0)
    P = 20
    a_lr, c_lr, k_epo = 1e-4 / min(P, 5), 1e-3 / min(P, 5), int(30 / min(P, 5))
    opt_a = cls_mod.SharedAdam([{'params': g_actor.parameters(), 'lr': a_lr}], eps=1e-5)
    opt_c = cls_mod.SharedAdam([{'params': g_critic.parameters(), 'lr': c_lr}], eps=1e-5)
    B = 1000
    ppo_msg = {'gamma': 0.99, 'k_epo': k_epo, 'eps_clip': 0.2, 'buffer_size': B, 'state_dim': 4,
               'action_dim': 1, 'device': 'cpu', 'set_adam_eps': True, 'lmd': 0.95,
               'use_adv_norm': True, 'mini_batch_size': 64, 'entropy_coef': 0.01,
               'use_grad_clip': True, 'use_lr_decay': True, 'max_train_steps': int(5e6),
               'using_mini_batch': False, 'action_range': [[-8., 8.]]}

    class _Env:
        state_dim, action_dim = 4, 1
    w = dmod.Worker(g_actor, l_actor, g_critic, l_critic, opt_c, opt_a, None, 0, "w0", _Env(),
                    None, None, ppo_msg)
    out = {"before_actor": _flat(g_actor), "before_critic": _flat(g_critic), "a_lr": a_lr,
           "c_lr": c_lr, "k_epo": k_epo, "gamma": 0.99, "std": np.float32(1.2)}
    for it in range(2):
        l_actor.load_state_dict(g_actor.state_dict())
        l_critic.load_state_dict(g_critic.state_dict())
        s, a, lp, r, s2, done, _ = _learn_buffer(g, B, 4, l_actor, 0.3)
        success = (g.uniform(size=B) < 0.9).astype(np.float64)     # `0 if flag == 1 else 1` (:138)
        for i in range(B):
            w.buffer.append(s=s[i], a=a[i], log_prob=lp[i], r=r[i], s_=s2[i], done=done[i],
                            success=success[i], index=i)
        w.learn()
        out.update({f"it{it}_s": s, f"it{it}_a": a, f"it{it}_a_lp": lp, f"it{it}_r": r,
                    f"it{it}_s_": s2, f"it{it}_done": done, f"it{it}_success": success,
                    f"it{it}_after_actor": _flat(g_actor), f"it{it}_after_critic": _flat(g_critic)})
    print("dppo2_learn", {k: float(np.abs(out[f"it1_after_{k}"] - out[f"before_{k}"]).max())
                          for k in ("actor", "critic")})
    np.savez_compressed(os.path.join(OUT, "dppo2_learn.npz"), **out)


class _NoiseTape:
    """Normal.sample() as loc + eps * scale with eps ~ N(0,1) drawn here and recorded: the
    driver's exploration noise becomes data a replay can inject."""

    def __init__(self):
        self.tape, self.orig = [], torch.distributions.Normal.sample

    def __enter__(self):
        tape = self

        def sample(dist, sample_shape=torch.Size()):
            shape = dist._extended_shape(sample_shape)
            eps = torch.randn(shape)
            tape.tape.append(eps.clone())
            return dist.loc + eps * dist.scale
        torch.distributions.Normal.sample = sample
        return self

    def __exit__(self, *a):
        torch.distributions.Normal.sample = self.orig


def gen_ppo2_transcript(key):
    """The N=1 PPO2 driver loop (train.py:184-224) for one buffer (1000 steps, int(timeMax/dt)*4)
    then learn() with the demo's ppo_msg (K_epochs 30, full batch; AngleOnly: grad clip + lr
    decay). Episode starts come from the env's own reset law (numpy seeded here) and are recorded,
    the exploration noise is recorded (_NoiseTape): a replay injects both."""
    if key == "cartpole":
        with quiet():
            tdrv = drv
        env = mods["cp_ppo2"].CartPole(0., 0.)
        over = {}
    else:
        with quiet():
            tdrv = load("demonstration/PPO2/PPO2-4-CartPoleAngleOnly/train.py", "ref_ppo2_ao_train")
        env = mods["ao_ppo2"].CartPoleAngleOnly(0.)
        over = {'use_grad_clip': True, 'use_lr_decay': True}
    np.random.seed(31 if key == "cartpole" else 32)
    torch.manual_seed(41 if key == "cartpole" else 42)
    ar = np.array(env.action_range)
    actor = tdrv.PPOActor_Gaussian(state_dim=env.state_dim, action_dim=env.action_dim,
                                   a_min=ar[:, 0], a_max=ar[:, 1], init_std=env.fm / 3,
                                   use_orthogonal_init=True)
    critic = tdrv.PPOCritic(state_dim=env.state_dim, use_orthogonal_init=True)
    B = int(env.timeMax / env.dt) * 4
    ppo_msg = {'gamma': 0.999, 'K_epochs': 30, 'eps_clip': 0.2, 'buffer_size': B,
               'state_dim': env.state_dim, 'action_dim': env.action_dim, 'a_lr': 3e-4, 'c_lr': 1e-3,
               'set_adam_eps': True, 'lmd': 0.95, 'use_adv_norm': True, 'mini_batch_size': 64,
               'entropy_coef': 0.01, 'use_grad_clip': False, 'use_lr_decay': False,
               'max_train_steps': int(5e6), 'using_mini_batch': False}
    ppo_msg.update(over)
    env_msg = {'state_dim': env.state_dim, 'action_dim': env.action_dim, 'name': env.name,
               'action_range': env.action_range}
    agent = ppo2_mod.Proximal_Policy_Optimization2(env_msg, ppo_msg, actor=actor, critic=critic)
    reward_norm = cls_mod.Normalization(shape=1)
    before_a, before_c = _flat(actor), _flat(critic)
    resets, raw_r, flags = [], [], []
    env.is_terminal = True
    idx = 0
    with _NoiseTape() as tape, quiet():
        while idx < B:
            if env.is_terminal:
                env.reset(True)
                resets.append([env.initTheta, getattr(env, "initX", 0.)])
            else:
                env.current_state = env.next_state.copy()
                a, a_lp = agent.choose_action(env.current_state)
                env.step_update(a)
                success = 0 if (env.is_terminal and env.terminal_flag == 3) else \
                    (1 if env.is_terminal else 0)
                raw_r.append(env.reward)
                flags.append(env.terminal_flag)
                agent.buffer.append(s=env.current_state, a=a, log_prob=a_lp,
                                    r=reward_norm(env.reward), s_=env.next_state,
                                    done=1.0 if env.is_terminal else 0.0, success=success,
                                    index=idx)
                idx += 1
        timestep = B
        agent.learn(timestep, buf_num=1)
    b = agent.buffer
    np.savez_compressed(
        os.path.join(OUT, f"ppo2_transcript_{key}.npz"), resets=np.array(resets),
        noise=np.concatenate([e.numpy().reshape(-1) for e in tape.tape]).astype(np.float32),
        s=b.s, a=b.a, a_lp=b.a_lp, r=b.r[:, 0], s_=b.s_, done=b.done[:, 0],
        success=b.success[:, 0], raw_reward=np.array(raw_r), flag=np.array(flags),
        before_actor=before_a, before_critic=before_c, after_actor=_flat(actor),
        after_critic=_flat(critic), std=np.float32(env.fm / 3), B=B)
    print("ppo2_transcript", key, len(resets), "episodes", "max |dW| actor %.3e critic %.3e" % (
        np.abs(_flat(actor) - before_a).max(), np.abs(_flat(critic) - before_c).max()))


if __name__ == "__main__" and len(sys.argv) > 2:   # selected generators only
    for name in sys.argv[2:]:
        if name.startswith("ugvoa_"):
            gen_ugvoa(name, n=400 if name == "ugvoa_env" else 300)
        elif name.startswith("ppo2_transcript_"):
            gen_ppo2_transcript(name[len("ppo2_transcript_"):])
        else:
            globals()["gen_" + name]()
    sys.exit(0)

if __name__ == "__main__":
    gen_cartpole("cartpole_ppo2", mods["cp_ppo2"])
    gen_cartpole("cartpole_dppo2", mods["cp_dppo2"], n=100)
    gen_angleonly("angleonly_ppo2", mods["ao_ppo2"])
    gen_angleonly_env()
    gen_soi("soi_env", mods["soi_env"])
    gen_soi("soi_dppo2", mods["soi_dppo2"], n=200)
    gen_ugv("ugvf_env", mods["ugvf_env"].UGVForward)
    gen_ugv("ugvf_ppo2", mods["ugvf_ppo2"].UGVForward, n=200)
    gen_ugv("ugvf_dppo2", mods["ugvf_dppo2"].UGVForward, n=200)
    gen_ugv("ugvb_env", mods["ugvb_env"].UGVBidirectional)
    gen_ugv("ugvb_ppo2", mods["ugvb_ppo2"].UGVBidirectional, n=200)
    gen_uav("uav_hover")
    gen_ugvoa("ugvoa_env")
    gen_ugvoa("ugvoa_ppo2", n=300)
    gen_ugvoa("ugvoa_dppo2", n=300)
    gen_nets()
    gen_gae()
    gen_reward_norm()
    gen_replay()
    gen_ddpg()
    gen_sac()
    gen_ddpg_grad()
    gen_sac_grad()
    gen_ppo2_learn()
    gen_ppo2_soi_learn()
    gen_ppo2_ugvoa_learn()
    gen_dppo2_learn()
    gen_ppo2_transcript("cartpole")
    gen_ppo2_transcript("angleonly")
    with open(os.path.join(OUT, "VERSIONS.txt"), "w") as f:
        f.write(f"numpy {np.__version__}\ntorch {torch.__version__}\npython {sys.version.split()[0]}\n"
                f"reference {REF} (HKPolyU-UAV/ReinforcementLearningPlatform @ 2025-02-28)\n")
