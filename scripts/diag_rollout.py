"""Diagnostic build of the shared-physics rollout kernel with per-phase s_memtime stamps.

Not product code: copies the csrc tree into csrc/build/diag/, inserts stamps into
rollout_sp_kernel (MLP pass / barrier after it / physics / barrier after it), builds
librlp_diag.so, and (with --run, on the GPU box) runs the bench workload through it and prints
per-wave-step cycle averages. Build here:  python scripts/diag_rollout.py --build
Run on the box:                           python scripts/diag_rollout.py --run [--n 65536 --T 128]
"""
import argparse
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "reinforcementlearningplatform_amd", "csrc")
DIAG = os.path.join(CSRC, "build", "diag")

STAMP = "__builtin_amdgcn_s_memtime()"


def patch(src):
    s = src
    s = s.replace("namespace rlp {\n", "namespace rlp {\n__device__ unsigned long long rlp_diag_acc[65536][9];\n", 1)
    old = """    for (int t = 0; t < ra.T; ++t) {
        const uint64_t gstep = ra.step0 + (uint64_t)t;
        mlp_pass(true);
        asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");  // (mean, V) of every env
        if (wave / PW == t % ROT && lane < PHL) {  // this step's physics waves"""
    new = """    unsigned long long dg[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    dg[6] = __builtin_amdgcn_s_memrealtime();
    dg[8] = __smid();
    for (int t = 0; t < ra.T; ++t) {
        const uint64_t gstep = ra.step0 + (uint64_t)t;
        const unsigned long long t0 = %s;
        mlp_pass(true);
        const unsigned long long t1 = %s;
        asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");  // (mean, V) of every env
        const unsigned long long t2 = %s;
        dg[0] += t1 - t0; dg[1] += t2 - t1;
        const bool physw = wave / PW == t %% ROT;
        if (wave / PW == t %% ROT && lane < PHL) {  // this step's physics waves""" % (STAMP, STAMP, STAMP)
    assert old in s, "stamp site 1"
    s = s.replace(old, new)
    old = """                for (int j = 0; j < S; ++j) sob[le][j] = on[j];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");  // next observations
    }"""
    new = """                for (int j = 0; j < S; ++j) sob[le][j] = on[j];
            }
        }
        const unsigned long long t3 = %s;
        asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");  // next observations
        const unsigned long long t4 = %s;
        if (physw) { dg[2] += t3 - t2; dg[4] += 1; }
        dg[3] += t4 - t3;
    }
    dg[5] = ra.T;
    dg[7] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0)
        for (int q = 0; q < 9; ++q) rlp_diag_acc[blockIdx.x * W + wave][q] = dg[q];""" % (STAMP, STAMP)
    assert old in s, "stamp site 2"
    s = s.replace(old, new)
    s += """
extern "C" int rlp_diag_read(void *host, long long bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(rlp::rlp_diag_acc), (size_t)bytes, 0,
                                    hipMemcpyDeviceToHost);
}
"""
    return s


VARIANTS = {
    "base": [],
    # timing experiments (results invalid by design): the hidden-layer tanh without its exp/rcp
    "cheap_hidden": [("rlp_mfma_x3.hpp",
                      "const float2v x = tanh2_scaled(pre, 2.8853900817779268f, kX3HScale);",
                      "const float2v x = pre * kX3HScale;")],
    # the output-layer tanh without its exp/rcp
    "cheap_out": [("rlp_mfma_x3.hpp",
                   "const float2v h = tanh2_scaled((float2v){acc[sb][j][r], acc[sb][j][r + 1]}, k_out, 1.0f);",
                   "const float2v h = (float2v){acc[sb][j][r], acc[sb][j][r + 1]} * k_out;")],
    # CartPole physics: no RK4 (one Euler-like update)
    "nophys": [("rlp_envs.hpp", "        while (time < tt) {  // fp64 time accumulation",
                "        if (false) {  // diag: no RK4")],
}


def lib_path(variant, rev=None):
    return os.path.join(DIAG, f"librlp_diag_{variant}{'_' + rev if rev else ''}.so")


def build(variant="base", rev=None, target="rlp_rollout.hip", patcher=None):
    src_root = os.path.join(DIAG, "a", "b", "csrc")
    if os.path.exists(os.path.join(DIAG, "a")):
        shutil.rmtree(os.path.join(DIAG, "a"))
    shutil.copytree(CSRC, src_root, ignore=shutil.ignore_patterns("build"))
    os.makedirs(os.path.join(DIAG, "a", "include"), exist_ok=True)
    shutil.copy(os.path.join(ROOT, "include", "rlp.h"), os.path.join(DIAG, "a", "include", "rlp.h"))
    if rev:   # A/B against a committed revision of the whole native tree
        shutil.rmtree(src_root)
        tmp = os.path.join(DIAG, "rev")
        if os.path.exists(tmp):
            shutil.rmtree(tmp)
        os.makedirs(tmp)
        arc = subprocess.run(["git", "-C", ROOT, "archive", rev, "reinforcementlearningplatform_amd/csrc",
                              "include"], check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", tmp], input=arc, check=True)
        shutil.copytree(os.path.join(tmp, "reinforcementlearningplatform_amd", "csrc"), src_root)
        shutil.copy(os.path.join(tmp, "include", "rlp.h"), os.path.join(DIAG, "a", "include", "rlp.h"))
        shutil.rmtree(tmp)
    p = os.path.join(src_root, target)
    with open(p) as f:
        s = f.read()
    with open(p, "w") as f:
        f.write((patcher or patch)(s))
    for fname, a, b in VARIANTS.get(variant, []):
        q = os.path.join(src_root, fname)
        with open(q) as f:
            t = f.read()
        assert a in t, (variant, a)
        with open(q, "w") as f:
            f.write(t.replace(a, b))
    subprocess.run(["make", "-s", "-j8", "-C", src_root, f"OUT={lib_path(variant, rev)}"], check=True)
    print("built", lib_path(variant, rev))


def run(n, T, iters, variant="base", sub=0, physics=1, rev=None, env="cartpole"):
    LIB = lib_path(variant, rev)
    os.environ["RLP_LIBRARY"] = LIB
    sys.path.insert(0, ROOT)
    import ctypes
    import numpy as np
    import torch
    import bench
    from reinforcementlearningplatform_amd import _native
    if sub:
        _native.set_rollout_sub(sub)
    _native.set_rollout_physics(physics)
    seg = bench.Segment(env, n, T, 3407, 0)
    for _ in range(2):
        seg.rollout()
    torch.cuda.synchronize()
    res = []
    for _ in range(iters):
        seg.rollout()
        torch.cuda.synchronize()
        buf = np.zeros((65536, 9), np.uint64)
        lib = ctypes.CDLL(LIB)
        assert lib.rlp_diag_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(buf.nbytes)) == 0
        es = sub or (2 if (n + 127) // 128 >= 512 else 1)     # rlp_rollout's auto choice
        nw = (n + 64 * es - 1) // (64 * es) * 4
        res.append(buf[:nw].astype(np.float64))
    d = np.mean(res, axis=0)
    steps = d[:, 5]
    mlp, bar1, phys, bar2, nphys = (d[:, i] / steps for i in range(5))
    phys_per = d[:, 2] / np.maximum(d[:, 4], 1)
    print(f"[{variant}{' @' + rev if rev else ''}] n={n} T={T} sub={sub or 'auto'} physics={physics}: cycles per step per wave (mean over {nw} waves):")
    print(f"  MLP pass (actor+critic) {mlp.mean():9.0f}  (min {mlp.min():.0f} max {mlp.max():.0f})")
    print(f"  barrier after MLP       {bar1.mean():9.0f}")
    print(f"  physics (its waves)     {phys_per.mean():9.0f}  per physics turn; share {nphys.mean():.2f}")
    print(f"  barrier after physics   {bar2.mean():9.0f}")
    print(f"  step total              {(mlp + bar1 + phys + bar2).mean():9.0f}")
    # block start / end on the 100 MHz real-time clock (last iteration), per wave 0 of each block
    b = res[-1][:nw].astype(np.float64)
    w0 = b[::4] if nw % 4 == 0 else b
    st, en = (w0[:, 6] - w0[:, 6].min()) / 100.0, (w0[:, 7] - w0[:, 6].min()) / 100.0   # us
    dur = en - st
    print(f"  blocks: start spread {st.max():.1f} us (p50 {np.median(st):.1f}), end min {en.min():.1f} "
          f"p50 {np.median(en):.1f} max {en.max():.1f} us; duration min {dur.min():.1f} p50 "
          f"{np.median(dur):.1f} max {dur.max():.1f} us")
    tot = (b[:, 0] + b[:, 1] + b[:, 2] + b[:, 3])
    hw = b[:, 8].astype(np.int64)
    print(f"  per-wave loop cycles: min {tot.min():.0f} p10 {np.percentile(tot, 10):.0f} p50 {np.median(tot):.0f} "
          f"p90 {np.percentile(tot, 90):.0f} max {tot.max():.0f}")
    np.save(os.path.join(ROOT, "gpurun_out", f"diag_waves_{variant}.npy"), b)
    try:   # by XCD (HW_ID's SE bits vary by ISA; report the raw low bits' grouping as a hint)
        import collections
        grp = collections.defaultdict(list)
        for h, t in zip(hw, tot):
            grp[int(h) % 8].append(t)
        print("  loop cycles by __smid() % 8:", {k: round(float(np.mean(v))) for k, v in sorted(grp.items())})
    except Exception as ex:
        print("  smid grouping failed:", ex)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--variant", default="base", choices=sorted(VARIANTS) + ["all"])
    ap.add_argument("--sub", type=int, default=0)
    ap.add_argument("--rev", default=None, help="build / run the native tree of this git revision")
    ap.add_argument("--env", default="cartpole")
    ap.add_argument("--physics", type=int, default=1, help="rlp_set_rollout_physics (3: 32x32x16 MLP)")
    a = ap.parse_args()
    if a.build:
        for v in (VARIANTS if a.variant == "all" else [a.variant]):
            build(v, a.rev)
    if a.run:
        run(a.n, a.T, a.iters, a.variant, a.sub, a.physics, a.rev, a.env)
