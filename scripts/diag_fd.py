"""Diagnostic build of the PPO2 update's ppo2_fd_kernel with per-phase s_memtime stamps.

Not product code: copies the native tree (or a git revision's, --rev) into csrc/build/diag/,
inserts stamps between the per-tile phases of ppo2_fd_kernel (forward GEMM, h2/z3, loss head,
dW3 transpose, g2 + store, backward GEMM, g1, dW1 transpose), builds librlp_diag_fd*.so and,
with --run on the GPU box, runs bench-size native updates through it and prints cycles per
16-row wave tile. Build here:  python scripts/diag_fd.py --build [--rev REV]
Run on the box:                python scripts/diag_fd.py --run [--rev REV]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import diag_rollout as dr  # noqa: E402  (shared tree-copy / build helpers)

ST = "__builtin_amdgcn_s_memtime()"
MARKS = [  # (anchor text in the tile loop, phase index the time since the previous mark goes to)
    ("        // ---- h2 = tanh(z2), z3 = W3 h2 + b3", 0),
    ("        // ---- head gradient g3 = dL/dz3", 1),
    ("        // ---- dW3 = sum_rows g3 h2^T", 2),
    ("        // ---- g2 = (W3^T g3) * (1 - h2^2) in place", 3),
    ("        // ---- backward: dh1 = W2^T g2", 4),
    ("        // ---- g1 = dh1 * (1 - h1^2)", 5),
    ("        // ---- dW1 | db1 = sum_rows g1", 6),
]
NAMES = ["fwd GEMM (+layer1/tanh/split)", "h2 tanh + z3", "loss head g3", "dW3 (row butterfly)",
         "g2 + G2 store + max", "bwd GEMM", "g1 (h1 recompute)", "dW1 (lane-group butterfly)"]


def patch(s):
    s = s.replace("namespace rlp {\n", "namespace rlp {\n__device__ unsigned long long rlp_fd_acc[16384][10];\n", 1)
    old = "    for (int64_t bt = blockIdx.x; bt < nbt; bt += gridDim.x) {\n"
    assert old in s
    s = s.replace(old, "    unsigned long long dg[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};\n" + old +
                  f"        unsigned long long tp = {ST};\n        dg[9] += 1;\n", 1)
    for anchor, ph in MARKS:
        assert anchor in s, anchor
        s = s.replace(anchor, f"        {{ const unsigned long long tn = {ST}; dg[{ph}] += tn - tp; tp = tn; }}\n" +
                      anchor, 1)
    old = """                for (int i = 0; i < 2 * NC; ++i) dW1p[h][i] += pair_sum_x16(v[i], v[i + 2 * NC]);
            }
        }
    }

    // ---- per-wave partials"""
    assert old in s
    s = s.replace(old, f"""                for (int i = 0; i < 2 * NC; ++i) dW1p[h][i] += pair_sum_x16(v[i], v[i + 2 * NC]);
            }}
        }}
        {{ const unsigned long long tn = {ST}; dg[7] += tn - tp; tp = tn; }}
    }}
    if (lane == 0 && blockIdx.x * kFdWaves + wv < 16384)
        for (int q = 0; q < 10; ++q) atomicAdd(&rlp_fd_acc[blockIdx.x * kFdWaves + wv][q], dg[q]);

    // ---- per-wave partials""", 1)
    s += """
extern "C" int rlp_diag_fd_read(void *host, long long bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(rlp::rlp_fd_acc), (size_t)bytes, 0,
                                    hipMemcpyDeviceToHost);
}
"""
    return s


def build(rev=None, variant="fd", waves=None):
    pt = patch
    if waves:
        pt = lambda s: patch(s.replace("#define RLP_FD_WAVES 8", f"#define RLP_FD_WAVES {waves}"))
    dr.build(variant, rev, target="rlp_update.hip", patcher=pt)


def run(rev=None, n=65536, T=128, epochs=2, variant="fd"):
    LIB = dr.lib_path(variant, rev)
    os.environ["RLP_LIBRARY"] = LIB
    sys.path.insert(0, dr.ROOT)
    import ctypes
    import numpy as np
    import torch
    import bench
    seg = bench.Segment("cartpole", n, T, 3407, 0)
    bench.e2e_iterations(seg, 1, k_epochs=epochs)
    torch.cuda.synchronize()
    buf = np.zeros((16384, 10), np.uint64)
    lib = ctypes.CDLL(LIB)
    assert lib.rlp_diag_fd_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(buf.nbytes)) == 0
    d = buf.astype(np.float64)
    d = d[d[:, 9] > 0]
    tiles = d[:, 9]
    per = d[:, :8] / tiles[:, None]
    print(f"[{variant}{' @' + rev if rev else ''}] n={n} T={T}: cycles per 16-row wave tile (mean over "
          f"{d.shape[0]} waves, {tiles.mean():.0f} tiles each over all launches):")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:32s} {per[:, i].mean():9.0f}")
    print(f"  {'total':32s} {per.sum(1).mean():9.0f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--rev", default=None)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--waves", type=int, default=None, help="RLP_FD_WAVES of the build (4 | 8)")
    a = ap.parse_args()
    variant = "fd" if a.waves is None else f"fd_w{a.waves}"
    if a.build:
        build(a.rev, variant, a.waves)
    if a.run:
        run(a.rev, epochs=a.epochs, variant=variant)
