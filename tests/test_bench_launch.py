"""bench.py's own N-rank launch (no torchrun): `python bench.py --gpus 2` starts two rank
processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set; each checks WORLD_SIZE == --gpus and
that one GPU per rank is visible, so on a node with fewer GPUs it fails with a clear message rather
than printing an n_gpus: 1 line. Runs on the CPU (no GPU visible here)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {}, RLP_BENCH_BACKEND="nccl")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_gpus2_launches_two_ranks_and_refuses_missing_gpus():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("needs a node with fewer than 2 GPUs")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr, r.stderr[-2000:]
    assert r.stderr.count("needs 2 visible GPUs") == 2   # both ranks ran the check
    assert '"n_gpus"' not in r.stdout


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]
