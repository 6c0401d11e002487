"""bench.py's multi-rank HIP path on ONE GPU: ``--shared-gpu`` puts every rank on
cuda:0 with gloo collectives (RCCL refuses two ranks on one device), so the fused
kernels, the row partition, the layer-2 all-gather (2 ranks) and the halo exchange
(4 ranks) run exactly as on a multi-GPU node; the run must reproduce the one-rank
losses and accuracies (dropout is keyed by the global row, gradients are summed
over ranks).  The 8-GPU RCCL run itself is the driver's scaling benchmark."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _run(nproc):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "4"
    args = [sys.executable, "bench.py", "--gpus", str(nproc), "--steps", "4", "--warmup", "2",
            "--scale", "0.02"]
    if nproc > 1:
        args.append("--shared-gpu")
    res = subprocess.run(args, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout
    return json.loads(lines[0])


def test_multirank_hip_path_matches_one_rank():
    one = _run(1)
    for n in (2, 4):
        out = _run(n)
        assert out["n_gpus"] == n and out["shared_gpu_rehearsal"]
        assert abs(out["train_loss"] - one["train_loss"]) < 1e-4 * one["train_loss"], (n, out, one)
        assert abs(out["val_acc"] - one["val_acc"]) < 2e-3, (n, out, one)
