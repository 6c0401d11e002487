"""bench.py's distributed logic end to end on CPU: gloo ranks launched by
torch.distributed.run or by bench.py itself (``--gpus N`` with no launcher
around it), a tiny graph on the PyTorch path; rank 0 prints the one JSON line
of the driver contract (the GPU run differs only in device/backend)."""
import json
import os

import pytest
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# 4: halo path; 8: the driver's node size (halo plans, train-column slots and row blocks
# at the shapes of the 8-GPU scaling run)
@pytest.mark.parametrize("nproc,launcher", [(2, "torchrun"), (2, "self"), (4, "self"), (8, "torchrun")])
def test_bench_gloo_ranks_print_one_json_line(nproc, launcher):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1" if nproc > 4 else "2"
    args = ["bench.py", "--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--device", "cpu",
            "--scale", "0.002", "--hidden", "64"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    res = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout
    out = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "val_acc"):
        assert key in out, key
    assert out["n_gpus"] == nproc and out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and abs(out["value"] * out["ms_per_step"] / 1000.0 - 1.0) < 1e-3
    assert out["config"]["parallelism"] == "graph-rowpart%d" % nproc
    # the process group that ran it (checked by the pre-timing collective self-test)
    assert out["backend"] == "gloo" and out["world_size"] == nproc


def test_bench_rejects_rank_count_mismatch():
    """--gpus must equal the launcher's world size (a silent 1-rank run is an error)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", OMP_NUM_THREADS="2")
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--scale", "0.002"],
                         cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         timeout=300)
    assert res.returncode != 0 and "launcher started 1 ranks" in res.stderr
