"""Host time against GPU time of one rank's GCN epoch at 8-rank size:
the products graph at scale 1/8 (one rank's share of the rows), reordered as bench.py
does, ``GCNTrainer`` with ``collectives=True`` on a 1-rank ``nccl`` group, so every exchange branch of the
multi-rank epoch runs (async all-gather / all-to-all on RCCL's stream, split
aggregation, backward all-gather overlap, gradient all-reduce), each the identity.

Per epoch: the host time of ``train_step`` (Python enqueue, no synchronisation) and the
GPU time between two events around it; plus the one-GPU path (no collectives, hipGraph
replay) on the same graph for comparison.  One JSON line per form.

    python tools/multirank_host.py [--scale 0.125] [--epochs 20]
"""
import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def measure(tr, epochs, warmup):
    for _ in range(warmup):
        tr.train_step()
    torch.cuda.synchronize()
    host, ev = [], []
    t_all = time.perf_counter()
    for _ in range(epochs):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t = time.perf_counter()
        tr.train_step()
        host.append((time.perf_counter() - t) * 1e3)
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_all) * 1e3 / epochs
    gpu = [a.elapsed_time(b) for a, b in ev]
    return {"host_ms": round(float(np.median(host)), 3), "gpu_ms": round(float(np.median(gpu)), 3),
            "wall_ms_per_epoch": round(wall, 3),
            "host_over_gpu": round(float(np.median(host)) / max(float(np.median(gpu)), 1e-9), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.125)
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--forms", default="one_gpu_captured,collectives,collectives_halo",
                    help="comma-separated subset of the forms to run")
    a = ap.parse_args()
    import torch.distributed as dist
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    g = synthetic("ogbn-products", seed=0, device=dev, scale=a.scale)
    forms = (("one_gpu_captured", {}), ("collectives", dict(collectives=True)),
             ("collectives_halo", dict(collectives=True, halo=True)))
    for name, kw in forms:
        if name not in a.forms.split(","):
            continue
        tr = GCNTrainer(g, hidden=256, rank=0, world=1, reorder=True, **kw)     # as bench.py
        res = {"form": name, "scale": a.scale, "rows": g.n, "nnz": g.nnz, "multi": bool(tr.multi),
               "captured": bool(getattr(tr, "_graph", None) is not None and
                                getattr(getattr(tr, "_graph", None), "graph", None) is not None)}
        res.update(measure(tr, a.epochs, a.warmup))
        res["captured"] = bool(getattr(getattr(tr, "_graph", None), "graph", None) is not None)
        print(json.dumps(res), flush=True)
        del tr
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
