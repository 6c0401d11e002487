"""Headline benchmark (BASELINE.json): epochs/sec + val-acc of a 2-layer GCN on
an ogbn-products-shaped graph, 1/2/4/8 MI355X.

    python bench.py --gpus N --steps K --warmup W          (starts N ranks itself)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full-graph training epoch (forward + backward + Adam) over all
2,449,029 nodes (both dense layers at every row; the layer-2 aggregation at the
train rows, the only rows whose logits reach the loss, and the layer-1
aggregation at the rows with a train neighbour, the only ones those read --
exact, see gnn/gcn.py; GCNTrainer(train_rows_only=False) aggregates every row).  Data: synthetic graph of the ogbn-products shape (no network
for the real dataset), random-init weights.  Multi-GPU: 1-D row partition of
the graph over ranks (strong scaling: the whole job trains the same graph),
an RCCL all-to-all of the layer-2 rows the rank's train rows read (a training
halo, negotiated once), an all-gather of the compact train-row gradient and an
all-reduce of the weight gradients.  W untimed warm-up epochs, then exactly K timed epochs
bracketed by barrier + device synchronize; the MAX time over ranks is reported.
"""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _launcher():
    """cgnn_amd/parallel/launch.py loaded standalone: the launching parent imports
    neither torch nor the package, so it cannot initialise a device."""
    spec = importlib.util.spec_from_file_location(
        "_cgnn_launch", os.path.join(ROOT, "cgnn_amd", "parallel", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod

METRIC = "epochs/sec + val-acc, 2-layer GCN ogbn-products, 1/2/4/8 MI355X"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dataset", default="ogbn-products")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the graph (debug only)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--feat-noise", type=float, default=4.0)
    ap.add_argument("--label-noise", type=float, default=0.25)
    ap.add_argument("--rows", choices=["auto", "aligned", "packed", "mixed"], default="auto",
                    help="row pitch of gathered matrices: whole 128-B lines, packed to 8 elements, "
                         "mixed (features aligned, layer-2 rows packed), "
                         "or auto (features aligned, layer-2 rows packed: the same as mixed)")
    ap.add_argument("--no-fused", action="store_true", help="hipBLASLt GEMMs + separate epilogues")
    ap.add_argument("--capture", action="store_true", help="replay the epoch from a hipGraph (one GPU)")
    ap.add_argument("--id-order", choices=["shuffled", "banded"], default="shuffled",
                    help="synthetic node ids: shuffled (no locality in the ids, like a real dataset) or "
                         "the generator's banded ids (locality for free; A/B only)")
    ap.add_argument("--reorder", choices=["lp-cm", "none"], default="lp-cm",
                    help="framework locality pass at setup (label-propagation clusters + Cuthill-McKee)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: gloo ranks on the PyTorch path (tests the script's distributed logic only)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal: every rank on cuda:0 with gloo collectives (exercises the multi-rank "
                         "HIP path on a one-GPU box; timings are not a scaling measurement)")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start the N ranks here (children re-run this script)
        sys.exit(_launcher().spawn_ranks(a.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))

    if os.environ.get("CGNN_TRACEBACK_AFTER"):
        # diagnostics: dump every thread's Python stack to stderr periodically (a hung rank
        # shows where it waits)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["CGNN_TRACEBACK_AFTER"]), repeat=True)
    import torch
    import torch.distributed as dist
    from cgnn_amd.parallel import dist as pdist
    from cgnn_amd.gnn.data import SHAPES, synthetic
    from cgnn_amd.gnn.gcn import GCNTrainer

    cuda = a.device == "cuda"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started %d ranks" % (a.gpus, world))
    shared = cuda and a.shared_gpu
    if cuda and not shared and torch.cuda.device_count() < world:
        sys.exit("bench.py: --gpus %d but only %d GPUs are visible" % (world, torch.cuda.device_count()))
    if world > 1:
        pdist.init_process_group("nccl" if (cuda and not shared) else "gloo")
        if pdist.world_size() != world:
            sys.exit("bench.py: process group has %d ranks, expected %d" % (pdist.world_size(), world))
    rank = pdist.rank()
    local = pdist.local_rank()
    if world > 1 and os.environ.get("OMP_NUM_THREADS") == "1":
        # torch.distributed.run pins OMP_NUM_THREADS=1: give the host C++ setup (graph
        # generation, locality reorder) this rank's share of the node's cores instead
        pdist.set_host_threads()
    if cuda:
        torch.cuda.set_device(0 if shared else local)
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    backend = {"backend": "none (one process)", "world_size": 1}
    if world > 1:
        # content-checked collectives before anything is timed: a mis-launched job (wrong
        # world size, transport that drops or reorders) exits non-zero instead of timing
        from cgnn_amd.parallel.collectives import selftest
        try:
            backend = selftest(dev)
        except RuntimeError as exc:
            sys.stderr.write("bench.py: %s\n" % exc)
            sys.exit(3)
        if backend["world_size"] != world:
            sys.exit("bench.py: process group has %d ranks, expected %d" % (backend["world_size"], world))

    def sync():
        if cuda:
            torch.cuda.synchronize()

    t_setup = time.perf_counter()
    # a rehearsal's ranks share one device: build the CSR with the host C++ path there
    # (N concurrent device radix sorts of the edge keys stalled the setup)
    g = synthetic(a.dataset, seed=a.seed, device="cpu" if shared else dev, scale=a.scale,
                  feat_noise=a.feat_noise, label_noise=a.label_noise, id_order=a.id_order)
    if shared:
        g = g.to(dev)
    sync()
    gen_s = time.perf_counter() - t_setup
    tr = GCNTrainer(g, hidden=a.hidden, dropout=a.dropout, lr=a.lr, seed=a.seed,
                    fused=not a.no_fused,
                    align_rows={'auto': None, 'aligned': True, 'packed': False, 'mixed': None}[a.rows],
                    align_c=False if a.rows == "mixed" else None,
                    capture=a.capture, reorder=a.reorder != "none")
    n_nodes, nnz = g.n, g.nnz
    del g
    sync()
    setup_s = time.perf_counter() - t_setup
    trainer_setup_s = setup_s - gen_s          # includes the reordering pass

    for _ in range(a.warmup):
        tr.train_step()
    pdist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_step()
    sync()
    pdist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    res = tr.evaluate()
    train_loss = tr.train_loss()

    n, m, F, C, _, _ = SHAPES[a.dataset]
    if rank == 0:
        eps = a.steps / dt
        out = {
            "metric": METRIC,
            "value": round(eps, 4),
            "unit": "epochs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16" if cuda else "fp32 (CPU reference path)",
            "data": "synthetic graph of the %s shape (%d nodes, %d undirected edges, %d features, "
                    "%d classes; planted communities; %s node ids), random-init weights"
                    % (a.dataset, n, m, F, C, a.id_order),
            "shared_gpu_rehearsal": bool(shared),
            "backend": backend["backend"],
            "world_size": backend["world_size"],
            "collective_selftest_ms": backend.get("ms"),
            "config": {"model": "GCN-2layer-hidden%d" % a.hidden, "global_batch": n_nodes,
                       "seq_len": None, "parallelism": "graph-rowpart%d" % world,
                       "dataset": a.dataset, "nnz_with_self_loops": nnz, "dropout": a.dropout,
                       "optimizer": "adam", "lr": a.lr, "id_order": a.id_order,
                       "reordered": a.reorder != "none",
                       # training epochs aggregate layer 2 at the rows the loss reads
                       "train_layer2_rows": "all" if tr._l2 is None else "train",
                       "train_layer1_rows": "all" if tr._l1 is None else "train-neighbours"},
            "val_acc": round(res["val_acc"], 4),
            "test_acc": round(res["test_acc"], 4),
            "train_loss": round(train_loss, 5),
            "epochs_trained": a.warmup + a.steps,
            "setup_s": round(setup_s, 2),
            "trainer_setup_s": round(trainer_setup_s, 2),
            "acc_note": "synthetic-task accuracy (label/feature noise set its ceiling); not comparable "
                        "with real ogbn-products accuracy",
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
