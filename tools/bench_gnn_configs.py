"""Benchmarks of the BASELINE.json GNN configs other than the headline one
(``bench.py``: 2-layer GCN on ogbn-products).  Synthetic graphs of the named
shapes (no network for the datasets), random-init weights; one JSON line per
run on rank 0.

    python tools/bench_gnn_configs.py --config cora-cpu
    python tools/bench_gnn_configs.py --config arxiv-gcn3
    python tools/bench_gnn_configs.py --config reddit-infer
    python tools/bench_gnn_configs.py --config products-sage3            # 1 GPU
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/bench_gnn_configs.py --config products-sage3                # DP over 8 GPUs
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/bench_gnn_configs.py --config papers-gat2                   # graph sharded over 8 GPUs

Timing: W untimed warm-up steps, then K steps bracketed by barrier + device
synchronize; the MAX over ranks is reported.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def _progress(msg):
    """A progress line on stderr (long setups: the GPU runner takes a silent job as hung)."""
    from cgnn_amd.parallel import dist as pdist
    sys.stderr.write("[bench_gnn_configs rank %d %.1fs] %s\n" % (pdist.rank(), time.perf_counter() - _T0, msg))
    sys.stderr.flush()


_T0 = time.perf_counter()


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _timed(fn, steps, warmup, dev):
    from cgnn_amd.parallel import dist as pdist
    for _ in range(warmup):
        fn()
    pdist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    _sync(dev)
    pdist.barrier()
    dt = time.perf_counter() - t0
    if pdist.world_size() > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True,
                    choices=["cora-cpu", "arxiv-gcn3", "reddit-infer", "products-sage3", "papers-gat2"])
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the graph (nodes and edges)")
    ap.add_argument("--hidden", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-capture", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--reorder", choices=["lp-cm", "none"], default="lp-cm",
                    help="framework locality pass on the (shuffled-id) synthetic graph, timed in setup")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="papers-gat2: one process plays rank --emulate-rank of this many ranks (its "
                         "rank-local shard, halo plan and buffers; received rows zero) -- memory / compute dry run")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--partition", choices=["locality", "none"], default="locality",
                    help="papers-gat2: locality partition of the sharded graph (data.partition_order, timed in setup)")
    ap.add_argument("--order-cache", default=None,
                    help="papers-gat2, one process: load the partition order from this .npy file, or compute and "
                         "save it there (A/B runs of one shape)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal: every rank on cuda:0 with gloo collectives (multi-rank path on one GPU)")
    ap.add_argument("--sampler", choices=["pipelined", "device", "host"], default=None,
                    help="products-sage3: neighbour sampler (default: pipelined on a GPU)")
    ap.add_argument("--halo-grad-bf16", action="store_true", help="papers-gat2: gradients on the halo wire in bf16")
    ap.add_argument("--unfused", action="store_true", help="arxiv-gcn3 / products-sage3 / papers-gat2: autograd + hipBLASLt path (A/B)")
    a = ap.parse_args()

    from cgnn_amd.gnn.data import SHAPES, reorder, synthetic
    from cgnn_amd.parallel import dist as pdist

    def _graph(name):
        g = synthetic(name, seed=a.seed, device=dev, scale=a.scale)
        if a.reorder != "none":
            g, _ = reorder(g, seed=a.seed)
        return g

    world = int(os.environ.get("WORLD_SIZE", "1"))
    cpu = a.config == "cora-cpu" or not torch.cuda.is_available()
    if world > 1:
        pdist.init_process_group("gloo" if (cpu or a.shared_gpu) else "nccl")
    rank = pdist.rank()
    if world > 1 and os.environ.get("OMP_NUM_THREADS") == "1":
        pdist.set_host_threads()          # this rank's share of the cores (torchrun pins 1)
    if cpu:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(0 if a.shared_gpu else pdist.local_rank() % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
    capture = None if not a.no_capture else False
    res = {"n_gpus": 0 if cpu else world, "scale": a.scale}
    t_setup = time.perf_counter()

    if a.config in ("cora-cpu", "arxiv-gcn3"):
        from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer
        name, layers = ("cora", 2) if a.config == "cora-cpu" else ("ogbn-arxiv", 3)
        hidden = a.hidden or (16 if name == "cora" else 256)
        steps, warmup = a.steps or (100 if cpu else 200), a.warmup or 10
        g = _graph(name)
        dtype = torch.float32 if cpu else torch.bfloat16
        tr = DeepGCNTrainer(g, hidden=hidden, layers=layers, dropout=0.5, lr=0.01, dtype=dtype, seed=a.seed,
                            capture=capture, fused=False if a.unfused else None)
        setup = time.perf_counter() - t_setup
        dt = _timed(tr.train_step, steps, warmup, dev)
        ev = tr.evaluate()
        res.update(metric="epochs/sec + val-acc, %d-layer GCN %s full-graph" % (layers, name),
                   value=round(steps / dt, 3), unit="epochs/s", ms_per_step=round(1e3 * dt / steps, 4),
                   val_acc=round(ev["val_acc"], 4), test_acc=round(ev["test_acc"], 4),
                   dtype=str(dtype).replace("torch.", ""), hipgraph=bool(tr._step_graph.graph is not None),
                   fused=bool(tr.fused),
                   config={"model": "GCN-%dlayer-hidden%d" % (layers, hidden), "dataset": name, "nodes": g.n,
                           "nnz_with_self_loops": g.nnz})
    elif a.config == "reddit-infer":
        from cgnn_amd.gnn.gcn_deep import GCNInference
        from cgnn_amd.gnn.layers import GCN
        hidden = a.hidden or 256
        steps, warmup = a.steps or 100, a.warmup or 5
        g = _graph("reddit")
        model = GCN([g.n_features, hidden, g.n_classes], seed=a.seed).to(dev).eval()
        inf = GCNInference.from_model(g, model, dtype=torch.float16, capture=capture)
        setup = time.perf_counter() - t_setup
        for _ in range(warmup):
            inf()
        _sync(dev)
        lat = []
        if dev.type == "cuda":
            st = torch.cuda.current_stream()
            for _ in range(steps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                inf()
                e1.record(st)
                e1.synchronize()
                lat.append(e0.elapsed_time(e1))
        else:
            for _ in range(steps):
                t0 = time.perf_counter()
                inf()
                lat.append(1e3 * (time.perf_counter() - t0))
        lat = np.array(lat)
        dt = lat.sum() / 1e3
        res.update(metric="latency, 2-layer GCN reddit full-graph inference", value=round(float(np.median(lat)), 4),
                   unit="ms", higher_is_better=False, p99_ms=round(float(np.percentile(lat, 99)), 4),
                   mean_ms=round(float(lat.mean()), 4), dtype=str(inf.dtype).replace("torch.", ""),
                   hipgraph=bool(inf._graph.graph is not None),
                   config={"model": "GCN-2layer-hidden%d" % hidden, "dataset": "reddit", "nodes": g.n,
                           "nnz_with_self_loops": g.nnz})
    elif a.config == "products-sage3":
        from cgnn_amd.gnn.sage import SAGETrainer
        hidden = a.hidden or 256
        steps, warmup = a.steps or 2, a.warmup or 1
        g = _graph("ogbn-products")
        tr = SAGETrainer(g, hidden=hidden, layers=3, dropout=0.5, lr=0.003, fanouts=(15, 10, 5),
                         batch_size=1024, seed=a.seed, fused=False if a.unfused else None,
                         sampler=a.sampler)
        setup = time.perf_counter() - t_setup
        per_epoch = len(tr._batches())
        dt = _timed(tr.train_epoch, steps, warmup, dev)
        ev = tr.evaluate()
        if world > 1 and tr.fused:          # DP replicas must stay bitwise identical
            import torch.distributed as dist
            pr = tr._fused.params.clone()
            pmax, pmin = pr.clone(), pr.clone()
            dist.all_reduce(pmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(pmin, op=dist.ReduceOp.MIN)
            res["replicas_identical"] = bool(torch.equal(pmax, pmin))
        seeds = len(tr.train_idx) * steps
        res.update(metric="epochs/sec + val-acc, 3-layer GraphSAGE ogbn-products mini-batch DP",
                   value=round(steps / dt, 4), unit="epochs/s", ms_per_step=round(1e3 * dt / steps, 3),
                   seeds_per_s=round(seeds / dt, 1), iterations_per_epoch=per_epoch, fused=bool(tr.fused),
                   sampler=tr.sampler,
                   val_acc=round(ev["val_acc"], 4), test_acc=round(ev["test_acc"], 4),
                   dtype="bf16 (fp32 accumulation, fp32 master weights)" if dev.type == "cuda" else "fp32",
                   scaling="strong (fixed global epoch; per-rank batch 1024)",
                   config={"model": "SAGE-3layer-hidden%d" % hidden, "fanouts": [15, 10, 5],
                           "batch_per_rank": 1024, "parallelism": "dp%d" % world, "nodes": g.n})
    else:
        from cgnn_amd.gnn.data import synthetic_shard
        from cgnn_amd.gnn.gat import ShardedGATTrainer
        steps, warmup = a.steps or 10, a.warmup or 2
        emu = (a.emulate_rank, a.emulate_world) if a.emulate_world > 1 else None
        srank, sworld = emu if emu else (rank, world)
        t0 = time.perf_counter()
        order = None
        if a.partition == "locality":
            # once per job (rank 0, every core) and broadcast: each rank computing the
            # whole 111 M-node pass held its own 13 GB structure and ran it on 1/8 of the cores
            from cgnn_amd.gnn.data import shared_partition_order
            # the cache holds what it was computed for; another seed or scale at the same n
            # would pass synthetic_shard's permutation check and silently skew the timing
            ident = np.array([a.seed, int(round(a.scale * 1e9))], dtype=np.int64)
            cached = None
            if a.order_cache and world == 1 and os.path.exists(a.order_cache):
                z = np.load(a.order_cache)          # a bare .npy (older caches) has no identity
                if isinstance(z, np.lib.npyio.NpzFile):
                    if ("ident" in z.files and "dataset" in z.files and str(z["dataset"]) == "ogbn-papers100M"
                            and np.array_equal(z["ident"], ident)):
                        cached = z["order"]
                    z.close()
                _progress("partition order from %s" % a.order_cache if cached is not None
                          else "order cache %s is for another graph: recomputing" % a.order_cache)
            if cached is not None:
                order = cached
            else:
                _progress("partition order (rank 0 computes, then broadcast)")
                order = shared_partition_order("ogbn-papers100M", seed=a.seed, scale=a.scale)
                if a.order_cache and world == 1:
                    with open(a.order_cache, "wb") as fh:
                        np.savez(fh, order=order, ident=ident, dataset=np.array("ogbn-papers100M"))
        part_s = time.perf_counter() - t0
        _progress("partition done in %.1f s; generating the shard" % part_s)
        shard = synthetic_shard("ogbn-papers100M", srank, sworld, seed=a.seed, device=dev, scale=a.scale,
                                order=order)
        del order
        gen_s = time.perf_counter() - t0 - part_s
        _progress("shard generated in %.1f s" % gen_s)
        if world > 1:                     # every rank's setup split, reported by rank 0
            import torch.distributed as dist
            split = [None] * world
            from cgnn_amd.gnn import data as gdata
            mine = {"partition_s": round(part_s, 2), "gen_s": round(gen_s, 2)}
            if a.partition == "locality":      # waiting in the broadcast vs running the pass
                mine.update(partition_computed_here=gdata.LAST_PARTITION["computed_here"],
                            partition_compute_s=gdata.LAST_PARTITION["compute_s"])
            dist.all_gather_object(split, mine)
            res["setup_per_rank"] = split
        n_nodes, nnz_local, n_local = shard.n, shard.nnz, shard.n_local
        tr = ShardedGATTrainer(shard, heads=4, head_dim=32, dropout=0.5, lr=0.005, seed=a.seed, emulate=emu,
                               fused=False if a.unfused else None)
        if tr.halo is not None and a.halo_grad_bf16:
            tr.halo.grad_wire = torch.bfloat16
        del shard
        setup = time.perf_counter() - t_setup
        _progress("trainer ready (setup %.1f s); timing %d + %d epochs" % (setup, warmup, steps))
        if dev.type == "cuda":
            torch.cuda.reset_peak_memory_stats(dev)
        dt = _timed(tr.train_step, steps, warmup, dev)
        ev = tr.evaluate()
        peak = torch.cuda.max_memory_allocated(dev) / 2 ** 30 if dev.type == "cuda" else None
        res.update(metric="epochs/sec + val-acc, 2-layer GAT ogbn-papers100M, graph sharded",
                   value=round(steps / dt, 4), unit="epochs/s", ms_per_step=round(1e3 * dt / steps, 3),
                   val_acc=round(ev["val_acc"], 4), test_acc=round(ev["test_acc"], 4),
                   dtype="bf16 storage of the edge-gathered / halo rows, fp32 scores, accumulation and gradients"
                   if dev.type == "cuda" else "fp32",
                   peak_gpu_mem_gib=round(peak, 2) if peak is not None else None,
                   shard={"rank": srank, "world": sworld, "rows": n_local, "nnz": nnz_local, "gen_s": round(gen_s, 2),
                          "partition": a.partition, "partition_s": round(part_s, 2), "rank_local_generation": True,
                          "partition_computed_by": "rank 0, broadcast" if world > 1 else "this process"},
                   halo=tr.halo_stats(), emulated=emu is not None, reordered=a.partition == "locality",
                   fused=tr.fused is not None,
                   layer1_train_pruned=bool(tr.fused is not None and tr.fused._g1 is not None),
                   note=("DRY RUN: one rank of %d in one process; received halo rows are zero (their train flags "
                         "are generated locally, so the layer-1 pruning is the real one), so timing / memory "
                         "are those of the rank's kernels and buffers without communication, accuracy is not "
                         "meaningful" % sworld) if emu else None,
                   config={"model": "GAT-2layer-4x32", "parallelism": "graph-rowpart%d" % sworld, "nodes": n_nodes})
    res.update(steps=steps, warmup=warmup, setup_s=round(setup, 2), data="synthetic graph of the named shape "
               "(planted communities, shuffled ids), random-init weights")
    res.setdefault("reordered", a.reorder != "none")
    res.setdefault("higher_is_better", True)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
