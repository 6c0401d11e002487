"""Node-property-prediction datasets for the GNN track (not in the reference).

There is no network access, so the OGB / Planetoid datasets are replaced by
synthetic graphs *of the same shape* (nodes, undirected edges, feature width,
classes, split sizes) from the C++ generator ``_rt.synthetic_graph``: planted
communities (one per class), homophilous edges joining nearby members of the
community, the rest uniform over the graph; node labels follow the community
except for a ``label_noise`` fraction, and features = centroid of the node's
label + Gaussian noise -- so neither the graph nor the features alone determine
the label and a GCN reaches a non-saturated accuracy (a synthetic-task number,
not comparable with any real-dataset accuracy).

Node ids: ``id_order="shuffled"`` (default) relabels every node through a seeded
bijection, so -- as with a real dataset -- ids carry no locality; ``"banded"``
keeps the generator's ids, whose homophilous edges join nearby ids (locality
handed out for free, kept only for A/B measurements).  :func:`reorder` is the
framework's own locality pass (label-propagation clusters laid out by a walk of
the cluster graph, Cuthill-McKee inside each cluster, median-smoothing refinement;
``csrc/runtime/reorder.cpp``)
that trainers run at setup.

The CSR holds A + I, symmetrised and de-duplicated; the GCN normalisation
D^-1/2 (A+I) D^-1/2 is kept as the vector ``dinv``.  On a GPU the CSR is built
with device sorts; on the CPU with the C++ runtime.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import numpy as np
import torch

from .. import native

# name: (nodes, undirected edges, features, classes, train, valid)  -- public dataset shapes
SHAPES = {
    "cora": (2708, 5278, 1433, 7, 140, 500),
    "citeseer": (3327, 4552, 3703, 6, 120, 500),
    "pubmed": (19717, 44324, 500, 3, 60, 500),
    "ogbn-arxiv": (169343, 1166243, 128, 40, 90941, 29799),
    "ogbn-products": (2449029, 61859140, 100, 47, 196615, 39323),
    "reddit": (232965, 57307946, 602, 41, 153431, 23831),
    "ogbn-papers100M": (111059956, 1615685872, 128, 172, 1207179, 125265),
}


@dataclasses.dataclass
class GraphData:
    n: int
    rowptr: torch.Tensor      # int32 [n+1] (A + I)
    col: torch.Tensor         # int32 [nnz]
    dinv: torch.Tensor        # fp32 [n]  (deg of A+I)^-1/2
    x: torch.Tensor           # fp32 [n, F] raw features
    y: torch.Tensor           # int32 [n]
    mask: torch.Tensor        # uint8 [n]: 1 train, 2 valid, 3 test
    n_classes: int
    name: str = "synthetic"

    @property
    def nnz(self):
        return int(self.col.numel())

    @property
    def n_features(self):
        return int(self.x.shape[1])

    def to(self, device):
        f = {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in dataclasses.asdict(self).items()}
        return GraphData(**f)


def build_csr(n: int, src: np.ndarray, dst: np.ndarray, device=None):
    """A + I symmetrised, de-duplicated CSR (int32 rowptr / col) on ``device``."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    if device.type == "cuda":
        s = torch.as_tensor(src, device=device, dtype=torch.int64)
        d = torch.as_tensor(dst, device=device, dtype=torch.int64)
        keep = s != d
        s, d = s[keep], d[keep]
        loops = torch.arange(n, device=device, dtype=torch.int64)
        rows = torch.cat([s, d, loops])
        cols = torch.cat([d, s, loops])
        del s, d
        key = torch.unique(rows * n + cols)          # sorted + de-duplicated
        del rows, cols
        r = key // n
        c = (key - r * n).to(torch.int32)
        counts = torch.bincount(r, minlength=n)
        rowptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
        rowptr[1:] = torch.cumsum(counts, 0)
        if rowptr[-1] >= 2 ** 31:
            raise ValueError("nnz >= 2^31 needs int64 CSR (graph must be sharded)")
        return rowptr.to(torch.int32), c
    rp, col = native.rt().csr_from_edges(n, np.asarray(src, np.int64), np.asarray(dst, np.int64),
                                         True, True, True)
    return torch.from_numpy(np.asarray(rp).astype(np.int32)), torch.from_numpy(np.asarray(col))


ID_ORDERS = {"banded": 0, "shuffled": 1}


def synthetic(name: str = "ogbn-products", seed: int = 0, device=None, scale: float = 1.0,
              homophily: float = 0.8, feat_noise: float = 4.0, label_noise: float = 0.25,
              id_order: str = "shuffled") -> GraphData:
    """Synthetic graph with the shape of ``name`` (``scale`` shrinks nodes and edges)."""
    n, m, F, C, n_train, n_val = SHAPES[name]
    n = max(int(n * scale), C * 4)
    m = max(int(m * scale), n)
    n_train = max(int(n_train * scale), C)
    n_val = max(int(n_val * scale), C)
    src, dst, x, y = native.rt().synthetic_graph(n, m, F, C, homophily, feat_noise, seed, label_noise,
                                                 ID_ORDERS[id_order])
    rowptr, col = build_csr(n, np.asarray(src), np.asarray(dst), device)
    del src, dst
    device = rowptr.device
    deg = (rowptr[1:] - rowptr[:-1]).to(torch.float32)
    dinv = deg.clamp_min(1).rsqrt()
    # split: train / valid / test by a per-node hash with OGB's split proportions (a pure
    # function of the node id, so a graph shard labels its rows without the full graph).
    # The split SIZES are therefore random counts near OGB's (binomial around them), not
    # the exact numbers; trainers normalise the loss by the real global train count
    # (an emulated dry-run rank, which cannot count other ranks' rows, uses the nominal
    # ``n_train_global`` of its shard -- its loss scale differs by that ratio).
    mask = np.asarray(native.rt().split_mask(n, n_train, n_val, seed + 1, np.arange(n, dtype=np.int64)))
    return GraphData(n=n, rowptr=rowptr, col=col, dinv=dinv.to(device),
                     x=torch.from_numpy(np.asarray(x)).to(device),
                     y=torch.from_numpy(np.asarray(y).astype(np.int32)).to(device),
                     mask=torch.from_numpy(mask).to(device), n_classes=C, name=name + "-synthetic")


def partition_rows(g: GraphData, rank: int, world: int):
    """Contiguous row block of ``rank`` (equal sizes, last one padded): local CSR
    with global column ids, plus the row range."""
    per = (g.n + world - 1) // world
    r0, r1 = min(g.n, rank * per), min(g.n, (rank + 1) * per)
    rp = g.rowptr[r0:r1 + 1].to(torch.int64)
    col = g.col[int(rp[0]): int(rp[-1])]
    rp = (rp - rp[0]).to(torch.int32)
    return r0, r1, per, rp, col


@dataclasses.dataclass
class GraphShard:
    """Rows [r0, r1) of an n-node graph (A + I, symmetric): CSR with GLOBAL column ids,
    the rows' features / labels / split.  Built by :func:`synthetic_shard` without the
    rest of the graph.  ``rowptr`` is int32 when the shard's nnz fits, else int64."""
    n: int
    r0: int
    r1: int
    rowptr: torch.Tensor
    col: torch.Tensor
    x: torch.Tensor
    y: torch.Tensor
    mask: torch.Tensor
    n_classes: int
    n_train_global: int = 0
    name: str = "synthetic-shard"
    # train flags of any global rows (rows of other ranks included): generation is
    # deterministic, so a one-rank dry run can flag the rows its halo would receive
    train_flags: Optional[object] = None

    @property
    def n_local(self):
        return self.r1 - self.r0

    @property
    def nnz(self):
        return int(self.col.numel())


def shard_rows(n: int, rank: int, world: int):
    """Row block of ``rank``: contiguous, equal sizes (the last one shorter)."""
    per = (n + world - 1) // world
    return rank * per, min(n, (rank + 1) * per), per


def _scaled_shape(name: str, scale: float):
    n, m, F, C, n_train, n_val = SHAPES[name]
    n = max(int(n * scale), C * 4)
    m = max(int(m * scale), n)
    n_train = max(int(n_train * scale), C)
    n_val = max(int(n_val * scale), C)
    return n, m, F, C, n_train, n_val


def partition_order(name: str, seed: int = 0, scale: float = 1.0, homophily: float = 0.8,
                    id_order: str = "shuffled", rounds: int = 8, max_cluster: int = 4096) -> np.ndarray:
    """Locality partition of ``synthetic(name, ...)`` computed from its structure alone:
    the framework's reorder pass (label-propagation clusters + Cuthill-McKee over them,
    ``reorder``) over the whole graph's CSR, generated without features (O(nnz) host
    memory: 13 GB of column ids for the papers100M shape).  Node ``f`` becomes row
    ``order[f]``; a rank then owns the contiguous block ``shard_rows(n, rank, world)`` of
    the new order, i.e. whole communities instead of random ids.  Deterministic for any
    thread count, so every rank computes the same order without an exchange."""
    n, m, F, C, _, _ = _scaled_shape(name, scale)
    rt = native.rt()
    rp, col = rt.synthetic_shard(n, m, F, C, homophily, 0.0, seed, 0.0, ID_ORDERS[id_order], 0, n,
                                 with_features=False)[:2]
    order = np.asarray(rt.locality_order(n, np.asarray(rp), np.asarray(col), rounds, max_cluster, seed))
    del rp, col
    return order


# who ran the last shared_partition_order pass in this process, and for how long
LAST_PARTITION = {"computed_here": False, "compute_s": 0.0}


def shared_partition_order(name: str, seed: int = 0, scale: float = 1.0, **kw) -> np.ndarray:
    """``partition_order`` computed ONCE per job: rank 0 runs the pass with every CPU of
    its node (the other ranks wait in the broadcast, holding no copy of the structure)
    and broadcasts the order (parallel.dist.broadcast_host_array).  One process: plain
    ``partition_order``."""
    import time
    from ..parallel import dist as pdist
    global LAST_PARTITION
    if not pdist.is_distributed():
        t = time.perf_counter()
        order = partition_order(name, seed=seed, scale=scale, **kw)
        LAST_PARTITION = {"computed_here": True, "compute_s": round(time.perf_counter() - t, 2)}
        return order
    n = _scaled_shape(name, scale)[0]
    order = None
    LAST_PARTITION = {"computed_here": False, "compute_s": 0.0}
    err = None
    if pdist.rank() == 0:
        pdist.set_host_threads(pdist.host_cpus())
        t = time.perf_counter()
        try:
            order = partition_order(name, seed=seed, scale=scale, **kw)
        except Exception as e:                # the other ranks learn it from the status word
            err = e
        finally:
            pdist.set_host_threads()          # back to this rank's share
        LAST_PARTITION = {"computed_here": True, "compute_s": round(time.perf_counter() - t, 2)}
    dt = np.int32 if n < (1 << 31) else np.int64
    try:
        out = pdist.broadcast_host_array(None if order is None else order.astype(dt), n, dtype=dt)
    except RuntimeError:
        if err is not None:
            raise err
        raise
    return out.astype(np.int64)


def synthetic_shard(name: str, rank: int, world: int, seed: int = 0, device=None, scale: float = 1.0,
                    homophily: float = 0.8, feat_noise: float = 4.0, label_noise: float = 0.25,
                    id_order: str = "shuffled", feature_dtype=torch.float32, partition: str = "none",
                    order: Optional[np.ndarray] = None) -> GraphShard:
    """This rank's rows of ``synthetic(name, ...)`` -- the same graph, generated shard-locally
    (the C++ generator hashes every edge once and keeps those touching the shard; memory
    is O(shard)).  ``feature_dtype`` bf16 halves the feature bytes of a 10^8-node graph.
    ``partition="locality"`` (or an explicit ``order``): the rows of the graph relabelled by
    :func:`partition_order`, so the rank owns communities and its halo shrinks; the
    graph equals ``reorder(synthetic(...))`` of the same arguments."""
    n, m, F, C, n_train, n_val = _scaled_shape(name, scale)
    if order is None and partition == "locality":
        order = partition_order(name, seed=seed, scale=scale, homophily=homophily, id_order=id_order)
    elif partition not in ("none", "locality"):
        raise ValueError("partition must be 'none' or 'locality'")
    r0, r1, _ = shard_rows(n, rank, world)
    rt = native.rt()
    ordv = np.zeros(0, np.int64) if order is None else np.asarray(order, np.int64)
    rp, col, x, y, ids = rt.synthetic_shard(n, m, F, C, homophily, feat_noise, seed, label_noise,
                                            ID_ORDERS[id_order], r0, r1, order=ordv)
    rp = np.asarray(rp)
    rp_t = torch.from_numpy(rp.astype(np.int32) if rp[-1] < 2 ** 31 else rp)
    mask = np.asarray(rt.split_mask(n, n_train, n_val, seed + 1, np.asarray(ids, np.int64)))
    dev = torch.device(device) if device is not None else torch.device("cpu")
    xt = torch.from_numpy(np.asarray(x))
    if feature_dtype != torch.float32:
        xt = xt.to(feature_dtype)
    inv = None
    if order is not None:
        inv = np.empty(n, np.int64)
        inv[ordv] = np.arange(n, dtype=np.int64)

    def train_flags(rows: torch.Tensor) -> torch.Tensor:
        """Train flag of global rows (of this shard's numbering)."""
        r = rows.detach().cpu().numpy().astype(np.int64)
        f = inv[r] if inv is not None else r
        return torch.from_numpy(np.asarray(rt.split_mask(n, n_train, n_val, seed + 1, f)) == 1).to(rows.device)

    tag = "-locality" if order is not None else ""
    return GraphShard(n=n, r0=r0, r1=r1, rowptr=rp_t.to(dev), col=torch.from_numpy(np.asarray(col)).to(dev),
                      x=xt.to(dev), y=torch.from_numpy(np.asarray(y).astype(np.int32)).to(dev),
                      mask=torch.from_numpy(mask).to(dev), n_classes=C, n_train_global=n_train,
                      name="%s-synthetic%s-shard%d/%d" % (name, tag, rank, world), train_flags=train_flags)


def locality(g: GraphData, windows=(64, 256, 1024, 4096, 65536), new_id=None):
    """Fraction of the (non-loop) CSR entries whose endpoints are within w ids, per
    window w: the reuse a row-ordered gather can find in L2 / the Infinity Cache."""
    rp = g.rowptr.cpu().numpy().astype(np.int64)
    col = g.col.cpu().numpy()
    nid = np.zeros(0, np.int64) if new_id is None else np.asarray(new_id, np.int64)
    return dict(zip(windows, native.rt().locality_stats(g.n, rp, col, nid, list(windows))))


def reorder(g: GraphData, rounds: int = 8, max_cluster: int = 4096, seed: int = 0,
            refine: int = 0):
    """Relabel the nodes of ``g`` for gather locality (``csrc/runtime/reorder.cpp``):
    label-propagation clusters + Cuthill-McKee, then ``refine`` rounds of median
    smoothing (default 0: on the products shape 4 rounds
    narrow the band -- edges within +-256 positions 56 -> 74 % -- yet the GCN epoch
    measured 5 % SLOWER, 197 vs 210 epochs/s: the cluster-walk order's grouping of whole
    communities serves the per-XCD L2 better than a tighter diagonal band).

    Returns ``(g2, new_id)``: ``g2`` is the same graph with node ``v`` renamed
    ``new_id[v]`` (CSR rows, features, labels, split and normalisation permuted
    alike, so losses and accuracies are unchanged), ``new_id`` an int64 tensor on
    the CPU.  Deterministic for any thread count, so every rank of a multi-GPU job
    computes the same order independently."""
    rt = native.rt()
    rp = g.rowptr.cpu().numpy().astype(np.int64)
    col = g.col.cpu().numpy()
    new_id = rt.locality_order(g.n, rp, col, rounds, max_cluster, seed)
    if refine > 0:
        new_id = rt.locality_refine(g.n, rp, col, new_id, refine)
    rp2, col2 = rt.permute_csr(g.n, rp, col, new_id)
    del rp, col
    dev = g.rowptr.device
    nid = torch.from_numpy(np.asarray(new_id))
    old_of = torch.empty_like(nid)
    old_of[nid] = torch.arange(g.n, dtype=torch.int64)
    o = old_of.to(dev)
    rp2 = np.asarray(rp2)
    if rp2[-1] >= 2 ** 31:
        raise ValueError("nnz >= 2^31 needs int64 CSR (graph must be sharded)")
    g2 = GraphData(n=g.n, rowptr=torch.from_numpy(rp2.astype(np.int32)).to(dev),
                   col=torch.from_numpy(np.asarray(col2)).to(dev), dinv=g.dinv[o], x=g.x[o], y=g.y[o],
                   mask=g.mask[o], n_classes=g.n_classes, name=g.name + "-reordered")
    return g2, nid
