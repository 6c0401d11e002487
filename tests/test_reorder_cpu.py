"""Shuffled synthetic ids and the locality reordering pass (csrc/runtime/reorder.cpp)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from cgnn_amd import native
from cgnn_amd.gnn.data import locality, reorder, synthetic
from cgnn_amd.gnn.gcn import GCNTrainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 65537])
def test_id_permutation_is_a_bijection(n):
    p = np.asarray(native.rt().id_permutation(n, 7, np.arange(n)))
    assert np.array_equal(np.sort(p), np.arange(n))
    if n > 100:
        assert np.mean(p == np.arange(n)) < 0.01


def test_shuffled_graph_is_the_banded_graph_relabelled():
    rt = native.rt()
    n, m = 5000, 40000
    s0, d0, x0, y0 = (np.asarray(a) for a in rt.synthetic_graph(n, m, 8, 5, 0.8, 1.0, 3, 0.1, 0))
    s1, d1, x1, y1 = (np.asarray(a) for a in rt.synthetic_graph(n, m, 8, 5, 0.8, 1.0, 3, 0.1, 1))
    # the bijection the generator used, recovered from the labels + features of every node
    perm = np.asarray(rt.id_permutation(n, 3 ^ 0x5A17, np.arange(n)))
    assert np.array_equal(s1, perm[s0]) and np.array_equal(d1, perm[d0])
    assert np.array_equal(y1[perm], y0) and np.array_equal(x1[perm], x0)


def test_reorder_restores_locality_and_is_a_permutation():
    g = synthetic("ogbn-products", seed=0, scale=0.01)           # shuffled ids (default)
    before = locality(g)
    g2, nid = reorder(g)
    assert torch.equal(torch.sort(nid).values, torch.arange(g.n))
    after = locality(g2)
    assert before[256] < 0.05 and after[1024] > 0.6, (before, after)
    banded = locality(synthetic("ogbn-products", seed=0, scale=0.01, id_order="banded"))
    assert after[4096] > banded[4096] - 0.05
    # same graph: edge (u, v) of g is edge (nid[u], nid[v]) of g2; node data follows
    rp, col = g.rowptr.long(), g.col.long()
    rows = torch.repeat_interleave(torch.arange(g.n), rp[1:] - rp[:-1])
    e1 = set((nid[rows] * g.n + nid[col]).tolist())
    rp2, col2 = g2.rowptr.long(), g2.col.long()
    rows2 = torch.repeat_interleave(torch.arange(g.n), rp2[1:] - rp2[:-1])
    assert e1 == set((rows2 * g.n + col2).tolist())
    assert torch.equal(g2.x[nid], g.x) and torch.equal(g2.y[nid], g.y) and torch.equal(g2.mask[nid], g.mask)
    assert torch.equal(g2.dinv[nid], g.dinv)


def test_reorder_is_independent_of_thread_count():
    code = ("import numpy as np; from cgnn_amd.gnn.data import synthetic, reorder; "
            "g = synthetic('ogbn-products', seed=1, scale=0.003); print(int(np.asarray(reorder(g)[1]) @ "
            "np.arange(g.n, dtype=np.int64) % 1000000007))")
    outs = []
    for t in ("1", "5"):
        env = dict(os.environ, OMP_NUM_THREADS=t, PYTHONPATH=ROOT)
        outs.append(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                   check=True).stdout.strip())
    assert outs[0] == outs[1]


def test_gcn_loss_is_invariant_under_reorder():
    g = synthetic("ogbn-products", seed=2, scale=0.002)
    a = GCNTrainer(g, hidden=32, dropout=0.0, seed=0, rank=0, world=1)
    b = GCNTrainer(g, hidden=32, dropout=0.0, seed=0, rank=0, world=1, reorder=True)
    for _ in range(3):
        a.train_step()
        b.train_step()
    ra, rb = a.evaluate(), b.evaluate()
    for k in ra:
        assert abs(ra[k] - rb[k]) < 2e-3, (k, ra, rb)


@pytest.mark.parametrize("world,id_order", [(3, "shuffled"), (2, "banded")])
def test_shards_reassemble_the_full_graph(world, id_order):
    """Rank-local shard generation gives exactly the rows of the full build."""
    from cgnn_amd.gnn.data import synthetic_shard
    full = synthetic("ogbn-products", seed=5, scale=0.002, id_order=id_order)
    parts = [synthetic_shard("ogbn-products", r, world, seed=5, scale=0.002, id_order=id_order) for r in range(world)]
    assert sum(p.n_local for p in parts) == full.n and all(p.n == full.n for p in parts)
    rp = torch.cat([parts[0].rowptr.long()] + [p.rowptr.long()[1:] + sum(q.nnz for q in parts[:i])
                                               for i, p in enumerate(parts) if i > 0])
    assert torch.equal(rp, full.rowptr.long())
    assert torch.equal(torch.cat([p.col for p in parts]), full.col)
    assert torch.equal(torch.cat([p.x for p in parts]), full.x)
    assert torch.equal(torch.cat([p.y for p in parts]), full.y)
    assert torch.equal(torch.cat([p.mask for p in parts]), full.mask)


@pytest.mark.parametrize("world", [2, 3])
def test_locality_shards_reassemble_the_reordered_graph(world):
    """partition='locality': the shards are exactly the rows of reorder(synthetic(...)),
    and every shard can flag any global row as train or not (the dry run's halo flags)."""
    from cgnn_amd.gnn.data import partition_order, synthetic_shard
    full, nid = reorder(synthetic("ogbn-products", seed=5, scale=0.002), seed=5)
    order = partition_order("ogbn-products", seed=5, scale=0.002)
    assert np.array_equal(order, nid.numpy())
    parts = [synthetic_shard("ogbn-products", r, world, seed=5, scale=0.002, order=order) for r in range(world)]
    rp = torch.cat([parts[0].rowptr.long()] + [p.rowptr.long()[1:] + sum(q.nnz for q in parts[:i])
                                               for i, p in enumerate(parts) if i > 0])
    assert torch.equal(rp, full.rowptr.long())
    assert torch.equal(torch.cat([p.col for p in parts]), full.col)
    assert torch.equal(torch.cat([p.x for p in parts]), full.x)
    assert torch.equal(torch.cat([p.y for p in parts]), full.y)
    assert torch.equal(torch.cat([p.mask for p in parts]), full.mask)
    rows = torch.arange(full.n)
    assert torch.equal(parts[0].train_flags(rows), full.mask == 1)


def test_locality_partition_shrinks_the_halo():
    """Rank 0 of 8: the rows its edges read from other ranks, shuffled ids vs the
    locality partition (the papers100M dry run's halo, at a small scale)."""
    from cgnn_amd.gnn.data import synthetic_shard
    world = 8
    kw = dict(seed=1, scale=0.02)
    plain = synthetic_shard("ogbn-products", 0, world, **kw)
    loc = synthetic_shard("ogbn-products", 0, world, partition="locality", **kw)

    def halo(sh):
        c = sh.col.long()
        return torch.unique(c[(c < sh.r0) | (c >= sh.r1)]).numel()
    h0, h1 = halo(plain), halo(loc)
    # the 20 % uniformly random edges (homophily 0.8) bound any partition from below:
    # ~n_other (1 - exp(-0.2 nnz_local / n_other)) distinct remote rows
    n_other = plain.n - plain.n_local
    floor = n_other * (1 - np.exp(-0.2 * loc.nnz / n_other))
    assert h1 < 0.75 * h0, (h0, h1)
    assert h1 < 1.15 * floor, (h1, floor)


def test_id_permutation_inverse():
    rt = native.rt()
    ids = np.arange(10007)
    p = np.asarray(rt.id_permutation(10007, 9, ids))
    assert np.array_equal(np.asarray(rt.id_permutation(10007, 9, p, True)), ids)


def test_median_refinement_is_a_permutation_and_narrows_the_band():
    """locality_refine (optional 4th stage of the reorder pass): a permutation that puts
    more edges within a short distance of the diagonal."""
    g = synthetic("ogbn-products", seed=0, scale=0.01)
    base = reorder(g, refine=0)[1]
    g2, nid = reorder(g, refine=3)
    assert torch.equal(torch.sort(nid).values, torch.arange(g.n))
    w = (64, 256)
    lb = locality(g, w, new_id=base.numpy())
    lr = locality(g, w, new_id=nid.numpy())
    assert lr[64] > lb[64] and lr[256] > lb[256], (lb, lr)


def test_shard_rejects_an_order_that_is_not_a_permutation():
    """a duplicate or out-of-range entry in ``order`` would leave rows without
    ids (split mask and labels read garbage): the generator refuses it."""
    from cgnn_amd.gnn.data import partition_order, synthetic_shard
    order = partition_order("ogbn-products", seed=5, scale=0.002)
    bad = order.copy()
    bad[1] = bad[0]                                   # a duplicate
    with pytest.raises(ValueError, match="permutation"):
        synthetic_shard("ogbn-products", 0, 2, seed=5, scale=0.002, order=bad)
    bad = order.copy()
    bad[3] = len(order)                               # out of range
    with pytest.raises(ValueError, match="permutation"):
        synthetic_shard("ogbn-products", 0, 2, seed=5, scale=0.002, order=bad)
