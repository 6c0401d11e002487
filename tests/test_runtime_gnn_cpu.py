"""Host C++ runtime (_rt), synthetic generators and the GNN track on CPU."""
import math

import numpy as np
import pandas as pd
import pytest
import torch

from cgnn_amd import native
from cgnn_amd.generators import RandomGraphGenerator, functions_default as fd
from cgnn_amd.gnn import ops
from cgnn_amd.gnn.data import SHAPES, build_csr, partition_rows, synthetic
from cgnn_amd.gnn.gcn import GCNTrainer
from cgnn_amd.utils.formats import CCEPC_PairsFileReader


def test_csr_builder_symmetric_dedup_self_loops():
    rt = native.rt()
    rp, col = rt.csr_from_edges(4, np.array([0, 0, 1, 2, 2]), np.array([1, 1, 2, 2, 3]), True, True, True)
    rp, col = np.asarray(rp), np.asarray(col)
    rows = {i: sorted(col[rp[i]:rp[i + 1]].tolist()) for i in range(4)}
    assert rows == {0: [0, 1], 1: [0, 1, 2], 2: [1, 2, 3], 3: [2, 3]}


def test_build_csr_matches_dense_adjacency():
    rng = np.random.default_rng(0)
    n = 50
    src, dst = rng.integers(0, n, 300), rng.integers(0, n, 300)
    rp, col = build_csr(n, src, dst, "cpu")
    A = np.zeros((n, n), bool)
    A[src, dst] = A[dst, src] = True
    np.fill_diagonal(A, True)
    B = np.zeros((n, n), bool)
    for i in range(n):
        B[i, col[rp[i]:rp[i + 1]].numpy()] = True
    assert (A == B).all()


def test_dag_acyclicity_and_hash():
    rt = native.rt()
    assert rt.is_acyclic(3, [(0, 1), (1, 2)]) and not rt.is_acyclic(2, [(0, 1), (1, 0)])
    assert rt.canonical_hash([(0, 1), (2, 3)]) == rt.canonical_hash([(2, 3), (0, 1)])
    assert rt.canonical_hash([(0, 1)]) != rt.canonical_hash([(1, 0)])


def test_neighbor_sampler_blocks():
    g = synthetic("cora", seed=0)
    seeds = np.arange(10)
    blocks = native.rt().sample_neighbors(g.rowptr.numpy().astype(np.int64), g.col.numpy(), seeds, [5, 3], 7)
    assert len(blocks) == 2
    rp, col, nodes = (np.asarray(x) for x in blocks[0])
    assert len(rp) == 11 and np.all(np.diff(rp) <= 5)
    assert list(nodes[:10]) == list(seeds)            # destination nodes are a prefix
    assert col.max() < len(nodes)
    # every sampled neighbour is a real neighbour
    for i in range(10):
        nb = set(g.col[g.rowptr[i]:g.rowptr[i + 1]].tolist())
        assert set(nodes[col[rp[i]:rp[i + 1]]].tolist()) <= nb


def test_synthetic_shapes_and_split():
    g = synthetic("ogbn-arxiv", seed=1, scale=0.01)
    n, m, F, C, ntr, nva = SHAPES["ogbn-arxiv"]
    assert g.n_features == F and g.n_classes == C
    assert int((g.mask == 1).sum()) == int(ntr * 0.01)
    assert g.y.max() < C
    r0, r1, per, rp, col = partition_rows(g, 1, 3)
    assert r0 == per and rp[-1] == col.numel()


def test_dropout_mask_is_partition_independent():
    full = ops.dropout_keep_mask(40, 64, 0.5, (1, 2), 3)
    part = ops.dropout_keep_mask(20, 64, 0.5, (1, 2), 3, row0=20)
    assert torch.equal(full[20:], part)
    assert 0.4 < full.float().mean() < 0.6


def _dense_norm_adj(g):
    n = g.n
    rows = torch.repeat_interleave(torch.arange(n), (g.rowptr[1:] - g.rowptr[:-1]).long())
    A = torch.zeros(n, n)
    A[rows, g.col.long()] = 1.0
    return g.dinv[:, None] * A * g.dinv[None, :]


@pytest.mark.parametrize("world", [1, 3])
def test_gcn_trainer_gradients_match_autograd(world):
    """The trainer's hand-written backward (compact train-row dlogits, train-column
    SpMM, split-K weight gradients) against PyTorch autograd of the same fp32 model;
    the world=3 case runs each rank's row block in one process (no collectives: the
    compact gradient slots of every rank are filled by hand)."""
    g = synthetic("ogbn-products", seed=3, scale=0.0015)
    trs = [GCNTrainer(g, hidden=32, dropout=0.0, seed=5, rank=r, world=world) for r in range(world)]
    tr0 = trs[0]
    W1 = tr0.W1.clone().requires_grad_()
    b1 = (torch.randn(32) * 0.1).requires_grad_()
    W2 = tr0.W2.clone().requires_grad_()
    b2 = (torch.randn(g.n_classes) * 0.1).requires_grad_()
    for tr in trs:
        tr.b1.copy_(b1.detach())
        tr.b2.copy_(b2.detach())
    A = _dense_norm_adj(g)
    X = g.x.to(torch.bfloat16).float()
    H = torch.relu(A @ X @ W1 + b1)
    logits = A @ (H @ W2) + b2
    tr_mask = g.mask == 1
    loss = torch.nn.functional.cross_entropy(logits[tr_mask], g.y[tr_mask].long())
    loss.backward()
    if world == 1:
        stats = tr0.forward(train=True)
        tr0.backward(stats)
        grads = tr0.grads
    else:
        # forward on every rank, then stitch the all-gathers by hand
        z2 = torch.zeros_like(tr0.Z2loc).repeat(world, 1)
        for r, tr in enumerate(trs):
            tr.Z2 = z2
        stats = []
        for r, tr in enumerate(trs):
            tr._aggregate_features(tr.AX)
            tr._ax_ready = True
            n = tr.nloc
            tr.W2b[:, :tr.C] = tr.W2.to(torch.bfloat16)
            H1 = tr.H1[:n]
            H1.copy_((tr.AX[:n, :tr.F].float() @ tr.W1.to(torch.bfloat16).float()).to(torch.bfloat16))
            ops.bias_relu_dropout_(H1, tr.b1, tr.hidden, 0.0, tr.key, tr.epoch, tr.r0)
            y2 = (H1.float() @ tr.W2b.float()) * tr.dinv[:, None]
            z2[r * tr.per: r * tr.per + n] = y2.to(torch.bfloat16)
        gc = torch.zeros(tr0.maxT * world, tr0.ldc, dtype=torch.bfloat16)
        for r, tr in enumerate(trs):
            st, _ = ops.spmm_ce(tr.rowptr, tr.col, z2, tr.C, tr.dinv, tr.b2, tr.y, tr.mask,
                                1.0 / tr.n_train, mode=0, G=tr.Gc_loc, gslot=tr.gslot)
            gc[r * tr.maxT:(r + 1) * tr.maxT] = tr.Gc_loc
            stats.append(st)
        grads = torch.zeros_like(tr0.grads)
        for r, tr in enumerate(trs):
            tr.Gc = gc
            tr.multi = False                 # backward without collectives
            tr.backward(stats[r])
            tr.multi = True
            grads += tr.grads
        grads[tr0.n_params - tr0.C:] = sum(s[4:4 + tr0.C] for s in stats)
    ref = torch.cat([W1.grad.flatten(), b1.grad, W2.grad.flatten(), b2.grad])
    scale = ref.abs().max()
    assert torch.allclose(grads, ref, atol=3e-2 * scale, rtol=0), float((grads - ref).abs().max() / scale)
    rel = (grads - ref).norm() / ref.norm()
    assert rel < 2e-2, float(rel)


def test_gcn_cpu_learns():
    g = synthetic("ogbn-products", seed=0, scale=0.005)
    tr = GCNTrainer(g, hidden=64)
    first = None
    for e in range(25):
        tr.train_step()
        if e == 0:
            first = tr.train_loss()
    res = tr.evaluate()
    assert tr.train_loss() < first
    assert res["val_acc"] > 0.4


def test_random_graph_generator(tmp_path):
    gen = RandomGraphGenerator(num_nodes=15, max_joint_causes=3, number_points=200, seed=3)
    G, data, cat, cat_idx = gen.generate()
    assert not G.is_cyclic()
    assert set(G.get_list_nodes()) == set(data.columns)
    effects = [c for c in data.columns if G.get_parents(c)]       # roots stay U(-1, 1)
    np.testing.assert_allclose(data[effects].values.mean(0), 0, atol=1e-9)
    roots = [c for c in data.columns if not G.get_parents(c)]
    assert len(roots) >= 2 and np.abs(data[roots].values).max() <= 1
    gen.save_data(str(tmp_path / "g"))
    t = pd.read_csv(tmp_path / "g_target.csv")
    assert list(t.columns) == ["Cause", "Effect"] and len(t) == len(G.get_list_edges())
    pairs, targets = gen.generate_pairs(4, prefix=str(tmp_path / "p"))
    df = CCEPC_PairsFileReader(str(tmp_path / "p_pairs.csv"))
    assert len(df) == 4 and set(targets.Target) <= {1.0, -1.0}


def test_mechanism_primitives():
    rng = np.random.default_rng(0)
    x = fd.cause(300, rng=rng)
    assert x.min() >= -1 and x.max() <= 1
    y = fd.effect(x, 300, 0.7, rng=rng)
    assert abs(y.mean()) < 1e-9 and abs(y.std() - 1) < 1e-9
    b = fd.rand_bin(y, rng=rng)
    assert b.dtype.kind == "i" and len(np.unique(b)) >= 2


def test_generators_module():
    from cgnn_amd.generators import (CGNN_generator, full_graph_polynomial_generator, linear_regressor,
                                     polynomial_regressor, support_vector_regressor)
    from cgnn_amd.utils.graph import DirectedGraph
    rng = np.random.default_rng(0)
    a = rng.normal(size=150)
    df = pd.DataFrame({"a": a, "b": a ** 2 + 0.1 * rng.normal(size=150)})
    g = DirectedGraph()
    g.add("a", "b")
    out = full_graph_polynomial_generator(df, g, train_epochs=20, gpu=False)
    assert out.shape == (150, 2) and np.isfinite(out.values).all()
    out = CGNN_generator(df, g, train_epochs=10, test_epochs=1, gpu=False)
    assert out.shape == (150, 2) and np.isfinite(out.values).all()
    y = polynomial_regressor(df[["a"]].values, df.b.values, ["a"], train_epochs=30)
    assert y.shape == (150,)
    assert linear_regressor(df[["a"]].values, df.b.values, ["a"]).shape == (150,)
    assert support_vector_regressor(df[["a"]].values, df.b.values, ["a"]).shape == (150,)


def test_sage_block_aggregate_and_backward():
    from cgnn_amd.gnn.sage import Block, mean_aggregate, transpose_csr
    rng = np.random.default_rng(0)
    n_src, n_dst = 30, 12
    rows = [rng.choice(n_src, size=rng.integers(0, 6), replace=False) for _ in range(n_dst)]
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])])
    col = np.concatenate([r for r in rows]).astype(np.int32)
    b = Block(rp, col, n_src, "cpu")
    rp_t, col_t = transpose_csr(b.rowptr, b.col, n_src)
    A = torch.zeros(n_dst, n_src, dtype=torch.float64)
    for i, r in enumerate(rows):
        A[i, torch.as_tensor(r, dtype=torch.long)] = 1.0 / max(len(r), 1)
    At = torch.zeros(n_src, n_dst)
    for i in range(n_src):
        At[i, col_t[rp_t[i]:rp_t[i + 1]].long()] = 1
    assert torch.equal(At, (A.t() > 0).float())
    h = torch.randn(n_src, 16, requires_grad=True)
    out = mean_aggregate(h, b)
    np.testing.assert_allclose(out.detach().numpy(), (A @ h.double()).detach().numpy(), rtol=1e-5, atol=1e-6)
    gout = torch.randn(n_dst, 16)
    out.backward(gout)
    np.testing.assert_allclose(h.grad.numpy(), (A.t() @ gout.double()).numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fanouts", [(5, 5), None])
def test_sage_learns_cpu(fanouts):
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-arxiv", seed=2, scale=0.01, feat_noise=2.0, label_noise=0.1)
    tr = SAGETrainer(g, hidden=64, fanouts=fanouts, batch_size=256, lr=0.01, prefetch=fanouts is not None)
    first = tr.train_epoch()
    for _ in range(12):
        last = tr.train_epoch()
    res = tr.evaluate()
    assert last < first
    assert res["val_acc"] > 0.3, res


def test_gat_aggregate_reference_matches_dense_softmax():
    from cgnn_amd.gnn.gat import GraphCSR, gat_aggregate
    n, K, Fh = 40, 2, 8
    rng = np.random.default_rng(4)
    rp, col = build_csr(n, rng.integers(0, n, 120), rng.integers(0, n, 120), "cpu")
    g = GraphCSR(rp, col, n)
    Wh = torch.randn(n, K * Fh, dtype=torch.float64)
    ss, sd = torch.randn(n, K, dtype=torch.float64), torch.randn(n, K, dtype=torch.float64)
    out = gat_aggregate(Wh, ss, sd, g, K, Fh)
    A = torch.zeros(n, n, dtype=torch.bool)
    for i in range(n):
        A[i, col[rp[i]:rp[i + 1]].long()] = True
    for k in range(K):
        e = torch.nn.functional.leaky_relu(sd[:, k:k + 1] + ss[None, :, k], 0.2)
        e = e.masked_fill(~A, -math.inf)
        al = torch.softmax(e, 1)
        ref = al @ Wh.view(n, K, Fh)[:, k]
        np.testing.assert_allclose(out.view(n, K, Fh)[:, k].numpy(), ref.numpy(), rtol=1e-10, atol=1e-12)


def test_gat_learns_cpu():
    from cgnn_amd.gnn.gat import GATTrainer
    g = synthetic("ogbn-arxiv", seed=2, scale=0.01, feat_noise=2.0, label_noise=0.1)
    tr = GATTrainer(g, heads=2, head_dim=16, lr=0.01)
    first = float(tr.train_step())
    for _ in range(25):
        last = float(tr.train_step())
    res = tr.evaluate()
    assert last < first and res["val_acc"] > 0.3, (first, last, res)


@pytest.mark.parametrize("fanouts", [(5, 5), None])
def test_fused_sage_matches_autograd_sage_cpu(fanouts):
    """The fused SAGE schedule (ops' CPU reference branches) computes the same step as the
    autograd model: same init, dropout off, same sampled blocks; then it learns."""
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-arxiv", seed=2, scale=0.01, feat_noise=2.0, label_noise=0.1)
    kw = dict(hidden=64, fanouts=fanouts, batch_size=256, lr=0.01, dropout=0.0, prefetch=False)
    a = SAGETrainer(g, fused=False, **kw)
    b = SAGETrainer(g, fused=True, **kw)
    assert b.fused and not a.fused
    # identical initial parameters
    f = b._fused
    for k in range(2):
        ref = torch.cat([a.model.w_self[k].detach(), a.model.w_neigh[k].detach()], 0)
        assert torch.equal(f.W[k], ref)
    la, lb = a.train_epoch(), b.train_epoch()
    assert lb == pytest.approx(la, rel=0.03), (la, lb)
    for _ in range(8):
        lb_last = b.train_epoch()
    assert lb_last < lb
    ra, rb = a.evaluate(), b.evaluate()
    assert rb["val_acc"] > 0.3, rb
