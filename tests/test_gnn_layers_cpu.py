"""CPU tests of the depth-generic GCN layers, the L-layer trainer (Cora-shaped
CPU reference path of BASELINE.json), the inference engine and GNN checkpoints."""
import numpy as np
import pytest
import torch

from cgnn_amd.gnn.data import build_csr, synthetic
from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer, GCNInference
from cgnn_amd.gnn.layers import GCN, NormGraph, norm_aggregate


def _dense_norm_adj(rp, col, n):
    A = torch.zeros(n, n, dtype=torch.float64)
    rows = torch.repeat_interleave(torch.arange(n), (rp[1:] - rp[:-1]).long())
    A[rows, col.long()] = 1.0
    deg = A.sum(1)
    d = deg.rsqrt()
    return d[:, None] * A * d[None, :], d


def test_norm_aggregate_forward_backward_match_dense():
    n = 120
    rng = np.random.default_rng(0)
    rp, col = build_csr(n, rng.integers(0, n, 500), rng.integers(0, n, 500), "cpu")
    Ahat, d = _dense_norm_adj(rp, col, n)
    g = NormGraph(rp, col, d.float())
    x = torch.randn(n, 13, dtype=torch.float32, requires_grad=True)     # width not a multiple of 8
    y = norm_aggregate(x, g)
    ref = Ahat @ x.detach().double()
    np.testing.assert_allclose(y.detach().double().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    gy = torch.randn(n, 13)
    y.backward(gy)
    np.testing.assert_allclose(x.grad.double().numpy(), (Ahat.t() @ gy.double()).numpy(), rtol=1e-5, atol=1e-5)


def test_deep_gcn_cora_cpu_learns():
    g = synthetic("cora", seed=0, device="cpu")
    tr = DeepGCNTrainer(g, hidden=64, layers=3, dropout=0.5, lr=0.01)
    first = float(tr.train_step())
    for _ in range(30):
        last = float(tr.train_step())
    res = tr.evaluate()
    assert last < first
    assert res["val_acc"] > 2.0 / g.n_classes, res


def test_inference_matches_model_forward():
    g = synthetic("cora", seed=1, device="cpu")
    tr = DeepGCNTrainer(g, hidden=32, layers=2)
    for _ in range(3):
        tr.train_step()
    tr.model.eval()
    with torch.no_grad():
        ref = tr.model(tr.x, tr.ng)
    inf = GCNInference.from_model(g, tr.model)
    got = inf()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


def test_deep_gcn_checkpoint_roundtrip(tmp_path):
    from cgnn_amd.gnn.checkpoint import load_trainer, save_trainer
    g = synthetic("cora", seed=2, device="cpu")
    a = DeepGCNTrainer(g, hidden=32, layers=3, seed=5, dropout=0.0)
    for _ in range(3):
        a.train_step()
    path = str(tmp_path / "gcn.safetensors")
    save_trainer(a, path, config={"hidden": 32, "layers": 3})
    b = DeepGCNTrainer(g, hidden=32, layers=3, seed=9, dropout=0.0)
    meta = load_trainer(b, path)
    assert meta["epoch"] == "3" and meta["config"]["layers"] == 3
    for _ in range(2):
        la, lb = float(a.train_step()), float(b.train_step())
        assert la == pytest.approx(lb, rel=1e-6)
    for pa, pb in zip(a.model.parameters(), b.model.parameters()):
        np.testing.assert_allclose(pa.detach().numpy(), pb.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_fused_gcn_checkpoint_roundtrip(tmp_path):
    from cgnn_amd.gnn.checkpoint import load_trainer, save_trainer
    from cgnn_amd.gnn.gcn import GCNTrainer
    g = synthetic("ogbn-products", seed=0, scale=0.001)
    a = GCNTrainer(g, hidden=32, rank=0, world=1)
    for _ in range(2):
        a.train_step()
    path = str(tmp_path / "gcn2.safetensors")
    save_trainer(a, path)
    b = GCNTrainer(g, hidden=32, rank=0, world=1, seed=3)
    load_trainer(b, path)
    a.train_step()
    b.train_step()
    np.testing.assert_array_equal(a.params.numpy(), b.params.numpy())


def test_linear_reference_ops_match_autograd():
    """CPU branch of gnn/linear.py (the GPU kernels' numerics oracle) = autograd of
    relu([x1 | x2] W + b) on bf16-rounded operands."""
    from cgnn_amd.gnn.linear import lin_bwd_data, lin_bwd_weight, lin_fwd
    g = torch.Generator().manual_seed(0)
    n, K1, K2, N = 64, 16, 8, 24
    x1 = torch.randn(n, K1, generator=g).to(torch.bfloat16)
    x2 = torch.randn(n, K2, generator=g).to(torch.bfloat16)
    W = torch.randn(K1 + K2, N, generator=g)
    b = torch.randn(N, generator=g)
    dY = torch.randn(n, N, generator=g).to(torch.bfloat16)
    y = lin_fwd(x1, W, b, x2=x2, relu=True)
    d1, d2 = lin_bwd_data(dY, W, K1, K2, Ym=y)
    dW, db = lin_bwd_weight(x1, dY, N, x2=x2, Ym=y)
    xr = torch.cat([x1, x2], 1).float().requires_grad_()
    Wr = W.to(torch.bfloat16).float().requires_grad_()
    br = b.clone().requires_grad_()
    yr = torch.relu(xr @ Wr + br)
    yr.backward(dY.float())
    assert torch.allclose(y[:, :N].float(), yr.detach(), rtol=1e-2, atol=1e-2)
    assert torch.allclose(torch.cat([d1[:, :K1], d2[:, :K2]], 1).float(), xr.grad, rtol=1e-2, atol=2e-2)
    assert torch.allclose(dW, Wr.grad, rtol=1e-4, atol=1e-3)
    assert torch.allclose(db, br.grad, rtol=1e-4, atol=1e-4)
    # dropout: the mask of ops.dropout_keep_mask, scaled by 1/(1-p)
    yd = lin_fwd(x1, W, b, x2=x2, relu=True, p=0.5, key=(1, 2), step=3)
    from cgnn_amd.gnn.ops import dropout_keep_mask
    keep = dropout_keep_mask(n, N, 0.5, (1, 2), 3)
    assert torch.equal(yd[:, :N].float() == 0, (~keep) | (y[:, :N].float() == 0))


@pytest.mark.parametrize("layers", [2, 3])
def test_fused_deep_gcn_matches_autograd_gcn(layers):
    """The hand-scheduled fused epoch (manual backward through SpMM, lin_* and spmm_ce)
    trains like the autograd GCN: same init, dropout off, bf16 storage vs fp32."""
    from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer
    g = synthetic("ogbn-arxiv", seed=4, scale=0.004)
    a = DeepGCNTrainer(g, hidden=64, layers=layers, dropout=0.0, lr=0.01, dtype=torch.float32, fused=False)
    b = DeepGCNTrainer(g, hidden=64, layers=layers, dropout=0.0, lr=0.01, fused=True)
    assert b.fused and not a.fused
    ra0, rb0 = a.evaluate(), b.evaluate()
    assert abs(ra0["train_loss"] - rb0["train_loss"]) < 0.02 * ra0["train_loss"], (ra0, rb0)
    for _ in range(5):
        a.train_step()
        b.train_step()
    ra, rb = a.evaluate(), b.evaluate()
    assert rb["train_loss"] < rb0["train_loss"] - 0.05            # it learns
    assert abs(ra["train_loss"] - rb["train_loss"]) < 0.03 * ra["train_loss"], (ra, rb)
    # gradients of the first step agree layer by layer
    a2 = DeepGCNTrainer(g, hidden=64, layers=layers, dropout=0.0, lr=0.01, dtype=torch.float32, fused=False)
    b2 = DeepGCNTrainer(g, hidden=64, layers=layers, dropout=0.0, lr=0.01, fused=True)
    a2.model.train()
    from cgnn_amd.gnn.gcn_deep import cross_entropy
    out = a2.model(a2.x, a2.ng)
    cross_entropy(out[a2.idx["train"]], a2.y_train).backward()
    f = b2._fused
    f.backward(f.forward(train=True))
    def rel(a, b):
        return float((a - b).norm() / b.norm())
    for l, conv in enumerate(a2.model.convs):
        gw_ref = conv.weight.grad[:f.dims[l]]
        assert rel(f.gW[l], gw_ref) < 0.02, (l, rel(f.gW[l], gw_ref))     # bf16 activations vs fp32
        assert rel(f.gb[l], conv.bias.grad) < 0.02, (l, rel(f.gb[l], conv.bias.grad))


def test_fused_deep_gcn_dropout_trains_on_cpu():
    from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer
    g = synthetic("ogbn-arxiv", seed=5, scale=0.004)
    t = DeepGCNTrainer(g, hidden=64, layers=3, dropout=0.5, lr=0.01, fused=True)
    r0 = t.evaluate()
    for _ in range(8):
        t.train_step()
    assert t.evaluate()["train_loss"] < r0["train_loss"]


def test_fused_bwd_grad_index_scatters_the_slab_layout():
    """The index map that scatters a fused-backward slab sum [HD][width] into the flat
    gradient buffer reproduces (gW1 = g[:, :F]^T, gb1 = g[:, F], gW2 = g[:, kf:kf+C])."""
    from cgnn_amd.gnn import ops
    F, HD, C, width = 100, 64, 47, 192
    kf = width - 64
    g = torch.randn(3, HD, width)
    flat = torch.zeros(F * HD + HD + HD * C + C)
    idx = ops.fused_bwd_grad_index(F, HD, C, width)
    ops.slab_sum(g.view(3, -1), flat, idx)
    s = g.sum(0)
    assert torch.allclose(flat[:F * HD].view(F, HD), s[:, :F].t())
    assert torch.allclose(flat[F * HD:F * HD + HD], s[:, F])
    assert torch.allclose(flat[F * HD + HD:F * HD + HD + HD * C].view(HD, C), s[:, kf:kf + C])
    assert torch.all(flat[F * HD + HD + HD * C:] == 0)


def test_fused_deep_gcn_train_row_last_layer_matches_all_rows():
    """The fused L-layer GCN aggregating its last layer only at the train rows in
    training: same losses and parameters as aggregating every row (CPU branches)."""
    g = synthetic("cora", seed=3, device="cpu")
    runs = []
    for rows_only in (False, True):
        tr = DeepGCNTrainer(g, hidden=32, layers=3, dropout=0.5, fused=True, train_rows_only=rows_only)
        assert (tr._fused._tr is None) == (not rows_only)
        losses = [float(tr.train_step()) for _ in range(4)]
        runs.append((losses, tr._fused.params.clone(), tr.evaluate()))
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=1e-4)
    torch.testing.assert_close(runs[1][1], runs[0][1], rtol=1e-3, atol=1e-4)
    assert runs[1][2]["val_acc"] == pytest.approx(runs[0][2]["val_acc"], abs=0.01)


def test_dropout_keep_mask_bit_and_byte_modes():
    """ops.dropout_keep_mask: p = 1/2 uses one random bit per decision (bit 16 (t % 8) + q
    of the draw keyed (row, DROP_BIT_CTR + 2 (t // 8) + h)), other p a byte per decision;
    both keep ~1 - p, depend only on the global row, and differ between the two modes."""
    import numpy as np
    from cgnn_amd.gnn.ops import dropout_keep_mask, DROP_BIT_CTR
    from cgnn_amd.utils import philox
    for p in (0.5, 0.25):
        m = dropout_keep_mask(400, 512, p, (9, 11), 5)
        assert abs(m.float().mean().item() - (1 - p)) < 0.02
        part = dropout_keep_mask(100, 512, p, (9, 11), 5, row0=300)
        assert torch.equal(part, m[300:])
    # one unit by hand in bit mode: row 17, unit n = 32 t + 8 g + 4 h + i
    n = 32 * 9 + 8 * 2 + 4 * 1 + 3
    t, g, h, i = 9, 2, 1, 3
    w = philox.philox4x32_10(np.uint32(17), np.uint32(DROP_BIT_CTR + 2 * (t // 8) + h), 5, philox.RNG_DROPOUT, 9, 11)
    b = 16 * (t % 8) + 4 * g + i
    bit = (int(np.asarray(w[b // 32])) >> (b % 32)) & 1
    assert bool(dropout_keep_mask(18, 512, 0.5, (9, 11), 5)[17, n]) == bool(bit)


def test_spmm_ell_reference_matches_spmm():
    from cgnn_amd.gnn import ops
    torch.manual_seed(4)
    n, C, ld = 300, 47, 48
    deg = torch.randint(0, 9, (n,))
    deg[:5] = torch.tensor([12, 30, 9, 64, 100])
    rp = torch.zeros(n + 1, dtype=torch.int32)
    rp[1:] = torch.cumsum(deg, 0).to(torch.int32)
    col = torch.randint(0, n, (int(rp[-1]),), dtype=torch.int32)
    X = torch.zeros(n, ld, dtype=torch.bfloat16)
    X[:, :C] = torch.randn(n, C).to(torch.bfloat16)
    rs = torch.rand(n) + 0.5
    ell = ops.ell_image(rp, col)
    assert int((ell.ell[:, 0] == -2).sum()) == 5 and ell.long_rows.tolist() == [0, 1, 2, 3, 4]
    got = ops.spmm_ell(ell, col, X, C, rscale=rs)
    ref = ops.spmm(rp, col, X, C, rscale=rs, out=torch.empty(n, ld, dtype=torch.bfloat16))
    assert torch.allclose(got.float(), ref.float(), rtol=1e-2, atol=1e-2)
