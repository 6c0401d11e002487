"""Fused GAT epoch (gnn/gat_fused.py) on its CPU reference branches vs the autograd
GAT model: same initial parameters, dropout off, gradients of the mean train
cross-entropy.  The fused path stores the gathered / GEMM operands in bf16 (as the
HIP kernels do), so the comparison is to bf16 accuracy."""
import numpy as np
import pytest
import torch

from cgnn_amd.gnn.data import synthetic
from cgnn_amd.gnn.gat import GATTrainer, GraphCSR
from cgnn_amd.gnn.gat_fused import FusedGAT, row_ce, wcat, wcat_bwd


def _setup(heads=4, head_dim=8, dropout=0.0, **kw):
    g = synthetic("ogbn-products", seed=2, scale=0.001)
    tr = GATTrainer(g, heads=heads, head_dim=head_dim, dropout=dropout, lr=0.01, seed=0, fused=True, **kw)
    assert tr.fused is not None
    return g, tr


def test_fused_gat_gradients_match_autograd():
    g, tr = _setup()
    f = tr.fused
    f.forward(train=True)
    f.backward()
    model = f.to_module()
    out = model(tr.x, tr.g)
    m = g.mask == 1
    loss = torch.nn.functional.cross_entropy(out[m], g.y[m].long())
    loss.backward()
    ref = torch.cat([t.grad.reshape(-1) for mod in (model.l1, model.l2)
                     for t in (mod.W, mod.a_src, mod.a_dst, mod.bias)])
    got = f.grads
    # per tensor: relative to the tensor's largest gradient.  The attention vectors'
    # gradients are sums of both signs over all rows of bf16-stored score gradients
    # (and the scores come from the bf16 folded columns W a), hence the wider bound
    off = 0
    for mod in (model.l1, model.l2):
        for name, t in (("W", mod.W), ("a_src", mod.a_src), ("a_dst", mod.a_dst), ("b", mod.bias)):
            k = t.numel()
            a, b = got[off:off + k], ref[off:off + k]
            scale = b.abs().max().item()
            tol = 0.03 if name in ("W", "b") else 0.08
            if scale > 0:
                assert (a - b).abs().max().item() < tol * scale, (name, t.shape, (a - b).abs().max().item(), scale)
            off += k


def test_fused_gat_train_row_layer2_matches_all_rows():
    """Training epochs aggregating layer 2 only at the train rows: the same first-step
    gradients as aggregating every row (dropout on: the same masks), up to the bf16
    rounding of the stored operands, and the same losses over a few Adam steps."""
    runs = []
    for rows_only in (False, True):
        g, tr = _setup(dropout=0.3, train_rows_only=rows_only)
        f = tr.fused
        assert (f._tr is None) == (not rows_only)
        f.forward(train=True)
        f.backward()
        grads = f.grads.clone()
        g, tr = _setup(dropout=0.3, train_rows_only=rows_only)
        runs.append((grads, [float(tr.train_step()) for _ in range(3)]))
    scale = runs[0][0].abs().max().item()
    assert (runs[1][0] - runs[0][0]).abs().max().item() < 2e-4 * scale
    np.testing.assert_allclose(runs[1][1], runs[0][1], rtol=1e-4)


def test_fused_gat_learns_and_evaluates():
    g, tr = _setup(dropout=0.3)
    first = float(tr.train_step())
    for _ in range(30):
        last = float(tr.train_step())
    assert last < first
    res = tr.evaluate()
    assert res["train_acc"] > 0.3 and 0 <= res["val_acc"] <= 1


def test_row_ce_matches_torch():
    torch.manual_seed(0)
    n, C, ld = 50, 13, 16
    Z = torch.randn(n, ld)
    b = torch.randn(C)
    y = torch.randint(0, C, (n,), dtype=torch.int32)
    mask = torch.randint(0, 4, (n,), dtype=torch.uint8)
    dZ = torch.zeros(n, ld)
    db = torch.zeros(C)
    tr = mask == 1
    st = row_ce(Z, b, C, y, mask, 1.0 / int(tr.sum()), dZ=dZ, db=db)
    logits = (Z[:, :C] + b).requires_grad_()
    loss = torch.nn.functional.cross_entropy(logits[tr], y[tr].long(), reduction="mean")
    loss.backward()
    np.testing.assert_allclose(float(st[0]) / int(tr.sum()), float(loss), rtol=1e-5)
    np.testing.assert_allclose(dZ[:, :C].numpy(), logits.grad.numpy(), atol=1e-6)
    assert float(dZ[:, C:].abs().sum()) == 0
    np.testing.assert_allclose(db.numpy(), logits.grad.sum(0).numpy(), atol=1e-6)


def test_wcat_backward_is_the_adjoint():
    torch.manual_seed(1)
    K, Fh, kin = 3, 8, 5
    W = torch.randn(kin, K * Fh, dtype=torch.float64, requires_grad=True)
    a_s = torch.randn(K, Fh, dtype=torch.float64, requires_grad=True)
    a_d = torch.randn(K, Fh, dtype=torch.float64, requires_grad=True)
    out = torch.zeros(kin, K * Fh + 2 * K, dtype=torch.float64)
    Wk = W.view(kin, K, Fh)
    ref = torch.cat([W, (Wk * a_s).sum(-1), (Wk * a_d).sum(-1)], 1)
    with torch.no_grad():
        wcat(W, a_s, a_d, out)
    np.testing.assert_allclose(out.numpy(), ref.detach().numpy())
    G = torch.randn_like(ref)
    ref.backward(G)
    gW, gs, gd = torch.zeros_like(W), torch.zeros_like(a_s), torch.zeros_like(a_d)
    with torch.no_grad():
        wcat_bwd(G, W, a_s, a_d, gW, gs, gd)
    np.testing.assert_allclose(gW.numpy(), W.grad.numpy(), rtol=1e-12)
    np.testing.assert_allclose(gs.numpy(), a_s.grad.numpy(), rtol=1e-12)
    np.testing.assert_allclose(gd.numpy(), a_d.grad.numpy(), rtol=1e-12)


def test_fused_gat_and_sage_checkpoint_resume(tmp_path):
    """safetensors checkpoints of the fused trainers: resuming equals training on.
    One intra-op thread: the CPU reference ops sum with index_add_, whose multi-thread
    order varies (~1e-8), and Adam's normalised step can amplify that to ~1e-5."""
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        _checkpoint_resume(tmp_path)
    finally:
        torch.set_num_threads(nt)


def _checkpoint_resume(tmp_path):
    from cgnn_amd.gnn.checkpoint import load_trainer, save_trainer
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-products", seed=6, scale=0.0005)
    for make, step in ((lambda: GATTrainer(g, heads=4, head_dim=8, dropout=0.3, lr=0.01, fused=True),
                        lambda t: t.train_step()),
                       (lambda: SAGETrainer(g, hidden=32, layers=2, fanouts=[5, 5], batch_size=64, fused=True),
                        lambda t: t.train_epoch())):
        a = make()
        step(a)
        path = str(tmp_path / "ck.safetensors")
        save_trainer(a, path)
        step(a)
        b = make()
        load_trainer(b, path)
        step(b)
        pa = a.state_tensors()["params"]
        pb = b.state_tensors()["params"]
        assert torch.allclose(pa, pb, rtol=0, atol=1e-6), (make, (pa - pb).abs().max())
