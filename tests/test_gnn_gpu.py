"""GNN-track HIP kernels vs the PyTorch reference path (same op, CPU tensors)."""
import numpy as np
import pytest
import torch

from cgnn_amd.gnn import ops
from cgnn_amd.gnn.data import build_csr, synthetic
from cgnn_amd.gnn.gcn import GCNTrainer

pytestmark = pytest.mark.gpu


def _graph(n=500, m=3000, seed=0):
    rng = np.random.default_rng(seed)
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
    rp, col = build_csr(n, src, dst, "cpu")
    return n, rp, col


@pytest.mark.parametrize("F,ld", [(47, 48), (100, 104), (256, 256), (8, 8)])
@pytest.mark.parametrize("xbf,ybf", [(True, True), (False, False), (True, False)])
def test_spmm_matches_reference(F, ld, xbf, ybf):
    n, rp, col = _graph()
    torch.manual_seed(0)
    X = torch.randn(n, ld)
    X[:, F:] = 0
    X = X.to(torch.bfloat16 if xbf else torch.float32)
    rs = torch.rand(n) + 0.5
    bias = torch.randn(F)
    odt = torch.bfloat16 if ybf else torch.float32
    ref = ops.spmm(rp, col, X, F, rscale=rs, bias=bias, relu=True, out_dtype=odt)
    got = ops.spmm(rp.cuda(), col.cuda(), X.cuda(), F, rscale=rs.cuda(), bias=bias.cuda(), relu=True,
                   out_dtype=odt).cpu()
    tol = 2e-2 if ybf else 1e-4
    np.testing.assert_allclose(got.float().numpy(), ref.float().numpy(), rtol=tol, atol=tol)


def test_spmm_ce_matches_reference():
    n, rp, col = _graph(700, 5000, 1)
    C, ld = 47, 48
    torch.manual_seed(1)
    Z = torch.zeros(n, ld, dtype=torch.bfloat16)
    Z[:, :C] = torch.randn(n, C).to(torch.bfloat16)
    rs = torch.rand(n) + 0.5
    b = torch.randn(C)
    y = torch.randint(0, C, (n,), dtype=torch.int32)
    mask = torch.randint(1, 4, (n,), dtype=torch.uint8)
    inv = 1.0 / float((mask == 1).sum())
    s_ref, g_ref = ops.spmm_ce(rp, col, Z, C, rs, b, y, mask, inv, mode=0)
    s_got, g_got = ops.spmm_ce(rp.cuda(), col.cuda(), Z.cuda(), C, rs.cuda(), b.cuda(), y.cuda(), mask.cuda(),
                               inv, mode=0)
    np.testing.assert_allclose(s_got.cpu().numpy()[:4], s_ref.numpy()[:4], rtol=1e-3, atol=1e-2)
    np.testing.assert_allclose(s_got.cpu().numpy()[4:4 + C], s_ref.numpy()[4:4 + C], atol=1e-5)
    np.testing.assert_allclose(g_got.cpu().float().numpy(), g_ref.float().numpy(), atol=2e-5, rtol=2e-2)


def test_dropout_mask_matches_reference():
    torch.manual_seed(2)
    H = torch.randn(300, 256).to(torch.bfloat16)
    b = torch.randn(256)
    ref = ops.bias_relu_dropout_(H.clone(), b, 256, 0.5, (123, 456), 7)
    got = ops.bias_relu_dropout_(H.clone().cuda(), b.cuda(), 256, 0.5, (123, 456), 7).cpu()
    np.testing.assert_allclose(got.float().numpy(), ref.float().numpy(), rtol=1e-2, atol=1e-2)
    keep = (got.float() != 0).float().mean().item()
    assert 0.2 < keep < 0.4   # relu (~1/2) x keep (1/2)


def test_gcn_steps_match_cpu():
    g = synthetic("cora", seed=3, device="cpu")
    cpu = GCNTrainer(g, hidden=64, rank=0, world=1)
    gpu = GCNTrainer(g.to("cuda:0"), hidden=64, rank=0, world=1)
    for _ in range(3):
        cpu.train_step()
        gpu.train_step()
    a, b = cpu.evaluate(), gpu.evaluate()
    assert abs(a["train_loss"] - b["train_loss"]) < 0.05 * max(a["train_loss"], 1e-3) + 1e-3
    assert abs(a["val_acc"] - b["val_acc"]) < 0.05


def test_gcn_learns_products_shape_small():
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=0.01, feat_noise=4.0)
    tr = GCNTrainer(g, hidden=128)
    for _ in range(40):
        tr.train_step()
    res = tr.evaluate()
    assert res["val_acc"] > 0.3, res
