"""Fused dense-layer kernels (gnn_linear.hip) against their fp32 PyTorch reference
(the CPU branch of gnn/linear.py: the same arithmetic on bf16-rounded operands)."""
import pytest
import torch

from cgnn_amd.gnn.linear import lin_bwd_data, lin_bwd_weight, lin_fwd

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bf(n, ld, K, gen, scale=1.0):
    x = torch.zeros(n, ld, dtype=torch.bfloat16)
    x[:, :K] = (torch.randn(n, K, generator=gen) * scale).to(torch.bfloat16)
    return x


def _close(a, b, rtol, atol):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), rtol=rtol, atol=atol)


@pytest.mark.parametrize("n,K,ld,N,ldy,relu,p,rs", [
    (5000, 100, 128, 256, 256, True, 0.5, True),     # layer 1 of GCN / SAGE on ogbn-products features
    (4133, 256, 256, 40, 40, False, 0.0, False),     # last layer to 40 classes (arxiv)
    (777, 47, 48, 256, 264, True, 0.0, True),        # odd K, padded output pitch
    (3, 128, 128, 96, 96, True, 0.3, False),         # fewer rows than one tile
    (6000, 256, 256, 256, 256, True, 0.5, True),     # arxiv hidden layer: weight-stationary form, bit-mode dropout
    (2000, 64, 64, 128, 128, True, 0.5, False),      # weight-stationary, 4 waves, a tile chunk per lane
    (1000, 128, 128, 40, 40, False, 0.0, True),      # narrow output on 8 waves (zero-weight columns unstored)
])
def test_lin_fwd_matches_reference(n, K, ld, N, ldy, relu, p, rs):
    g = torch.Generator().manual_seed(n)
    x = _bf(n, ld, K, g)
    W = torch.randn(K, N, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    r = torch.rand(n, generator=g) + 0.5 if rs else None
    key = (123, 456)
    ref = lin_fwd(x, W, b, K1=K, relu=relu, p=p, key=key, step=7, row0=11, rscale=r, ldy=ldy)
    out = lin_fwd(x.to(DEV), W.to(DEV), b.to(DEV), K1=K, relu=relu, p=p, key=key,
                  step=torch.tensor([7], dtype=torch.int32, device=DEV), row0=11,
                  rscale=r.to(DEV) if rs else None, ldy=ldy)
    torch.cuda.synchronize()
    _close(out, ref, 2e-2, 2e-2)
    if p > 0:   # identical dropout masks
        assert torch.equal(out.cpu()[:, :N] == 0, ref[:, :N] == 0) or \
            (out.cpu()[:, :N] == 0).ne(ref[:, :N] == 0).float().mean() < 1e-3
    assert torch.all(out.cpu()[:, N:] == 0)


@pytest.mark.parametrize("n,K,ld,N,ldy,dt", [
    (3001, 602, 608, 256, 256, torch.float16),    # Reddit's first layer (fp16 inference)
    (3001, 602, 608, 256, 256, torch.bfloat16),
    (1000, 700, 704, 100, 104, torch.bfloat16),   # one 128-column feature group, odd K
    (70, 1000, 1000, 200, 200, torch.float16),    # fewer rows than one block
])
def test_lin_fwd_k_chunked_matches_reference(n, K, ld, N, ldy, dt):
    """Weights too wide for LDS whole take the K-chunked GEMM (lin_fwd_kc_kernel): bias,
    ReLU and row scale against the fp32 reference; padding columns of X hold NaN, which
    must not leak into the product."""
    from cgnn_amd import native
    assert native.hip().gnn_lin_fwd_kc_wanted(K, N, ldy)
    g = torch.Generator().manual_seed(K + N)
    x = torch.full((n, ld), float("nan"), dtype=dt)
    x[:, :K] = torch.randn(n, K, generator=g).to(dt)
    W = torch.randn(K, N, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    r = torch.rand(n, generator=g) + 0.5
    ref = (x[:, :K].float() @ W.to(dt).float() + b).relu() * r[:, None]
    out = lin_fwd(x.to(DEV), W.to(DEV), b.to(DEV), K1=K, relu=True, rscale=r.to(DEV), ldy=ldy)
    torch.cuda.synchronize()
    assert out.dtype == dt
    _close(out[:, :N], ref, 2e-2, 2e-2)
    assert torch.all(out.cpu()[:, N:] == 0)


def test_lin_fwd_gathered_concatenation_matches_reference():
    """[x1[idx] | x2] on the weight-stationary form (SAGE-style layer, K = 64 + 64)."""
    g = torch.Generator().manual_seed(5)
    n, table, K, N = 3001, 9000, 64, 256
    x1, x2 = _bf(table, K, K, g), _bf(n, K, K, g)
    idx = torch.randint(0, table, (n,), generator=g, dtype=torch.int32)
    W = torch.randn(2 * K, N, generator=g) / 11
    b = torch.randn(N, generator=g) * 0.1
    step = torch.tensor([3], dtype=torch.int32)
    ref = lin_fwd(x1, W, b, x2=x2, K1=K, K2=K, relu=True, p=0.5, key=(5, 6), step=3, idx1=idx, n=n)
    out = lin_fwd(x1.to(DEV), W.to(DEV), b.to(DEV), x2=x2.to(DEV), K1=K, K2=K, relu=True, p=0.5, key=(5, 6),
                  step=step.to(DEV), idx1=idx.to(DEV), n=n)
    torch.cuda.synchronize()
    _close(out, ref, 2e-2, 2e-2)
    assert (out.cpu() == 0).ne(ref == 0).float().mean() < 1e-3


def test_lin_fwd_two_inputs_is_the_concatenation():
    g = torch.Generator().manual_seed(1)
    n, K1, K2, N = 3000, 256, 256, 256
    x1, x2 = _bf(n, K1, K1, g), _bf(n, K2, K2, g)
    W = torch.randn(K1 + K2, N, generator=g) / 20
    b = torch.randn(N, generator=g)
    out = lin_fwd(x1.to(DEV), W.to(DEV), b.to(DEV), x2=x2.to(DEV), relu=True)
    cat = lin_fwd(torch.cat([x1, x2], 1).to(DEV), W.to(DEV), b.to(DEV), relu=True)
    ref = lin_fwd(x1, W, b, x2=x2, relu=True)
    _close(out, ref, 2e-2, 3e-2)
    assert torch.equal(out, cat)


@pytest.mark.parametrize("n,N,K1,K2,mask,ms,rs", [
    (5000, 256, 100, 0, True, 2.0, True),
    (3000, 128, 64, 64, True, 2.0, False),            # weight-stationary form with both outputs
    (777, 40, 256, 0, False, 1.0, True),              # the arxiv last layer's backward (N = 40)
    (3001, 256, 256, 256, True, 1.0, False),
    (700, 47, 256, 0, False, 1.0, True),
])
def test_lin_bwd_data_matches_reference(n, N, K1, K2, mask, ms, rs):
    g = torch.Generator().manual_seed(n + N)
    ldd = (N + 7) // 8 * 8
    dY = _bf(n, ldd, N, g)
    Ym = torch.relu(_bf(n, ldd, N, g).float()).to(torch.bfloat16) if mask else None
    W = torch.randn(K1 + K2, N, generator=g) / N ** 0.5
    r = torch.rand(n, generator=g) + 0.5 if rs else None
    ref1, ref2 = lin_bwd_data(dY, W, K1, K2, Ym=Ym, mscale=ms, rscale=r)
    o1, o2 = lin_bwd_data(dY.to(DEV), W.to(DEV), K1, K2, Ym=Ym.to(DEV) if mask else None, mscale=ms,
                          rscale=r.to(DEV) if rs else None)
    torch.cuda.synchronize()
    _close(o1[:, :K1], ref1[:, :K1], 2e-2, 2e-2)
    if K2:
        _close(o2[:, :K2], ref2[:, :K2], 2e-2, 2e-2)


@pytest.mark.parametrize("n,K1,K2,N,mask", [
    (10007, 128, 0, 256, True),       # arxiv hidden layer
    (5000, 100, 0, 47, False),        # odd widths
    (4100, 256, 256, 256, True),      # SAGE [h_dst | agg]
    (17, 64, 0, 64, True),            # a single partial tile
    (3001, 104, 104, 256, True),      # SAGE layer 1 [h_dst | agg], K = 208 (7 k-tiles, one slab)
    (2000, 544, 0, 47, False),        # 17 k-tiles, 2 column tiles
    (999, 64, 0, 256, True),          # 2 k-tiles: 4 column groups of waves
    (1500, 96, 0, 128, False),        # 3 k-tiles in a 4-k-tile block
    (700, 320, 0, 200, True),         # 10 k-tiles, two 128-column slabs, ragged last slab
])
def test_lin_bwd_weight_matches_reference(n, K1, K2, N, mask):
    g = torch.Generator().manual_seed(n)
    ld1 = (K1 + 7) // 8 * 8
    ldd = (N + 7) // 8 * 8
    x1 = _bf(n, ld1, K1, g)
    x2 = _bf(n, K2, K2, g) if K2 else None
    dY = _bf(n, ldd, N, g, 0.01)
    Ym = torch.relu(_bf(n, ldd, N, g).float()).to(torch.bfloat16) if mask else None
    dW_ref, db_ref = lin_bwd_weight(x1, dY, N, x2=x2, K1=K1, Ym=Ym, mscale=2.0 if mask else 1.0)
    args = dict(x2=x2.to(DEV) if K2 else None, K1=K1, Ym=Ym.to(DEV) if mask else None, mscale=2.0 if mask else 1.0)
    dW, db = lin_bwd_weight(x1.to(DEV), dY.to(DEV), N, **args)
    dW2, db2 = lin_bwd_weight(x1.to(DEV), dY.to(DEV), N, **args)
    torch.cuda.synchronize()
    scale = dW_ref.abs().max().item()
    _close(dW, dW_ref, 1e-3, 1e-4 * scale)
    _close(db, db_ref, 1e-3, 1e-4 * db_ref.abs().max().item())
    assert torch.equal(dW, dW2) and torch.equal(db, db2)          # deterministic (no atomics)


def test_lin_layer_gradients_match_autograd():
    """fwd + both backward kernels = autograd of relu(x W + b) (dropout off), fp32 reference."""
    g = torch.Generator().manual_seed(3)
    n, K, N = 2048, 128, 256
    x = _bf(n, K, K, g)
    W = torch.randn(K, N, generator=g) / 12
    b = torch.randn(N, generator=g) * 0.1
    dY = _bf(n, N, N, g, 0.1)
    y = lin_fwd(x.to(DEV), W.to(DEV), b.to(DEV), relu=True)
    dX, _ = lin_bwd_data(dY.to(DEV), W.to(DEV), K, Ym=y)
    dW, db = lin_bwd_weight(x.to(DEV), dY.to(DEV), N, Ym=y)
    xr = x.float().requires_grad_()
    Wr = W.to(torch.bfloat16).float().requires_grad_()
    br = b.clone().requires_grad_()
    yr = torch.relu(xr @ Wr + br)
    yr.backward(dY.float())
    _close(dX, xr.grad, 3e-2, 3e-2)
    _close(dW, Wr.grad, 2e-2, 2e-2 * Wr.grad.abs().max().item())
    _close(db, br.grad, 2e-2, 2e-2 * br.grad.abs().max().item())


@pytest.mark.parametrize("n,table,K,N", [
    (3001, 20000, 104, 256),          # SAGE layer 0: [x[idx] | agg], K = 208
    (700, 5000, 64, 47),              # narrow output
])
def test_lin_bwd_weight_gathered_rows_match_reference(n, table, K, N):
    """idx1 (row r of the first operand is x1[idx1[r]]): the row ids are staged in LDS by
    the weight-gradient kernel; against the CPU reference on the gathered rows."""
    g = torch.Generator().manual_seed(n + 7)
    x1 = _bf(table, K, K, g)
    x2 = _bf(n, K, K, g)
    idx = torch.randint(0, table, (n,), generator=g, dtype=torch.int32)
    ldd = (N + 7) // 8 * 8
    dY = _bf(n, ldd, N, g, 0.01)
    Ym = torch.relu(_bf(n, ldd, N, g).float()).to(torch.bfloat16)
    dW_ref, db_ref = lin_bwd_weight(x1[idx.long()].contiguous(), dY, N, x2=x2, K1=K, Ym=Ym, mscale=2.0)
    dW, db = lin_bwd_weight(x1.to(DEV), dY.to(DEV), N, x2=x2.to(DEV), K1=K, Ym=Ym.to(DEV), mscale=2.0,
                            idx1=idx.to(DEV), n=n)
    torch.cuda.synchronize()
    _close(dW, dW_ref, 1e-3, 1e-4 * dW_ref.abs().max().item())
    _close(db, db_ref, 1e-3, 1e-4 * db_ref.abs().max().item())
