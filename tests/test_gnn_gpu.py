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


@pytest.mark.parametrize("n_rows", [1, 5, 1000, 70001])
@pytest.mark.parametrize("F,ld", [(100, 104), (64, 64), (8, 8), (128, 128)])
def test_spmm_fan_matches_spmm(n_rows, F, ld):
    """The pipelined kernel for rows of <= 8 entries (a sampled block's input layer)
    equals the CSR SpMM bit for bit: rows of 0-8 entries (8: the 8-step; 4-7: a 4-step
    and 1-steps; < 4: 1-steps), with and without the row scale; rows past n untouched."""
    rng = np.random.default_rng(n_rows + F)
    n_src = 3000
    deg = rng.integers(0, 9, n_rows)
    deg[::11] = 8
    deg[::13] = 0
    rp = torch.zeros(n_rows + 1, dtype=torch.int32)
    rp[1:] = torch.as_tensor(np.cumsum(deg), dtype=torch.int32)
    col = torch.as_tensor(rng.integers(0, n_src, int(deg.sum())), dtype=torch.int32)
    X = torch.zeros(n_src, ld)
    X[:, :F] = torch.randn(n_src, F)
    X = X.to(torch.bfloat16).cuda()
    rs = (torch.rand(n_rows) + 0.5).cuda()
    rpc, colc = rp.cuda(), col.cuda()
    for rscale in (rs, None):
        ref = ops.spmm(rpc, colc, X, F, rscale=rscale,
                       out=torch.full((n_rows + 3, ld), 7.0, dtype=torch.bfloat16).cuda()[:n_rows])
        got_full = torch.full((n_rows + 3, ld), 7.0, dtype=torch.bfloat16).cuda()
        got = ops.spmm_fan(rpc, colc, X, F, 8, rscale=rscale, out=got_full[:n_rows])
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
        assert torch.all(got_full[n_rows:] == 7.0)
    # a bound above 8 falls back to the CSR SpMM (same result)
    got = ops.spmm_fan(rpc, colc, X, F, 9, rscale=rs)
    assert torch.equal(got.view(torch.int16), ops.spmm(rpc, colc, X, F, rscale=rs).view(torch.int16))


def _short_csr(n_rows, n_src, seed):
    """CSR with mostly 0-3 entries per row and a few long rows (4..40), at random places."""
    rng = np.random.default_rng(seed)
    deg = rng.choice([0, 1, 1, 1, 2, 3], n_rows)
    longr = rng.random(n_rows) < 0.05
    deg[longr] = rng.integers(4, 41, int(longr.sum()))
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    col = rng.integers(0, n_src, int(rp[-1])).astype(np.int32)
    return torch.from_numpy(rp), torch.from_numpy(col)


@pytest.mark.parametrize("F,ld", [(256, 256), (100, 104), (40, 40), (600, 608)])
@pytest.mark.parametrize("xdt,ydt,cs,init", [(torch.bfloat16, torch.bfloat16, True, True),
                                             (torch.bfloat16, torch.bfloat16, False, False),
                                             (torch.float32, torch.float32, True, False),
                                             (torch.bfloat16, torch.float32, False, True),
                                             (torch.float16, torch.float16, True, True)])
def test_spmm_short_rows_bitwise_equals_row_kernel(F, ld, xdt, ydt, cs, init):
    """The 4-rows-per-sub-group kernel (transposed sampled blocks) against the one-row
    kernel: bit-identical, every row-length class (0-3 entries, long rows, rows past a
    sub-group's first L edges, a partial last group); and against the fp32 reference."""
    n_rows, n_src = 5003, 3001
    rp, col = _short_csr(n_rows, n_src, 7)
    torch.manual_seed(1)
    X = torch.randn(n_src, ld)
    X[:, F:] = 0
    X = X.to(xdt).cuda()
    csc = (torch.rand(n_src) + 0.5).cuda() if cs else None
    rs = (torch.rand(n_rows) + 0.5).cuda()
    ini = torch.randn(1200, ld).cuda() if init else None
    kw = dict(rscale=rs, cscale=csc, init=ini, init_rows=1200 if init else None, out_dtype=ydt)
    rpc, colc = rp.cuda(), col.cuda()
    a = ops.spmm(rpc, colc, X, F, short_rows=True, **kw)
    b = ops.spmm(rpc, colc, X, F, short_rows=False, **kw)
    assert torch.equal(a, b)
    ref = ops.spmm(rp, col, X.cpu().float(), F, rscale=rs.cpu(), cscale=None if csc is None else csc.cpu(),
                   init=None if ini is None else ini.cpu(), init_rows=1200 if init else None, out_dtype=torch.float32)
    tol = 1e-4 if ydt == torch.float32 and xdt == torch.float32 else 3e-2
    np.testing.assert_allclose(a.float().cpu().numpy(), ref.numpy(), rtol=tol, atol=tol)


@pytest.mark.parametrize("F,ld", [(1433, 1440), (1024, 1032), (600, 608)])
def test_spmm_wide_rows_with_ones_column(F, ld):
    """Rows wider than one 512-column slab (Cora / Citeseer / Reddit widths): every
    slab writes only its own columns, the last ones the padding and the ones column."""
    n, rp, col = _graph(300, 2000, 2)
    torch.manual_seed(1)
    X = torch.randn(n, ld)
    X[:, F:] = 0
    X = X.to(torch.bfloat16)
    rs = torch.rand(n) + 0.5
    ref = ops.spmm(rp, col, X, F, rscale=rs, unit_col=F)
    got = ops.spmm(rp.cuda(), col.cuda(), X.cuda(), F, rscale=rs.cuda(), unit_col=F).cpu()
    np.testing.assert_allclose(got.float().numpy(), ref.float().numpy(), rtol=2e-2, atol=2e-2)
    assert torch.all(got[:, F] == 1) and torch.all(got[:, F + 1:] == 0)


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


def test_fused_dense_matches_reference():
    torch.manual_seed(5)
    n, F, HD, C = 777, 100, 256, 47
    AX = torch.zeros(n, 104, dtype=torch.bfloat16)
    AX[:, :F] = torch.randn(n, F).to(torch.bfloat16)
    AX[:, F] = 1
    W1, b1 = torch.randn(F, HD) * 0.1, torch.randn(HD) * 0.1
    W2 = torch.randn(HD, C) * 0.1
    dinv = torch.rand(n) + 0.5
    dY2 = torch.zeros(n, 48, dtype=torch.bfloat16)
    dY2[:, :C] = (torch.randn(n, C) * 0.01).to(torch.bfloat16)
    outs, h1_gpu = [], None
    for dev in ("cuda:0", "cpu"):
        H1 = torch.zeros(n, HD, dtype=torch.bfloat16, device=dev)
        Z2 = torch.zeros(n, 48, dtype=torch.bfloat16, device=dev)
        assert ops.dense_fwd(AX.to(dev), W1.to(dev), b1.to(dev), W2.to(dev), dinv.to(dev), H1, Z2, F, 0.5,
                             (9, 10), 3)
        # the backward of both paths uses the SAME H1 (the GPU one): its mask defines dP1
        h1_gpu = H1.cpu() if h1_gpu is None else h1_gpu
        dP1 = torch.zeros(n, HD, dtype=torch.bfloat16, device=dev)
        assert ops.dense_bwd(dY2.to(dev), W2.to(dev), h1_gpu.to(dev), dP1, 0.5)
        outs.append((H1.cpu().float(), Z2.cpu().float(), dP1.cpu().float()))
    (h, z, d), (h_ref, z_ref, d_ref) = outs
    # same dropout mask; bf16 rounding of the GEMM inputs/outputs only
    assert ((h_ref > 0) != (h > 0)).float().mean() < 0.01
    np.testing.assert_allclose(h.numpy(), h_ref.numpy(), atol=3e-2, rtol=3e-2)
    np.testing.assert_allclose(z.numpy(), z_ref.numpy(), atol=3e-2, rtol=5e-2)
    np.testing.assert_allclose(d.numpy(), d_ref.numpy(), atol=2e-3, rtol=5e-2)


@pytest.mark.parametrize("p", [0.5, 0.3])     # bit mode (p = 1/2) and byte mode
def test_dropout_mask_matches_reference(p):
    torch.manual_seed(2)
    H = torch.randn(300, 256).to(torch.bfloat16)
    b = torch.randn(256)
    ref = ops.bias_relu_dropout_(H.clone(), b, 256, p, (123, 456), 7)
    got = ops.bias_relu_dropout_(H.clone().cuda(), b.cuda(), 256, p, (123, 456), 7).cpu()
    np.testing.assert_allclose(got.float().numpy(), ref.float().numpy(), rtol=1e-2, atol=1e-2)
    keep = (got.float() != 0).float().mean().item()
    assert 0.5 * (1 - p) - 0.05 < keep < 0.5 * (1 - p) + 0.05   # relu (~1/2) x keep (1 - p)


def test_spmm_ce_long_rows_on_whole_waves_match_reference():
    """spmm_ce with n_long > 0 (the rows ordered long-first, each on a whole wave: its
    8 sub-groups walk every 8th chunk and combine) equals the CPU reference, whose
    result does not depend on n_long."""
    torch.manual_seed(3)
    n, C, ld = 900, 47, 48
    deg = torch.randint(0, 20, (n,))
    deg[torch.randperm(n)[:60]] = torch.randint(100, 700, (60,))     # power-law-ish tail
    order, n_long = ops.long_row_order(deg, threshold=64)
    assert n_long == 60
    deg = deg[order]
    rp = torch.zeros(n + 1, dtype=torch.int32)
    rp[1:] = torch.cumsum(deg, 0).to(torch.int32)
    col = torch.randint(0, n, (int(rp[-1]),), dtype=torch.int32)
    Z = torch.zeros(n, ld, dtype=torch.bfloat16)
    Z[:, :C] = torch.randn(n, C).to(torch.bfloat16)
    rs = torch.rand(n) + 0.5
    b = torch.randn(C)
    y = torch.randint(0, C, (n,), dtype=torch.int32)
    mask = torch.randint(1, 4, (n,), dtype=torch.uint8)
    init = torch.randn(n, ld) * 0.1
    inv = 1.0 / float((mask == 1).sum())
    s_ref, g_ref = ops.spmm_ce(rp, col, Z, C, rs, b, y, mask, inv, mode=0, init=init)
    s_got, g_got = ops.spmm_ce(rp.cuda(), col.cuda(), Z.cuda(), C, rs.cuda(), b.cuda(), y.cuda(), mask.cuda(),
                               inv, mode=0, init=init.cuda(), n_long=n_long)
    np.testing.assert_allclose(s_got.cpu().numpy()[:4], s_ref.numpy()[:4], rtol=1e-3, atol=1e-2)
    np.testing.assert_allclose(s_got.cpu().numpy()[4:4 + C], s_ref.numpy()[4:4 + C], atol=1e-5)
    np.testing.assert_allclose(g_got.cpu().float().numpy(), g_ref.float().numpy(), atol=2e-5, rtol=2e-2)
    # and equal to the same launch without the long-row mode
    s0, g0 = ops.spmm_ce(rp.cuda(), col.cuda(), Z.cuda(), C, rs.cuda(), b.cuda(), y.cuda(), mask.cuda(),
                         inv, mode=0, init=init.cuda(), n_long=0)
    np.testing.assert_allclose(g_got.cpu().float().numpy(), g0.cpu().float().numpy(), atol=1e-6, rtol=1e-2)


@pytest.mark.parametrize("name,fused", [("cora", True), ("ogbn-arxiv", True), ("ogbn-products", True),
                                        ("ogbn-products", False)])
def test_gcn_steps_match_cpu(name, fused):
    g = synthetic(name, seed=3, device="cpu", scale=1.0 if name == "cora" else 0.003)
    cpu = GCNTrainer(g, hidden=64, rank=0, world=1)
    gpu = GCNTrainer(g.to("cuda:0"), hidden=64, rank=0, world=1, fused=fused)
    for _ in range(3):
        cpu.train_step()
        gpu.train_step()
    a, b = cpu.evaluate(), gpu.evaluate()
    # the CPU path is the fp32 reference of the same bf16-stored arithmetic with the same
    # dropout masks: after 3 Adam steps only summation order separates the two
    dp = (gpu.params.cpu() - cpu.params).abs().max().item()
    print("gcn %s fused=%s: loss cpu %.6f gpu %.6f, val_acc %.4f / %.4f, max |dparam| %.2e"
          % (name, fused, a["train_loss"], b["train_loss"], a["val_acc"], b["val_acc"], dp))
    assert abs(a["train_loss"] - b["train_loss"]) < 5e-3 * max(a["train_loss"], 1e-3)
    assert abs(a["val_acc"] - b["val_acc"]) < 0.01
    # Adam moves each weight by <= lr = 0.01 per step; a wrong gradient sign or a
    # dropped term shows up as a difference of order lr
    assert dp < 2e-3, dp


@pytest.mark.parametrize("reorder", [False, True])
def test_gcn_benched_config_matches_cpu(reorder):
    """The composed path bench.py times -- hidden 256 (the fused MFMA dense forward and
    backward: gcn_dense_fwd / gcn_fused_bwd, slab_sum straight into the flat gradient),
    layer 2 aggregated at the train rows, layer 1 at the rows with a train neighbour,
    dropout 0.5 -- against the fp32 CPU reference of the same bf16-stored arithmetic
    over 4 epochs (the benched graph shape, scaled down; reorder pass on and off)."""
    g = synthetic("ogbn-products", seed=3, device="cpu", scale=0.004)
    cpu = GCNTrainer(g, hidden=256, rank=0, world=1, reorder=reorder)
    gpu = GCNTrainer(g.to("cuda:0"), hidden=256, rank=0, world=1, reorder=reorder)
    assert gpu.fused and gpu.fused_bwd
    assert gpu._l2 is not None and gpu._l1 is not None       # train-row layer 2, train-neighbour layer 1
    lc, lg = [], []
    for _ in range(4):
        cpu.train_step()
        gpu.train_step()
        lc.append(cpu.train_loss())
        lg.append(gpu.train_loss())
    np.testing.assert_allclose(lg, lc, rtol=3e-3)
    a, b = cpu.evaluate(), gpu.evaluate()
    dp = (gpu.params.cpu() - cpu.params).abs()
    print("gcn-256 reorder=%s: losses cpu %s gpu %s, val %.4f / %.4f, max |dparam| %.2e, >1e-4: %.4f"
          % (reorder, lc, lg, a["val_acc"], b["val_acc"], dp.max().item(), (dp > 1e-4).float().mean().item()))
    assert abs(a["train_loss"] - b["train_loss"]) < 5e-3 * max(a["train_loss"], 1e-3)
    assert abs(a["val_acc"] - b["val_acc"]) < 0.01
    # Adam moves a weight by <= lr per step; a wrong gradient term shows as O(lr) on many
    assert (dp > 2e-3).float().mean().item() < 1e-3, (dp > 2e-3).float().mean().item()
    assert dp.max().item() < 4 * 0.01


def test_gcn_learns_products_shape_small():
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=0.01, feat_noise=4.0)
    tr = GCNTrainer(g, hidden=128)
    for _ in range(40):
        tr.train_step()
    res = tr.evaluate()
    assert res["val_acc"] > 0.3, res


@pytest.mark.parametrize("HD,p,row0,ldx,ldc", [(256, 0.5, 0, 104, 48), (256, 0.0, 0, 104, 48),
                                              (128, 0.5, 4096, 104, 48), (256, 0.5, 0, 128, 64)])
def test_fused_backward_matches_reference(HD, p, row0, ldx, ldc):
    """Fused dense backward (H1 recomputed from AX, weight gradients contracted over the
    rows in the same pass) vs the unfused math on CPU with the same dropout mask; row
    pitches packed to 8 elements or padded to whole 128-B lines."""
    torch.manual_seed(3)
    n, F, C = 1000, 100, 47
    AX = torch.zeros(n, ldx)
    AX[:, :F] = torch.randn(n, F) * 0.5
    AX[:, F] = 1.0                                   # ones column -> gb1
    AX = AX.to(torch.bfloat16)
    dY2 = torch.zeros(n, ldc)
    dY2[:, :C] = torch.randn(n, C) * 0.1
    dY2 = dY2.to(torch.bfloat16)
    W1 = torch.randn(F, HD) * 0.1
    b1 = torch.randn(HD) * 0.1
    W2 = torch.randn(HD, C) * 0.1
    key, step = (123, 456), 7
    assert ops.fused_bwd_supported(F, HD, C)
    gW1, gb1, gW2, _ = ops.fused_bwd(AX.cuda(), dY2.cuda(), W1.cuda(), b1.cuda(), W2.cuda(), n, F, p, key, step,
                                     row0)
    # reference: same bf16 roundings as the kernel (operands, H1 and dP1 images)
    P1 = AX[:, :F].float() @ W1.to(torch.bfloat16).float() + b1
    H1 = torch.relu(P1)
    if p > 0:
        keep = ops.dropout_keep_mask(n, HD, p, key, step, row0)
        H1 = torch.where(keep, H1 / (1 - p), torch.zeros_like(H1))
    dH = dY2[:, :C].float() @ W2.to(torch.bfloat16).float().t()
    dP1 = torch.where(H1 > 0, dH / (1 - p), torch.zeros_like(dH))
    H1b, dP1b = H1.to(torch.bfloat16).double(), dP1.to(torch.bfloat16).double()
    rW1 = AX[:, :F].double().t() @ dP1b
    rb1 = dP1b.sum(0)
    rW2 = H1b.t() @ dY2[:, :C].double()
    for got, ref in ((gW1, rW1), (gb1, rb1), (gW2, rW2)):
        got = got.double().cpu()
        scale = ref.abs().max().item()
        np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=2e-2 * scale, rtol=0)
        assert (got - ref).abs().mean().item() < 2e-3 * scale


@pytest.mark.parametrize("p,HD,n", [(0.5, 256, 1000), (0.3, 256, 777), (0.5, 128, 70)])
def test_forward_keep_image_matches_drawn_and_reference(p, HD, n):
    """The keep image the fused forward writes for the backward (bit mode: from the
    forward's own draw; byte mode: the side launch) equals the standalone draw, and its
    bits are the reference dropout mask (ops.dropout_keep_mask) in the documented layout:
    halfword (T * HD/32 + t) * 64 + 32 uh + r, bit 4 g + i <-> row 32 T + r, unit
    32 t + 8 g + 4 uh + i."""
    torch.manual_seed(1)
    F, C = 100, 47
    dev = "cuda:0"
    AX = torch.zeros(n, 104, dtype=torch.bfloat16, device=dev)
    AX[:, :F] = torch.randn(n, F, device=dev).to(torch.bfloat16)
    AX[:, F] = 1
    W1, b1, W2 = torch.randn(F, HD, device=dev) * 0.1, torch.zeros(HD, device=dev), torch.randn(HD, C, device=dev)
    dinv = torch.ones(n, device=dev)
    Z2 = torch.zeros(n, 48, dtype=torch.bfloat16, device=dev)
    key, step, row0 = (31, 41), 5, 64
    kf = ops.keep_image(n, HD, dev).fill_(0x5555)
    assert ops.dense_fwd(AX, W1, b1, W2, dinv, None, Z2, F, p, key, step, row0, kimg=kf)
    kd = ops.draw_keep_image(ops.keep_image(n, HD, dev), n, HD, p, key, step, row0)
    assert torch.equal(kf, kd)
    # decode against the reference mask
    nt, NB = (n + 31) // 32, HD // 32
    words = kd.cpu().view(nt, NB, 2, 32).to(torch.int32) & 0xffff          # [T][t][uh][r]
    bits = (words[..., None] >> torch.arange(16)) & 1                        # [T][t][uh][r][q]
    q = torch.arange(16)
    g, i = q // 4, q % 4
    keep = torch.zeros(nt * 32, HD, dtype=torch.bool)
    for uh in range(2):
        for t in range(NB):
            units = 32 * t + 8 * g + 4 * uh + i
            keep[:, units] = bits[:, t, uh].reshape(nt * 32, 16).bool()
    ref = ops.dropout_keep_mask(n, HD, p, key, step, row0)
    assert torch.equal(keep[:n], ref)


def test_sage_aggregate_gpu_matches_cpu():
    from cgnn_amd.gnn.sage import Block, mean_aggregate
    g = synthetic("ogbn-arxiv", seed=1, scale=0.01)
    from cgnn_amd import native
    raw = native.rt().sample_neighbors(g.rowptr.numpy().astype(np.int64), g.col.numpy(),
                                       np.arange(0, 300, dtype=np.int64), [7, 5], 11)
    rp, col, nodes = raw[1]
    h = torch.randn(len(nodes), 64)
    gout = torch.randn(len(rp) - 1, 64)
    outs = []
    for dev in ("cpu", "cuda:0"):
        b = Block(rp, col, len(nodes), dev)
        hh = h.detach().clone().to(dev).requires_grad_(True)
        out = mean_aggregate(hh, b)
        out.backward(gout.to(dev))
        outs.append((out.detach().cpu(), hh.grad.cpu()))
    np.testing.assert_allclose(outs[1][0].numpy(), outs[0][0].numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(outs[1][1].numpy(), outs[0][1].numpy(), rtol=1e-5, atol=1e-5)


def test_sage_minibatch_learns_gpu():
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=0.005, feat_noise=4.0)
    tr = SAGETrainer(g, hidden=128, fanouts=(10, 5), batch_size=128, lr=0.003)
    first = tr.train_epoch()
    for _ in range(8):
        last = tr.train_epoch()
    res = tr.evaluate()
    assert last < first and res["val_acc"] > 0.3, (first, last, res)


@pytest.mark.parametrize("lowp", [False, True])
@pytest.mark.parametrize("K,Fh", [(4, 16), (1, 64), (8, 32), (3, 8), (1, 176), (1, 40)])
def test_gat_kernels_match_torch_autograd(K, Fh, lowp):
    """HIP GAT forward / backward vs PyTorch autograd in fp64.  lowp: the gathered
    rows (Wh, dout) are stored bf16 -- the reference then takes bf16-rounded Wh and
    dout; the row half also reads the forward's LeakyReLU split q stored bf16, one more
    rounding inside d s_dst = -0.8 <dout, q> (its tolerance is 4e-3)."""
    from cgnn_amd.gnn.gat import GraphCSR, gat_aggregate
    n = 700
    rng = np.random.default_rng(K * 100 + Fh)
    rp, col = build_csr(n, rng.integers(0, n, 4000), rng.integers(0, n, 4000), "cpu")
    torch.manual_seed(5)
    Wh = torch.randn(n, K * Fh, dtype=torch.float64)
    ss, sd = torch.randn(n, K, dtype=torch.float64), torch.randn(n, K, dtype=torch.float64)
    gout = torch.randn(n, K * Fh, dtype=torch.float64)
    if lowp:
        Wh, gout = Wh.to(torch.bfloat16).double(), gout.to(torch.bfloat16).double()
    res = []
    for dev in ("cpu", "cuda:0"):
        g = GraphCSR(rp.to(dev), col.to(dev), n)
        a, b, c = (t.detach().clone().to(dev).requires_grad_(True) for t in (Wh, ss, sd))
        if dev != "cpu":
            a, b, c = (t.float().detach().requires_grad_(True) for t in (a, b, c))
        out = gat_aggregate(a, b, c, g, K, Fh, lowp=lowp)
        out.backward(gout.to(dev, out.dtype))
        res.append([t.detach().double().cpu() for t in (out, a.grad, b.grad, c.grad)])
    for x, y, name in zip(res[1], res[0], ("out", "dWh", "ds_src", "ds_dst")):
        tol = (4e-3 if name == "ds_dst" else 2e-3) if lowp else 1e-4
        scale = y.abs().max().item()
        np.testing.assert_allclose(x.numpy(), y.numpy(), rtol=0, atol=tol * scale + 1e-6, err_msg=name)


def test_gat_trainer_learns_gpu():
    from cgnn_amd.gnn.gat import GATTrainer
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=0.005, feat_noise=4.0)
    tr = GATTrainer(g, heads=4, head_dim=32, lr=0.005)
    first = float(tr.train_step())
    for _ in range(40):
        last = float(tr.train_step())
    res = tr.evaluate()
    assert last < first and res["val_acc"] > 0.3, (first, last, res)


def test_split_aggregation_with_init_matches_full():
    """Edges split into two CSRs (rank-local / remote): the second pass adds the
    first pass's fp32 partial -- equals one pass over all edges (SpMM and SpMM-CE)."""
    n, rp, col = _graph(600, 5000, 7)
    torch.manual_seed(2)
    C, ld = 47, 48
    Z = torch.zeros(n, ld)
    Z[:, :C] = torch.randn(n, C)
    Z = Z.to(torch.bfloat16)
    rs = torch.rand(n) + 0.5
    rows = torch.repeat_interleave(torch.arange(n), (rp[1:] - rp[:-1]).long())
    sel = (col.long() % 3) == 0

    def sub(m):
        counts = torch.bincount(rows[m], minlength=n)
        r = torch.zeros(n + 1, dtype=torch.int64)
        r[1:] = torch.cumsum(counts, 0)
        return r.to(torch.int32), col[m]

    (ra, ca), (rb, cb) = sub(sel), sub(~sel)
    d = "cuda:0"
    full = ops.spmm(rp.to(d), col.to(d), Z.to(d), C, rscale=rs.to(d)).float().cpu()
    part = ops.spmm(ra.to(d), ca.to(d), Z.to(d), C, out_dtype=torch.float32)
    two = ops.spmm(rb.to(d), cb.to(d), Z.to(d), C, rscale=rs.to(d), init=part).float().cpu()
    np.testing.assert_allclose(two.numpy(), full.numpy(), rtol=2e-2, atol=2e-2)
    y = torch.randint(0, C, (n,), dtype=torch.int32)
    mask = torch.randint(0, 4, (n,), dtype=torch.uint8)
    b2 = torch.randn(C)
    s_full, g_full = ops.spmm_ce(rp.to(d), col.to(d), Z.to(d), C, rs.to(d), b2.to(d), y.to(d), mask.to(d), 0.01)
    s_two, g_two = ops.spmm_ce(rb.to(d), cb.to(d), Z.to(d), C, rs.to(d), b2.to(d), y.to(d), mask.to(d), 0.01,
                               init=part)
    np.testing.assert_allclose(s_two.cpu().numpy(), s_full.cpu().numpy(), rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(g_two.float().cpu().numpy(), g_full.float().cpu().numpy(), rtol=2e-2, atol=1e-4)


@pytest.mark.parametrize("F,ld", [(41, 48), (256, 256), (602, 608)])
@pytest.mark.parametrize("odt", [torch.float16, torch.float32])
def test_spmm_fp16_matches_reference(F, ld, odt):
    """fp16 storage (inference path): gathered rows fp16, fp32 accumulation."""
    n, rp, col = _graph(400, 3000, 4)
    torch.manual_seed(3)
    X = torch.randn(n, ld)
    X[:, F:] = 0
    X = X.to(torch.float16)
    rs = torch.rand(n) + 0.5
    bias = torch.randn(F)
    ref = ops.spmm(rp, col, X.float(), F, rscale=rs, bias=bias, relu=True, out_dtype=torch.float32)
    got = ops.spmm(rp.cuda(), col.cuda(), X.cuda(), F, rscale=rs.cuda(), bias=bias.cuda(), relu=True,
                   out_dtype=odt).cpu()
    tol = 5e-3 if odt == torch.float16 else 1e-4
    np.testing.assert_allclose(got.float().numpy(), ref.numpy(), rtol=tol, atol=tol)


def test_deep_gcn_captured_matches_eager_and_cpu():
    """3-layer GCN: hipGraph-replayed steps equal eager steps; both track the fp32
    CPU reference (no dropout, so the three runs see the same function)."""
    from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer
    g = synthetic("ogbn-arxiv", seed=2, device="cpu", scale=0.02)
    cpu = DeepGCNTrainer(g, hidden=64, layers=3, dropout=0.0)
    gd = g.to("cuda:0")
    cap = DeepGCNTrainer(gd, hidden=64, layers=3, dropout=0.0, dtype=torch.float32, capture=True)
    eag = DeepGCNTrainer(gd, hidden=64, layers=3, dropout=0.0, dtype=torch.float32, capture=False)
    for _ in range(6):
        lc, lg, le = float(cpu.train_step()), float(cap.train_step()), float(eag.train_step())
        assert lg == pytest.approx(le, rel=1e-5)
        assert lg == pytest.approx(lc, rel=1e-3)
    assert cap._step_graph.graph is not None          # the later steps were graph replays
    bf = DeepGCNTrainer(gd, hidden=64, layers=3, dropout=0.5, dtype=torch.bfloat16)
    first = float(bf.train_step())
    for _ in range(30):
        last = float(bf.train_step())
    assert last < first


def test_gcn_inference_fp16_graph_matches_cpu():
    from cgnn_amd.gnn.gcn_deep import GCNInference
    from cgnn_amd.gnn.layers import GCN
    g = synthetic("reddit", seed=0, device="cpu", scale=0.003)
    model = GCN([g.n_features, 128, g.n_classes], seed=1)
    model.eval()
    ref = GCNInference.from_model(g, model)()                       # fp32 CPU reference
    inf = GCNInference.from_model(g.to("cuda:0"), model.to("cuda:0"), dtype=torch.float16)
    assert inf._lin                       # transforms on the hand-written fp16 MFMA layer
    for _ in range(4):                                              # warm-up, capture, replays
        got = inf()
    assert inf._graph.graph is not None
    got = got.float().cpu()
    scale = ref.abs().max().item()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=2e-2 * scale, rtol=0)
    assert (got.argmax(1) == ref.argmax(1)).float().mean() > 0.98


def test_deep_gcn_checkpoint_resume_gpu(tmp_path):
    from cgnn_amd.gnn.checkpoint import load_trainer, save_trainer
    from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer
    g = synthetic("ogbn-arxiv", seed=1, device="cuda:0", scale=0.01)
    a = DeepGCNTrainer(g, hidden=64, layers=3, dropout=0.0, dtype=torch.float32)
    for _ in range(5):
        a.train_step()
    save_trainer(a, str(tmp_path / "a.safetensors"))
    b = DeepGCNTrainer(g, hidden=64, layers=3, dropout=0.0, dtype=torch.float32, seed=4)
    load_trainer(b, str(tmp_path / "a.safetensors"))
    for _ in range(3):
        assert float(a.train_step()) == pytest.approx(float(b.train_step()), rel=1e-5)


def test_sage_three_layer_gpu():
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=0.005, feat_noise=4.0)
    tr = SAGETrainer(g, hidden=128, layers=3, fanouts=(15, 10, 5), batch_size=64, lr=0.003)
    first = tr.train_epoch()
    for _ in range(8):
        last = tr.train_epoch()
    res = tr.evaluate()
    assert last < first and res["val_acc"] > 0.3, (first, last, res)


def test_device_sampler_matches_reference():
    """HIP neighbour sampler + device relabelling == the NumPy twin (same Philox
    draws, Floyd's algorithm, same local ids), and every pick is a real neighbour."""
    from cgnn_amd.gnn.sampler import DeviceSampler, sample_reference
    g = synthetic("ogbn-arxiv", seed=4, scale=0.01)
    rp, col = g.rowptr.numpy(), g.col.numpy()
    seeds = np.random.default_rng(0).choice(g.n, 50, replace=False)
    fanouts = [7, 3, 20]
    ds = DeviceSampler(g.rowptr.cuda(), g.col.cuda(), fanouts, seed=3)
    blocks, nodes_in = ds.sample(torch.as_tensor(seeds).cuda(), salt=11)
    ref = sample_reference(rp, col, seeds, fanouts, 11, seed=3)
    for blk, (r_rp, r_col, r_src) in zip(blocks[::-1], ref):
        np.testing.assert_array_equal(blk.rowptr.cpu().numpy(), r_rp)
        np.testing.assert_array_equal(blk.col.cpu().numpy(), r_col)
        assert blk.n_src == len(r_src)
    np.testing.assert_array_equal(nodes_in.cpu().numpy(), ref[-1][2])
    # picks are distinct neighbours of their row
    r_rp, r_col, r_src = ref[0]
    for i, v in enumerate(seeds):
        picks = r_src[r_col[r_rp[i]:r_rp[i + 1]]]
        nb = set(col[rp[v]:rp[v + 1]].tolist())
        assert len(set(picks.tolist())) == len(picks) and set(picks.tolist()) <= nb
    assert int(ds.map.max()) == -1                   # the relabel map is reset
    assert not bool(ds.flag.any())                   # and so is the new-source bitmap


def test_gcn_hipgraph_epochs_equal_eager():
    """The captured one-GPU epoch (replayed hipGraph; dropout step read from the device
    step counter) is bitwise equal to eager launches, epoch after epoch -- in
    particular every replay draws a fresh dropout mask."""
    g = synthetic("ogbn-products", seed=1, device="cuda:0", scale=0.003)
    eager = GCNTrainer(g, hidden=256, capture=False)
    graph = GCNTrainer(g, hidden=256, capture=True)
    assert graph._graph.enabled and not eager._graph.enabled
    for _ in range(7):                       # 3 warm-up calls, the capture, then replays
        eager.train_step()
        graph.train_step()
    torch.cuda.synchronize()
    assert graph._graph.graph is not None
    assert torch.equal(eager.params, graph.params)
    assert torch.equal(eager.last_stats, graph.last_stats)
    assert int(graph.step_t.item()) == 7 == graph.epoch


def test_fused_deep_gcn_gpu_matches_cpu_reference():
    """3-layer fused GCN epoch on the HIP kernels (hipGraph-captured and eager) vs the
    same epoch on the ops' CPU reference branches -- identical Philox dropout masks,
    so the runs see the same function up to bf16 rounding / accumulation order."""
    from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer
    g = synthetic("ogbn-arxiv", seed=3, device="cpu", scale=0.01)
    cpu = DeepGCNTrainer(g, hidden=64, layers=3, dropout=0.5, fused=True)
    gd = g.to("cuda:0")
    cap = DeepGCNTrainer(gd, hidden=64, layers=3, dropout=0.5, capture=True)
    eag = DeepGCNTrainer(gd, hidden=64, layers=3, dropout=0.5, capture=False)
    assert cap.fused and eag.fused
    for _ in range(8):
        lc, lg, le = float(cpu.train_step()), float(cap.train_step()), float(eag.train_step())
        assert lg == le                                    # replay is bitwise the eager epoch
        assert lg == pytest.approx(lc, rel=1e-2)
    assert cap._step_graph.graph is not None
    rc, rg = cpu.evaluate(), cap.evaluate()
    assert rg["train_loss"] == pytest.approx(rc["train_loss"], rel=1e-2)
    assert abs(rg["val_acc"] - rc["val_acc"]) < 0.02


def test_fused_sage_gpu_matches_cpu_reference():
    """Fused GraphSAGE mini-batch epoch on the HIP kernels vs the same schedule on the
    CPU reference branches (same host-sampled blocks, same Philox dropout)."""
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-arxiv", seed=2, device="cpu", scale=0.01, feat_noise=2.0, label_noise=0.1)
    kw = dict(hidden=64, layers=3, fanouts=(5, 5, 5), batch_size=256, lr=0.01, dropout=0.5, prefetch=False,
              sampler="host")
    cpu = SAGETrainer(g, fused=True, **kw)
    gpu = SAGETrainer(g.to("cuda:0"), fused=True, **kw)
    for _ in range(3):
        lc, lg = cpu.train_epoch(), gpu.train_epoch()
        assert lg == pytest.approx(lc, rel=2e-2), (lc, lg)
    rc, rg = cpu.evaluate(), gpu.evaluate()
    assert abs(rc["val_acc"] - rg["val_acc"]) < 0.03, (rc, rg)
    # device sampler path trains too
    dev = SAGETrainer(g.to("cuda:0"), hidden=64, layers=3, fanouts=(5, 5, 5), batch_size=256, lr=0.01)
    assert dev.fused
    first = dev.train_epoch()
    for _ in range(4):
        last = dev.train_epoch()
    assert last < first


@pytest.mark.parametrize("S,W,G,mapped", [(76531, 68, None, False), (256, 49152, None, True), (7, 5, 1, False),
                                          (5000, 130, 64, True)])
def test_slab_sum_matches_torch(S, W, G, mapped):
    """Fixed-order column sums of block partials (one or two passes, optional scatter)."""
    torch.manual_seed(0)
    P = torch.randn(S, W, device="cuda:0")
    ref = P.double().sum(0).float()
    if mapped:
        perm = torch.randperm(W + 9, device="cuda:0")[:W].to(torch.int32)
        perm[::7] = -1
        out = torch.zeros(W + 9, device="cuda:0")
        ops.slab_sum(P, out, perm, groups=G)
        keep = perm >= 0
        got, want = out[perm[keep].long()], ref[keep]
        assert torch.all(out[torch.tensor(sorted(set(range(W + 9)) - set(perm[keep].tolist())),
                                          dtype=torch.long, device="cuda:0")] == 0)
    else:
        out = torch.empty(W, device="cuda:0")
        ops.slab_sum(P, out, groups=G)
        got, want = out, ref
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-3)
    out2 = out.clone()
    ops.slab_sum(P, out2, perm if mapped else None, groups=G)
    assert torch.equal(out, out2)          # deterministic


def test_gcn_train_row_layer2_gpu_matches_all_rows():
    """One GPU, HIP path: training epochs that aggregate layer 2 only at the train rows
    (default) give the losses, parameters and evaluation of the all-row aggregation
    (train_rows_only=False) up to summation order."""
    g = synthetic("ogbn-products", seed=4, device="cuda:0", scale=0.004)
    runs = []
    for rows_only in (False, True):
        tr = GCNTrainer(g, hidden=64, rank=0, world=1, train_rows_only=rows_only)
        assert (tr._l2 is None) == (not rows_only)
        losses = []
        for _ in range(4):
            tr.train_step()
            losses.append(tr.train_loss())
        runs.append((losses, tr.params.clone().cpu(), tr.evaluate()))
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=1e-4)
    d = (runs[1][1] - runs[0][1]).abs()
    assert d.max().item() < 1e-3 and (d > 1e-4).float().mean().item() < 0.01, (d.max(), (d > 1e-4).float().mean())
    assert runs[1][2]["val_acc"] == pytest.approx(runs[0][2]["val_acc"], abs=2e-3)


def test_spmm_ell_matches_csr_spmm():
    """The ELL short-row aggregation (rows up to 8 entries from the image, longer rows
    through their CSR range) equals the CSR SpMM, bf16 in / out."""
    torch.manual_seed(4)
    n_src, n, C, ld = 3000, 2500, 47, 48
    deg = torch.randint(0, 9, (n,))
    deg[torch.randperm(n)[:40]] = torch.randint(9, 140, (40,))
    rp = torch.zeros(n + 1, dtype=torch.int32)
    rp[1:] = torch.cumsum(deg, 0).to(torch.int32)
    col = torch.randint(0, n_src, (int(rp[-1]),), dtype=torch.int32)
    X = torch.zeros(n_src, ld, dtype=torch.bfloat16)
    X[:, :C] = torch.randn(n_src, C).to(torch.bfloat16)
    rs = torch.rand(n) + 0.5
    rpc, colc, Xc, rsc = rp.cuda(), col.cuda(), X.cuda(), rs.cuda()
    ell = ops.ell_image(rpc, colc)
    cpu_img = ops.ell_image(rp, col)
    assert torch.equal(ell.ell.cpu(), cpu_img.ell)
    assert torch.equal(ell.long_rows.cpu(), cpu_img.long_rows) and ell.n_long == 40
    got = ops.spmm_ell(ell, colc, Xc, C, rscale=rsc)
    ref = ops.spmm(rpc, colc, Xc, C, rscale=rsc, out=torch.empty(n, ld, dtype=torch.bfloat16, device="cuda"))
    np.testing.assert_allclose(got.cpu().float().numpy(), ref.cpu().float().numpy(), rtol=1e-2, atol=1e-2)
    assert torch.all(got[:, C:] == 0)
    mirror = ops.spmm_ell(cpu_img, col, X, C, rscale=rs)          # the CPU mirror of the image
    np.testing.assert_allclose(got.cpu().float().numpy(), mirror.float().numpy(), rtol=1e-2, atol=1e-2)
    # no row computed twice / skipped at any grid size: a shape with a ragged last group
    # and more row groups than the persistent grid's waves
    for n2 in (1, 7, 9, 70001):
        rp2 = torch.zeros(n2 + 1, dtype=torch.int32)
        d2 = torch.randint(0, 11, (n2,))
        rp2[1:] = torch.cumsum(d2, 0).to(torch.int32)
        c2 = torch.randint(0, n_src, (int(rp2[-1]),), dtype=torch.int32)
        img2 = ops.ell_image(rp2.cuda(), c2.cuda())
        y2 = torch.full((n2 + 5, ld), 3.0, dtype=torch.bfloat16, device="cuda")
        ops.spmm_ell(img2, c2.cuda(), Xc, C, out=y2)
        r2 = ops.spmm(rp2.cuda(), c2.cuda(), Xc, C, out=torch.empty(n2, ld, dtype=torch.bfloat16, device="cuda"))
        assert torch.equal(y2[:n2].view(torch.int16), r2.view(torch.int16))
        assert torch.all(y2[n2:] == 3.0)

