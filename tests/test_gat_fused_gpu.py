"""HIP kernels of the fused GAT epoch (gnn_gat.hip dense-side kernels, lin_fwd's
fp32 score planes) against their CPU reference branches, and the whole fused epoch
on the GPU against the same epoch on the CPU."""
import numpy as np
import pytest
import torch

from cgnn_amd.gnn import ops
from cgnn_amd.gnn.data import synthetic
from cgnn_amd.gnn.gat import GATTrainer
from cgnn_amd.gnn.gat_fused import act_bwd, act_fwd, pack_grad, row_ce
from cgnn_amd.gnn.linear import lin_fwd

pytestmark = pytest.mark.gpu


def _cuda(*ts):
    return [t.cuda() if t is not None else None for t in ts]


def _ring_graph(n, deg, seed):
    from cgnn_amd.gnn.gat import GraphCSR
    g = torch.Generator().manual_seed(seed)
    d = torch.randint(1, deg + 1, (n,), generator=g)
    d[::17] = 0                                            # some rows without edges
    rp = torch.zeros(n + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(d, 0)
    col = torch.randint(0, n, (int(rp[-1]),), generator=g, dtype=torch.int64)
    return GraphCSR(rp.to(torch.int32), col.to(torch.int32), n)


@pytest.mark.parametrize("F,p,row0", [(128, 0.5, 0), (256, 0.3, 1000), (32, 0.0, 7)])
def test_fused_activation_fwd_bwd_match_reference(F, p, row0):
    """The hidden layer's activation runs inside the aggregation kernels on a GPU: the
    forward writes bf16(dropout(elu(out + b))) (act_fwd's CPU reference), the row half of
    the backward makes dout = dH * mask * elu'(out + b) and db (act_bwd's)."""
    from cgnn_amd.gnn.gat_fused import _agg_fwd, _agg_rows
    torch.manual_seed(0)
    n, K = 777, F // 32
    Fh = F // K
    g = _ring_graph(n, 9, 1)
    Wh = (torch.randn(n, F) * 2).to(torch.bfloat16)
    s_src, s_dst = torch.randn(n, K), torch.randn(n, K)
    b = torch.randn(F) * 0.1
    key, step = (11, 22), 5
    out, _ = _agg_fwd(Wh, s_src, s_dst, g, K, Fh)
    H = torch.zeros(n, F, dtype=torch.bfloat16)
    act_fwd(out, b, H, p, key, step, row0)
    Hg = torch.zeros(n, F, dtype=torch.bfloat16, device="cuda")
    stp = torch.tensor([step], dtype=torch.int32, device="cuda")
    gg = _ring_graph(n, 9, 1)
    gg.rowptr, gg.col = gg.rowptr.cuda(), gg.col.cuda()
    outg, lse = _agg_fwd(*_cuda(Wh, s_src, s_dst), gg, K, Fh, q=torch.empty(n, F, dtype=torch.bfloat16, device="cuda"),
                         act=(b.cuda(), Hg, p, key, stp, row0))
    np.testing.assert_allclose(outg.cpu().numpy(), out.numpy(), rtol=1e-4, atol=1e-4)
    # the GPU activation reads its own fp32 out: compare against the reference on it
    Hr = torch.zeros(n, F, dtype=torch.bfloat16)
    act_fwd(outg.cpu(), b, Hr, p, key, step, row0)
    np.testing.assert_allclose(Hg.cpu().float().numpy(), Hr.float().numpy(), rtol=8e-3, atol=1e-6)
    np.testing.assert_allclose(Hg.cpu().float().numpy(), H.float().numpy(), rtol=2e-2, atol=1e-3)
    dH = torch.randn(n, F).to(torch.bfloat16)
    dout, doutb, db = torch.zeros(n, F), torch.zeros(n, F, dtype=torch.bfloat16), torch.zeros(F)
    act_bwd(dH, outg.cpu(), b, p, key, step, row0, dout, doutb, db)
    dgb, dbg = torch.zeros(n, F, dtype=torch.bfloat16, device="cuda"), torch.zeros(F, device="cuda")
    rstat = torch.empty(n, K, 4, device="cuda")
    q = torch.zeros(n, F, dtype=torch.bfloat16, device="cuda")
    _agg_rows(outg, q, lse, s_dst.cuda(), None, K, Fh, rstat, dH=dH.cuda(),
              act=(dgb, b.cuda(), dbg, p, key, stp, row0), ds_dst=torch.empty(n, K, device="cuda"))
    np.testing.assert_allclose(dgb.cpu().float().numpy(), doutb.float().numpy(), rtol=8e-3, atol=1e-6)
    np.testing.assert_allclose(dbg.cpu().numpy(), db.numpy(), rtol=1e-4, atol=1e-4)
    D = (dgb.float() * outg).view(n, K, Fh).sum(-1)
    np.testing.assert_allclose(rstat[:, :, 2].cpu().numpy(), D.cpu().numpy(), rtol=1e-4, atol=1e-4)
    # (s_dst, lse) are handed to the column half in log2 units
    L2E = 1.4426950408889634
    np.testing.assert_allclose(rstat[:, :, 0].cpu().numpy(), s_dst.numpy() * L2E, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rstat[:, :, 1].cpu().numpy(), lse.cpu().numpy() * L2E, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("K,Fh", [(4, 32), (1, 48), (8, 16)])
def test_row_half_split_equals_edge_sum(K, Fh):
    """d s_dst from the forward's LeakyReLU split (-0.8 <dout, q>) equals the per-edge sum
    sum_j alpha_ij (dalpha_ij - D_i) LeakyReLU'_ij of the autograd reference."""
    from cgnn_amd.gnn.gat import _gat_aggregate_torch
    from cgnn_amd.gnn.gat_fused import _agg_fwd, _agg_rows
    torch.manual_seed(3)
    n = 1500
    HF = K * Fh
    g = _ring_graph(n, 20, 2)
    Wh = torch.randn(n, HF).to(torch.bfloat16)
    s_src, s_dst = torch.randn(n, K), torch.randn(n, K)
    dout = torch.randn(n, HF).to(torch.bfloat16)
    with torch.enable_grad():
        c = s_dst.clone().requires_grad_()
        o = _gat_aggregate_torch(Wh.float(), s_src, c, g, K, Fh)
        (ref,) = torch.autograd.grad(o, (c,), dout.float())
    gg = _ring_graph(n, 20, 2)
    gg.rowptr, gg.col = gg.rowptr.cuda(), gg.col.cuda()
    q = torch.empty(n, HF, dtype=torch.bfloat16, device="cuda")
    out, lse = _agg_fwd(*_cuda(Wh, s_src, s_dst), gg, K, Fh, q=q)
    rstat = torch.empty(n, K, 4, device="cuda")
    dsd = torch.empty(n, K, device="cuda")
    _agg_rows(out, q, lse, s_dst.cuda(), None, K, Fh, rstat, dout=dout.cuda(), ds_dst=dsd)
    scale = ref.abs().max().item()
    np.testing.assert_allclose(dsd.cpu().numpy(), ref.numpy(), rtol=2e-2, atol=1e-2 * scale)


@pytest.mark.parametrize("C,ld", [(47, 48), (172, 176), (7, 8), (256, 256)])
def test_row_ce_matches_reference(C, ld):
    torch.manual_seed(1)
    n = 5000
    Z = torch.randn(n, ld) * 3
    b = torch.randn(C)
    y = torch.randint(0, C, (n,), dtype=torch.int32)
    mask = torch.randint(0, 4, (n,), dtype=torch.uint8)
    inv = 1.0 / max(int((mask == 1).sum()), 1)
    dZ, dZb, db = torch.zeros(n, ld), torch.zeros(n, ld, dtype=torch.bfloat16), torch.zeros(C)
    st = row_ce(Z, b, C, y, mask, inv, dZ=dZ, dZb=dZb, db=db)
    g = _cuda(Z, b, y, mask)
    dZg = torch.full((n, ld), 7.0, device="cuda")
    dZbg = torch.zeros(n, ld, dtype=torch.bfloat16, device="cuda")
    dbg = torch.zeros(C, device="cuda")
    stg = row_ce(*g[:2], C, g[2], g[3], inv, dZ=dZg, dZb=dZbg, db=dbg)
    np.testing.assert_allclose(stg.cpu().numpy(), st.numpy(), rtol=1e-4)
    np.testing.assert_allclose(dZg.cpu().numpy(), dZ.numpy(), atol=1e-7)
    np.testing.assert_allclose(dZbg.cpu().float().numpy(), dZb.float().numpy(), rtol=8e-3, atol=1e-9)
    np.testing.assert_allclose(dbg.cpu().numpy(), db.numpy(), atol=1e-6)
    ste = row_ce(*g[:2], C, g[2], g[3], inv)               # evaluation: statistics only
    np.testing.assert_allclose(ste.cpu().numpy(), st.numpy(), rtol=1e-4)


def test_pack_grad_and_lin_fwd_score_planes():
    torch.manual_seed(2)
    n, HF, K = 1000, 128, 4
    dWh, ds, dd = torch.randn(n, HF), torch.randn(n, K), torch.randn(n, K)
    dy = torch.zeros(n, 136, dtype=torch.bfloat16)
    pack_grad(dWh, ds, dd, dy)
    dyg = torch.full((n, 136), 3.0, dtype=torch.bfloat16, device="cuda")
    pack_grad(*_cuda(dWh, ds, dd), dyg)
    assert torch.equal(dyg.cpu(), dy)
    # lin_fwd with the fp32 tail: [Wh (bf16) | s planes (fp32)]
    x = torch.randn(n, 104).to(torch.bfloat16)
    W = torch.randn(100, HF + 2 * K) * 0.1
    Wh, s = torch.zeros(n, HF, dtype=torch.bfloat16), torch.zeros(2, n, K)
    lin_fwd(x, W, None, K1=100, out=Wh, tail=s, nsplit=HF, tk=K)
    Whg, sg = torch.zeros(n, HF, dtype=torch.bfloat16, device="cuda"), torch.zeros(2, n, K, device="cuda")
    lin_fwd(x.cuda(), W.cuda(), None, K1=100, out=Whg, tail=sg, nsplit=HF, tk=K)
    np.testing.assert_allclose(Whg.cpu().float().numpy(), Wh.float().numpy(), rtol=1e-2, atol=1e-2)
    np.testing.assert_allclose(sg.cpu().numpy(), s.numpy(), rtol=1e-4, atol=1e-4)
    ref = x[:, :100].float() @ W.to(torch.bfloat16).float()
    np.testing.assert_allclose(sg[0].cpu().numpy(), ref[:, HF:HF + K].numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(sg[1].cpu().numpy(), ref[:, HF + K:].numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("heads,head_dim", [(4, 32), (8, 32), (4, 8)])
def test_fused_gat_epoch_gpu_matches_cpu(heads, head_dim):
    g = synthetic("ogbn-products", seed=3, scale=0.002)
    cpu = GATTrainer(g, heads=heads, head_dim=head_dim, dropout=0.5, lr=0.01, seed=0, fused=True)
    gpu = GATTrainer(g.to("cuda:0"), heads=heads, head_dim=head_dim, dropout=0.5, lr=0.01, seed=0)
    assert gpu.fused is not None
    lc, lg = [], []
    for it in range(3):
        lc.append(float(cpu.train_step()))
        lg.append(float(gpu.train_step()))
        if it == 0:
            # first-step gradients: same bf16-stored operands, fp32 MFMA accumulation in
            # another order (a bf16 rounding of an intermediate can flip by one ulp)
            gc, gg = cpu.fused.grads.clone(), gpu.fused.grads.cpu()
            assert (gg - gc).abs().max() < 1e-2 * gc.abs().max(), ((gg - gc).abs().max(), gc.abs().max())
            assert (gg - gc).norm() < 5e-3 * gc.norm(), ((gg - gc).norm(), gc.norm())
    # (parameters are not compared after the update: Adam's first steps move every weight
    # by ~lr * sign(g), so a near-zero gradient's rounding decides a 2 lr difference)
    np.testing.assert_allclose(lg, lc, rtol=2e-3)
    a, b = cpu.evaluate(), gpu.evaluate()
    assert abs(a["val_acc"] - b["val_acc"]) < 0.01 and abs(a["train_loss"] - b["train_loss"]) < 2e-3 * a["train_loss"]


def test_fused_gat_learns_products_shape_gpu():
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=0.01)
    tr = GATTrainer(g, heads=4, head_dim=32, dropout=0.5, lr=0.01)
    assert tr.fused is not None
    for _ in range(30):
        tr.train_step()
    res = tr.evaluate()
    assert res["val_acc"] > 0.3, res


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_halo_row_kernel_matches_reference(mode):
    from cgnn_amd.parallel.halo import _rows
    torch.manual_seed(4)
    n, m, w = 3000, 1200, 36
    sdt = torch.bfloat16 if mode == 2 else torch.float32
    src = torch.randn(n, w + 4).to(sdt)
    dst = torch.randn(n, w + 8)
    si = torch.randperm(n)[:m]
    di = torch.randperm(n)[:m]                      # distinct destination rows
    ref = dst.clone()
    _rows(src[:, 2:2 + w] if mode else src[:, :w], ref[:, 4:4 + w], src_idx=si, dst_idx=di, mode=mode)
    got = dst.cuda()
    srcg = src.cuda()
    _rows(srcg[:, 2:2 + w] if mode else srcg[:, :w], got[:, 4:4 + w], src_idx=si.cuda(), dst_idx=di.cuda(), mode=mode)
    np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)
    # byte views: gather bf16 rows into a packed uint8 buffer
    b = torch.randn(n, 16).to(torch.bfloat16)
    buf_ref = torch.zeros(m, 40, dtype=torch.uint8)
    _rows(b.view(torch.uint8), buf_ref[:, 8:40], src_idx=si)
    buf = torch.zeros(m, 40, dtype=torch.uint8, device="cuda")
    _rows(b.cuda().view(torch.uint8), buf[:, 8:40], src_idx=si.cuda())
    assert torch.equal(buf.cpu(), buf_ref)


def _gat_gpu_shard_worker(rank, world, port, out, chunk):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)     # both ranks on cuda:0
    torch.cuda.set_device(0)
    from cgnn_amd.gnn.data import synthetic_shard
    from cgnn_amd.gnn.gat import ShardedGATTrainer
    shard = synthetic_shard("ogbn-products", rank, world, seed=1, device="cuda:0", scale=0.003)
    tr = ShardedGATTrainer(shard, heads=4, head_dim=32, dropout=0.3, lr=0.01, seed=0, halo_chunk_bytes=chunk)
    assert tr.fused is not None and tr.halo.rounds >= 1
    losses = []
    for _ in range(3):
        l = tr.train_step().clone()
        dist.all_reduce(l)
        losses.append(float(l))
    out[rank] = (losses, tr.evaluate(), tr.fused.params.cpu().numpy(), tr.halo.rounds)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk", [(2, 4 << 30), (3, 64 << 10)])
def test_sharded_fused_gat_gpu_matches_one_rank(world, chunk):
    """The graph-sharded fused GAT on the GPU (HIP projection / aggregation / halo row
    kernels, halo exchange in one or several rounds; ranks share the one GPU over gloo)
    against the unsharded fused model on the same GPU."""
    import socket
    import torch.multiprocessing as mp
    from cgnn_amd.gnn.gat import ShardedGATTrainer
    g = synthetic("ogbn-products", seed=1, device="cuda:0", scale=0.003)
    ref = ShardedGATTrainer(g, heads=4, head_dim=32, dropout=0.3, lr=0.01, seed=0)
    ref_losses = [float(ref.train_step()) for _ in range(3)]
    ref_res = ref.evaluate()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_gat_gpu_shard_worker, args=(world, port, out, chunk), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        losses, res, params, rounds = out[r]
        if chunk < (1 << 20):
            assert rounds > 1
        np.testing.assert_allclose(losses, ref_losses, rtol=2e-3)
        assert abs(res["val_acc"] - ref_res["val_acc"]) < 5e-3
    np.testing.assert_array_equal(out[0][2], out[1][2])              # replicas identical


def test_fused_gat_train_row_layer2_gpu_matches_all_rows():
    """HIP path: layer 2 aggregated at the train rows only in training (default) gives
    the first-step gradients and the losses of the all-row aggregation."""
    g = synthetic("ogbn-products", seed=5, device="cuda:0", scale=0.003)
    runs = []
    for rows_only in (False, True):
        tr = GATTrainer(g, heads=4, head_dim=32, dropout=0.5, lr=0.01, seed=0, train_rows_only=rows_only)
        assert tr.fused is not None and (tr.fused._tr is None) == (not rows_only)
        losses = [float(tr.train_step())]
        grads = tr.fused.grads.clone().cpu()
        losses += [float(tr.train_step()) for _ in range(2)]
        runs.append((losses, grads, tr.evaluate()))
    ga, gb = runs[0][1], runs[1][1]
    assert (gb - ga).abs().max() < 2e-3 * ga.abs().max(), ((gb - ga).abs().max(), ga.abs().max())
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=1e-3)
    assert abs(runs[1][2]["val_acc"] - runs[0][2]["val_acc"]) < 5e-3
