"""Graph attention networks (GAT) -- GNN track, not in the reference.

Attention aggregation over the CSR of A + I (multi-head):

    e_ijk = LeakyReLU(a_dst_k . Wh_ik + a_src_k . Wh_jk),  alpha = softmax_j(e),
    out_ik = sum_j alpha_ijk Wh_jk

On a GPU the aggregation runs on three HIP kernels (``gnn_gat.hip``): a fused
forward with an online softmax (edge scores never stored; per-(row, head)
log-sum-exp kept, plus the LeakyReLU split q), a row-wise backward that is a
per-row product (the destination-score gradient is -0.8 <dout_i, q_i>, so it
gathers nothing), and a column-wise backward over the transposed CSR that
recomputes the attention weights and gathers ``dWh`` and the source score
gradient -- no atomics anywhere.  The projections ``Wh = h W`` and the
scores ``s = <Wh, a>`` are PyTorch ops (hipBLASLt), so autograd chains through.
On the CPU the same math is written with PyTorch index ops (the reference the
GPU kernels are tested against).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .. import native
from ..utils import checks
from .data import GraphData
from .sage import transpose_csr


def _st(t):
    return torch._C._cuda_getCurrentRawStream(t.get_device())


class GraphCSR:
    """CSR (A + I) plus its lazily built transpose with the edge permutation.
    ``n`` destination rows; ``n_cols`` source rows (default ``n``; a row block of a
    partitioned graph keeps global source ids, so ``n_cols`` is the global count)."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, n: int, n_cols: Optional[int] = None):
        self.rowptr, self.col, self.n = rowptr.contiguous(), col.contiguous(), int(n)
        self.n_cols = int(n) if n_cols is None else int(n_cols)
        self._t = None
        self._rows = None

    @property
    def nnz(self):
        return int(self.col.numel())

    def transposed(self):
        if self._t is None:
            self._t = transpose_csr(self.rowptr, self.col, self.n_cols)
        return self._t

    def edge_rows(self):
        if self._rows is None:
            counts = (self.rowptr[1:] - self.rowptr[:-1]).long()
            self._rows = torch.repeat_interleave(torch.arange(self.n, device=self.col.device), counts)
        return self._rows


def _check_graph(g: "GraphCSR", Wh, s_src, s_dst, what):
    if checks.enabled():
        checks.csr(g.rowptr, g.col, g.n_cols, what, n_rows=g.n)
        checks.rows(Wh, g.n_cols, what + " Wh")
        checks.rows(s_src, g.n_cols, what + " s_src")
        checks.rows(s_dst, g.n, what + " s_dst")


def _check_transposed(g: "GraphCSR", what):
    if checks.enabled():
        rp_t, col_t = g.transposed()
        checks.csr(rp_t, col_t, g.n, what, n_rows=g.n_cols)


def _gat_forward_kernels(Whg, s_src, s_dst, g: GraphCSR, K: int, Fh: int, lowp: bool, need_q: bool = True):
    """(out, lse, q): the forward plus the LeakyReLU split ``q`` the row half of the
    backward reads (gnn_gat.hip), stored like Whg.  ``need_q=False`` (no backward will
    run: inference, no_grad): q is neither allocated nor written (None)."""
    _check_graph(g, Whg, s_src, s_dst, "gat_fwd")
    n = g.n
    out = torch.empty(n, K * Fh, dtype=torch.float32, device=Whg.device)
    lse = torch.empty(n, K, dtype=torch.float32, device=Whg.device)
    q = torch.empty(n, K * Fh, dtype=Whg.dtype, device=Whg.device) if need_q else None
    native.hip().gnn_gat_fwd(g.rowptr.data_ptr(), g.col.data_ptr(), Whg.data_ptr(), s_src.data_ptr(),
                             s_dst.data_ptr(), out.data_ptr(), lse.data_ptr(), n, K, Fh, _st(Whg), int(lowp),
                             q=q.data_ptr() if q is not None else 0)
    return out, lse, q


def _gat_backward_kernels(Whg, s_src, s_dst, out, lse, q, dout, g: GraphCSR, K: int, Fh: int, lowp: bool):
    """(dWh [n_cols, K*Fh] fp32, ds_src [n_cols, K], ds_dst [n, K]): the row half (per-row
    products: d s_dst and the statistics (s_dst, lse, D) -- no gather) then the column
    half over the transposed CSR, which recomputes the attention weights -- nothing is
    stored per edge."""
    hip = native.hip()
    n, dev = g.n, Whg.device
    _check_graph(g, Whg, s_src, s_dst, "gat_bwd")
    _check_transposed(g, "gat_bwd transposed")
    doutg = dout.contiguous().to(torch.bfloat16 if lowp else torch.float32)
    rstat = torch.empty(n, K, 4, dtype=torch.float32, device=dev)
    ds_dst = torch.empty(n, K, dtype=torch.float32, device=dev)
    st = _st(Whg)
    hip.gnn_gat_rows(0, doutg.data_ptr(), 0, out.data_ptr(), q.data_ptr(), lse.data_ptr(), s_dst.data_ptr(), 0,
                     rstat.data_ptr(), ds_dst.data_ptr(), 0, 0, 0, 0, 0, 0, 0.0, 0, 0, 0, 0, 0, n, K, Fh, int(lowp), st)
    rp_t, col_t = g.transposed()
    dWh = torch.empty(g.n_cols, K * Fh, dtype=torch.float32, device=dev)   # one row per source
    ds_src = torch.empty(g.n_cols, K, dtype=torch.float32, device=dev)
    hip.gnn_gat_col(rp_t.data_ptr(), col_t.data_ptr(), Whg.data_ptr(), s_src.data_ptr(), rstat.data_ptr(),
                    doutg.data_ptr(), dWh.data_ptr(), ds_src.data_ptr(), 0, 0, g.n_cols, K, Fh, st, int(lowp))
    return dWh, ds_src, ds_dst


class _GATAggregate(torch.autograd.Function):
    """HIP attention aggregation.  ``lowp``: the edge-gathered matrices (Wh in the
    forward and the row backward, dout in the column backward) are stored bf16,
    halving the bytes of every gathered row; scores, softmax statistics, the
    accumulation and all gradients stay fp32."""

    @staticmethod
    def forward(ctx, Wh, s_src, s_dst, g: GraphCSR, K: int, Fh: int, lowp: bool):
        Whg = Wh.to(torch.bfloat16).contiguous() if lowp else Wh.contiguous()
        s_src, s_dst = s_src.contiguous(), s_dst.contiguous()
        # q only when a backward can follow (the tensors' grad flags survive into forward)
        need_q = any(ctx.needs_input_grad[:3])
        out, lse, q = _gat_forward_kernels(Whg, s_src, s_dst, g, K, Fh, lowp, need_q=need_q)
        if need_q:
            ctx.save_for_backward(Whg, s_src, s_dst, out, lse, q)
        ctx.g, ctx.K, ctx.Fh, ctx.lowp = g, K, Fh, lowp
        return out

    @staticmethod
    def backward(ctx, dout):
        Whg, s_src, s_dst, out, lse, q = ctx.saved_tensors
        dWh, ds_src, ds_dst = _gat_backward_kernels(Whg, s_src, s_dst, out, lse, q, dout, ctx.g, ctx.K, ctx.Fh,
                                                    ctx.lowp)
        return dWh, ds_src, ds_dst, None, None, None, None


class _HaloGAT(torch.autograd.Function):
    """Graph-sharded attention aggregation: the source-side ``[Wh | s_src]`` of this
    rank's rows goes through ONE halo all-to-all (Wh as bf16 on the wire when ``lowp``,
    the attention scores exactly as fp32), the HIP kernels (or the CPU reference)
    aggregate over the extended rows ``[own | received]``, and the backward returns
    the gradients of the received rows to their owners (fp32) through the transposed
    exchange."""

    @staticmethod
    def forward(ctx, Wh, s_src, s_dst, g: GraphCSR, K: int, Fh: int, lowp: bool, halo,
                grad_wire=torch.float32):
        wdt = torch.bfloat16 if (lowp and Wh.is_cuda) else torch.float32
        ctx.grad_wire = grad_wire
        Wh_ext, s_ext = halo.exchange_parts([Wh.to(wdt).contiguous(), s_src.float().contiguous()])
        ctx.g, ctx.K, ctx.Fh, ctx.lowp, ctx.halo = g, K, Fh, lowp, halo
        s_dst = s_dst.contiguous()
        if Wh.is_cuda:
            need_q = any(ctx.needs_input_grad[:3])
            out, lse, q = _gat_forward_kernels(Wh_ext, s_ext, s_dst, g, K, Fh, wdt == torch.bfloat16,
                                               need_q=need_q)
            if need_q:
                ctx.save_for_backward(Wh_ext, s_ext, s_dst, out, lse, q)
            return out
        ctx.save_for_backward(Wh_ext, s_ext, s_dst)
        return _gat_aggregate_torch(Wh_ext, s_ext, s_dst, g, K, Fh)

    @staticmethod
    def backward(ctx, dout):
        g, K, Fh, halo = ctx.g, ctx.K, ctx.Fh, ctx.halo
        if dout.is_cuda:
            Wh_ext, s_ext, s_dst, out, lse, q = ctx.saved_tensors
            dWh, ds_src, ds_dst = _gat_backward_kernels(Wh_ext, s_ext, s_dst, out, lse, q, dout, g, K, Fh,
                                                        Wh_ext.dtype == torch.bfloat16)
        else:
            Wh_ext, s_ext, s_dst = ctx.saved_tensors
            with torch.enable_grad():
                a = Wh_ext.detach().requires_grad_()
                b = s_ext.detach().requires_grad_()
                c = s_dst.detach().requires_grad_()
                o = _gat_aggregate_torch(a, b, c, g, K, Fh)
                dWh, ds_src, ds_dst = torch.autograd.grad(o, (a, b, c), dout)
        dWh_loc, ds_loc = halo.reduce_back([dWh.float(), ds_src.float()], ctx.grad_wire)
        return dWh_loc, ds_loc, ds_dst, None, None, None, None, None, None


def _gat_aggregate_torch(Wh, s_src, s_dst, g: GraphCSR, K: int, Fh: int):
    rows = g.edge_rows()
    cols = g.col.long()
    raw = s_dst[rows] + s_src[cols]                                   # [nnz, K]
    e = torch.nn.functional.leaky_relu(raw, 0.2)
    m = torch.full((g.n, K), -math.inf, dtype=e.dtype, device=e.device)
    m = m.scatter_reduce(0, rows[:, None].expand(-1, K), e, "amax", include_self=True)
    w = torch.exp(e - m[rows].detach())
    den = torch.zeros(g.n, K, dtype=e.dtype, device=e.device).index_add(0, rows, w)
    alpha = w / den[rows]
    msg = alpha[:, :, None] * Wh.view(-1, K, Fh)[cols]
    out = torch.zeros(g.n, K, Fh, dtype=Wh.dtype, device=Wh.device).index_add(0, rows, msg)
    return out.view(g.n, K * Fh)


def gat_aggregate(Wh: torch.Tensor, s_src: torch.Tensor, s_dst: torch.Tensor, g: GraphCSR, K: int, Fh: int,
                  lowp: bool = True):
    """Multi-head attention aggregation; Wh [n_cols, K*Fh] fp32, s_src [n_cols, K],
    s_dst [n, K]; returns [n, K*Fh] fp32.  On a GPU ``lowp`` stores the
    edge-gathered rows bf16 (see ``_GATAggregate``); the CPU path is fp32."""
    if Wh.shape[0] != g.n_cols or s_src.shape[0] != g.n_cols or s_dst.shape[0] != g.n:
        raise ValueError("gat_aggregate: operand rows do not match the graph (%d x %d)" % (g.n, g.n_cols))
    if Wh.is_cuda:
        if Fh % 8 or (K > 1 and (Fh // 8) & (Fh // 8 - 1)) or K * Fh > 512:
            raise ValueError("HIP GAT needs Fh % 8 == 0 (8 * 2^m with several heads) and K * Fh <= 512")
        return _GATAggregate.apply(Wh.float(), s_src.float(), s_dst.float(), g, K, Fh, bool(lowp))
    return _gat_aggregate_torch(Wh, s_src, s_dst, g, K, Fh)


class GATLayer(torch.nn.Module):
    def __init__(self, in_dim, heads, head_dim, generator=None):
        super().__init__()
        self.K, self.Fh = heads, head_dim
        bound = math.sqrt(6.0 / (in_dim + heads * head_dim))
        self.W = torch.nn.Parameter((torch.rand(in_dim, heads * head_dim, generator=generator) * 2 - 1) * bound)
        ab = math.sqrt(6.0 / (head_dim + 1))
        self.a_src = torch.nn.Parameter((torch.rand(heads, head_dim, generator=generator) * 2 - 1) * ab)
        self.a_dst = torch.nn.Parameter((torch.rand(heads, head_dim, generator=generator) * 2 - 1) * ab)
        self.bias = torch.nn.Parameter(torch.zeros(heads * head_dim))

    def forward(self, h, g: GraphCSR, halo=None):
        """``halo`` (graph-sharded training, ``parallel.halo.HaloExchange``): the
        source-side [Wh | s_src] of this rank's rows goes through ONE all-to-all and the
        aggregation runs over [own | received] rows (``g`` holds the extended columns)."""
        # the attention logits are linear in h: fold a_src / a_dst into the weight,
        # s = h (W a), so [Wh | s_src | s_dst] is ONE GEMM (no [n, K, Fh] temporary,
        # no broadcast multiply + reduction over all rows)
        K, KF = self.K, self.K * self.Fh
        Wk = self.W.view(-1, K, self.Fh)
        Wcat = torch.cat([self.W, (Wk * self.a_src).sum(-1), (Wk * self.a_dst).sum(-1)], 1)
        y = h @ Wcat
        Wh, s_src, s_dst = y[:, :KF], y[:, KF:KF + K], y[:, KF + K:]
        if halo is not None:
            return _HaloGAT.apply(Wh, s_src, s_dst, g, self.K, self.Fh, True, halo,
                                  getattr(halo, "grad_wire", torch.float32)) + self.bias
        return gat_aggregate(Wh, s_src, s_dst, g, self.K, self.Fh) + self.bias


class GAT(torch.nn.Module):
    """2-layer GAT: K heads of width Fh (concatenated, ELU), then one output head
    whose width is the class count padded to a multiple of 8 (a single head is
    reduced over the whole row's lanes, so its width need not be a power of two)."""

    def __init__(self, in_dim, n_classes, heads=8, head_dim=32, dropout=0.5, seed=0):
        super().__init__()
        gen = torch.Generator().manual_seed(seed)
        out_w = (n_classes + 7) // 8 * 8
        self.C = n_classes
        self.l1 = GATLayer(in_dim, heads, head_dim, gen)
        self.l2 = GATLayer(heads * head_dim, 1, out_w, gen)
        self.dropout = float(dropout)

    def forward(self, x, g: GraphCSR, halo=None):
        h = torch.nn.functional.elu(self.l1(x, g, halo))
        if self.training and self.dropout > 0:
            h = torch.nn.functional.dropout(h, self.dropout)
        return self.l2(h, g, halo)[:, :self.C]


def _use_fused(fused, dev, F, heads, head_dim, n_classes):
    """Default: the fused HIP epoch (gat_fused.py) on a GPU when its kernels cover the
    shape, the autograd model otherwise; ``fused=True`` on a CPU runs its fp32
    reference branches (tests)."""
    from .gat_fused import FusedGAT
    ok = FusedGAT.supported(F, heads, head_dim, n_classes)
    if fused is None:
        return ok and dev.type == "cuda"
    if fused and not ok:
        raise ValueError("fused GAT: no kernel variant for F=%d heads=%d head_dim=%d classes=%d"
                         % (F, heads, head_dim, n_classes))
    return bool(fused)


def _gat_state_tensors(tr):
    if tr.fused is not None:
        return tr.fused.state_tensors()
    from .checkpoint import module_optimizer_tensors
    return module_optimizer_tensors(tr.model, tr.opt)


def _gat_load_state_tensors(tr, t):
    if tr.fused is not None:
        tr.fused.load_state_tensors(t)
    else:
        from .checkpoint import load_module_optimizer_tensors
        load_module_optimizer_tensors(tr.model, tr.opt, t)


class GATTrainer:
    """Full-graph GAT node classification (Adam, cross-entropy on the train split).
    ``fused`` (default: on a GPU): the whole epoch on HIP kernels (``gat_fused``);
    otherwise the autograd model over the HIP aggregation."""

    def __init__(self, gd: GraphData, heads=8, head_dim=32, dropout=0.5, lr=0.005, seed=0, standardize=True,
                 fused: Optional[bool] = None, reorder: bool = False, train_rows_only: bool = True,
                 l1_train_neighbours: bool = True):
        # reorder=True: the framework's locality pass first (data.reorder; the attention
        # kernels gather rows like the SpMM, so their L2 hit rate follows the order);
        # evaluation and dropout-0 training are invariant, with dropout > 0 the masks are
        # keyed by the relabelled rows (equal in distribution only); ``new_id`` maps
        # caller ids to trainer rows
        self.new_id = None
        if reorder:
            from .data import reorder as _reorder
            gd, self.new_id = _reorder(gd, seed=seed)
        self.gd = gd
        self.dev = gd.rowptr.device
        x = gd.x.float()
        if standardize:
            x = (x - x.mean(0)) / x.std(0).clamp_min(1e-6)
        self.x = x
        self.g = GraphCSR(gd.rowptr, gd.col, gd.n)
        self.tr = gd.mask == 1
        self.fused = None
        if _use_fused(fused, self.dev, x.shape[1], heads, head_dim, gd.n_classes):
            from .gat_fused import FusedGAT
            self.fused = FusedGAT(x, gd.y, gd.mask, gd.n_classes, self.g, heads, head_dim, dropout, lr, seed,
                                  train_rows_only=train_rows_only, l1_train_neighbours=l1_train_neighbours)
            self.model = self.opt = None
            return
        self.model = GAT(x.shape[1], gd.n_classes, heads, head_dim, dropout, seed).to(self.dev)
        self.opt = torch.optim.Adam(self.model.parameters(), lr=lr, fused=self.dev.type == "cuda")

    def state_tensors(self):
        return _gat_state_tensors(self)

    def load_state_tensors(self, t):
        _gat_load_state_tensors(self, t)

    def train_step(self):
        if self.fused is not None:
            return self.fused.train_step()
        self.model.train()
        out = self.model(self.x, self.g)
        loss = torch.nn.functional.cross_entropy(out[self.tr], self.gd.y[self.tr].long())
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        return loss.detach()

    @torch.no_grad()
    def evaluate(self):
        if self.fused is not None:
            c = self.fused.evaluate_counts().cpu().double().numpy()
            m = self.gd.mask
            res = {"train_loss": float(c[0]) / self.fused.n_train}
            for i, name in ((1, "train_acc"), (2, "val_acc"), (3, "test_acc")):
                cnt = int((m == i).sum())
                res[name] = float(c[i]) / cnt if cnt else float("nan")
            return res
        self.model.eval()
        pred = self.model(self.x, self.g).argmax(1)
        res = {}
        for name, k in (("train_acc", 1), ("val_acc", 2), ("test_acc", 3)):
            m = self.gd.mask == k
            res[name] = float((pred[m] == self.gd.y[m].long()).float().mean()) if bool(m.any()) else float("nan")
        return res


class ShardedGATTrainer:
    """Graph-sharded full-graph GAT (BASELINE config "ogbn-papers100M 2-layer GAT,
    graph sharded across 8 x 288 GB HBM").

    Rank r owns a contiguous block of rows: its CSR rows (global source ids), features,
    labels and every activation of those rows -- built by ``data.synthetic_shard``
    from rank-local generation (no rank ever holds the whole graph; 10^8 nodes and
    3.2 x 10^9 CSR entries at full size).  Per layer the source-side [Wh | s_src] rows
    a rank's edges read -- and only those -- arrive through one halo all-to-all
    (``parallel.halo``: bf16 activations + exact fp32 scores on the wire); the
    backward returns their gradients to the owners.  Parameters are replicated and
    their gradients averaged by the bucketed all-reduce; feature standardisation
    uses globally all-reduced moments, so for any rank count the model equals the
    single-GPU one (``tests/test_dist_cpu.py``).

    ``emulate=(rank, world)``: one rank of a larger job in a single process (the
    halo plan and buffers of that rank, received rows left zero) -- a memory /
    compute dry run of a full-size shard on one GPU, not a numerics run.
    """

    def __init__(self, shard, heads=8, head_dim=32, dropout=0.5, lr=0.005, seed=0, standardize=True,
                 bucket_mb: float = 16.0, emulate=None, fused: Optional[bool] = None,
                 halo_chunk_bytes: int = 4 << 30, train_rows_only: bool = True, train_halo: bool = True,
                 l1_exchange: bool = False, l1_train_neighbours: bool = True):
        # train_rows_only / train_halo / l1_train_neighbours: see gcn.GCNTrainer;
        # l1_exchange=True: exchange the layer-1 projections every epoch instead of the
        # input rows once at setup.  All must agree across ranks.
        import torch.distributed as dist
        from ..parallel import dist as pdist
        from ..parallel.ddp import GradBucketer
        from ..parallel.halo import HaloExchange
        from .data import GraphShard, shard_rows
        if not isinstance(shard, GraphShard):          # a full graph: take this rank's rows of it
            shard = shard_of(shard, pdist.rank(), pdist.world_size())
        self.emulate = emulate
        if emulate is not None:
            self.rank, self.world = int(emulate[0]), int(emulate[1])
        else:
            self.rank, self.world = pdist.rank(), pdist.world_size()
        self.dev = shard.rowptr.device
        self.n = shard.n
        r0, r1, per = shard_rows(shard.n, self.rank, self.world)
        if (r0, r1) != (shard.r0, shard.r1):
            raise ValueError("shard rows [%d, %d) are not rank %d/%d's block" % (shard.r0, shard.r1, self.rank,
                                                                                 self.world))
        self.r0, self.r1, self.per = r0, r1, per
        nloc = r1 - r0
        distributed = self.world > 1 and emulate is None
        self.halo = None
        if self.world > 1:
            # widest row on the wire: the fp32 layer gradients [dWh | ds_src] (exchange rounds
            # are sized so that one round moves at most halo_chunk_bytes of it)
            ow = (shard.n_classes + 7) // 8 * 8
            wide = 4 * max(heads * head_dim + heads, ow + 1)
            self.halo = HaloExchange(shard.col, r0, r1, per, shard.n, emulate=emulate, max_row_bytes=wide,
                                     chunk_bytes=halo_chunk_bytes)
            self.g = GraphCSR(shard.rowptr, self.halo.col_ext, nloc, n_cols=self.halo.n_ext)
        else:
            self.g = GraphCSR(shard.rowptr, shard.col, nloc, n_cols=shard.n)
        x = shard.x.float()
        if standardize:
            mom = torch.stack([x.sum(0), (x * x).sum(0)]).double()
            if distributed:
                dist.all_reduce(mom)
            mean = mom[0] / shard.n
            var = (mom[1] / shard.n - mean * mean) * shard.n / max(shard.n - 1, 1)
            x = ((x - mean.float()) / var.clamp_min(1e-12).sqrt().float().clamp_min(1e-6))
        self.x = x.contiguous()
        self.y = shard.y.long()
        self.mask = shard.mask
        self.tr = self.mask == 1
        n_train = torch.tensor([float(self.tr.sum())], dtype=torch.float64, device=self.dev)
        if distributed:
            dist.all_reduce(n_train)
        self.n_train = float(n_train.item()) if emulate is None else float(shard.n_train_global or n_train.item())
        self.ddp = None
        self.fused = None
        if _use_fused(fused, self.dev, x.shape[1], heads, head_dim, shard.n_classes):
            # the whole epoch on HIP kernels; one all-reduce of the flat gradient buffer
            from .gat_fused import FusedGAT
            train_l2 = None
            if self.world > 1 and train_rows_only and train_halo:
                train_l2 = self._train_halo(shard, r0, r1, per, emulate, wide, halo_chunk_bytes)
            # layer 1 without communication: its input rows are static, so the rows of the
            # layer-1 halo cross the links ONCE here (bf16), and every epoch each rank
            # projects [Wh | s_src] of the received rows itself (lin_fwd) and takes their
            # weight-gradient share as x_ext^T dy_ext -- per epoch only the layer-2 halo and
            # the weight all-reduce remain (l1_exchange=True: exchange per epoch).
            x_ext = None
            self.l1_setup_bytes = 0
            if self.halo is not None and not l1_exchange:
                F = self.x.shape[1]
                xb = torch.zeros(nloc, (F + 7) // 8 * 8, dtype=torch.bfloat16, device=self.dev)
                xb[:, :F] = self.x.to(torch.bfloat16)
                x_ext = self.halo.exchange_parts([xb])[0]
                self.l1_setup_bytes = self.halo.n_recv * xb.shape[1] * 2
                del xb
            self.fused = FusedGAT(self.x, self.y, self.mask, shard.n_classes, self.g, heads, head_dim, dropout, lr,
                                  seed, halo=self.halo, row0=r0, n_train=int(self.n_train), distributed=distributed,
                                  train_l2=train_l2, x_ext=x_ext, train_rows_only=train_rows_only,
                                  l1_train_neighbours=l1_train_neighbours,
                                  train_flag_fn=getattr(shard, "train_flags", None) if emulate is not None
                                  else None)
            self.model = self.opt = None
            self.epoch = 0
            return
        self.model = GAT(x.shape[1], shard.n_classes, heads, head_dim, dropout, seed).to(self.dev)
        self.opt = torch.optim.Adam(self.model.parameters(), lr=lr, fused=self.dev.type == "cuda")
        if distributed:
            self.ddp = GradBucketer(list(self.model.parameters()), bucket_mb)
            self.ddp.broadcast_parameters(0)
        self.epoch = 0

    def _train_halo(self, shard, r0, r1, per, emulate, wide, chunk):
        """Training epochs aggregate layer 2 at the train rows only (gat_fused), so they
        get a halo of their own: the remote rows those rows' edges read (papers100M
        shape: ~1 % train rows, so a small fraction of the full halo).  Collective: every
        rank builds it; a rank without train rows brings one placeholder row (non-train,
        its self edge only).  Returns (rows, CSR over the halo's row space, halo,
        placeholder) for ``FusedGAT(train_l2=...)``."""
        from ..parallel.halo import HaloExchange
        dev = self.dev
        trows = torch.nonzero(shard.mask == 1).flatten()
        placeholder = trows.numel() == 0
        rp = shard.rowptr.long()
        if placeholder:
            trows = torch.zeros(1, dtype=torch.int64, device=dev)
            trp = torch.tensor([0, 1], dtype=torch.int64, device=dev)
            tcol = torch.full((1,), r0, dtype=shard.col.dtype, device=dev)
        else:
            lo, deg = rp[trows], rp[trows + 1] - rp[trows]
            trp = torch.zeros(trows.numel() + 1, dtype=torch.int64, device=dev)
            trp[1:] = torch.cumsum(deg, 0)
            eid = torch.arange(int(trp[-1]), device=dev) + torch.repeat_interleave(lo - trp[:-1], deg)
            tcol = shard.col[eid]
        th = HaloExchange(tcol, r0, r1, per, shard.n, emulate=emulate, max_row_bytes=wide, chunk_bytes=chunk)
        gT = GraphCSR(trp.to(torch.int32), th.col_ext, trows.numel(), n_cols=th.n_ext)
        return trows, gT, th, placeholder
    def state_tensors(self):
        return _gat_state_tensors(self)

    def load_state_tensors(self, t):
        _gat_load_state_tensors(self, t)

    def halo_stats(self):
        """Rows / bytes this rank receives and sends per layer-1 exchange (Wh bf16 + fp32 scores)."""
        if self.halo is None:
            return {"recv_rows": 0, "send_rows": 0}
        l1 = self.fused.layers[0] if self.fused is not None else self.model.l1
        w = 2 * l1.K * l1.Fh + 4 * l1.K
        rb, sb = self.halo.bytes_per_exchange(w)
        local = self.fused is not None and self.fused.l1_local
        out = {"recv_rows": self.halo.n_recv, "send_rows": self.halo.n_send, "local_rows": self.halo.nloc,
               # per epoch (forward; the backward returns as many fp32 bytes): 0 when layer 1 is
               # projected locally from the setup-time input rows
               "layer1_recv_bytes": 0 if local else rb, "layer1_send_bytes": 0 if local else sb,
               "layer1_local": bool(local), "layer1_setup_recv_bytes": getattr(self, "l1_setup_bytes", 0)}
        tr = self.fused._tr if self.fused is not None else None
        if tr is not None and tr.halo is not None and tr.halo is not self.halo:
            out["layer2_train_recv_rows"] = tr.halo.n_recv    # the training epochs' layer-2 halo
            out["layer2_train_send_rows"] = tr.halo.n_send
        return out

    def train_step(self):
        if self.fused is not None:
            self.epoch += 1
            return self.fused.train_step()
        self.model.train()
        out = self.model(self.x, self.g, self.halo)
        # sum over this rank's train rows scaled so that the rank-average of the
        # gradients is the gradient of the global mean loss
        loss = torch.nn.functional.cross_entropy(out[self.tr], self.y[self.tr], reduction="sum")
        (loss * (self.world / self.n_train)).backward()
        if self.ddp is not None:
            self.ddp.finish()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.epoch += 1
        return loss.detach() / self.n_train        # this rank's share of the global mean loss

    @torch.no_grad()
    def evaluate(self):
        import torch.distributed as dist
        cnt = torch.zeros(6, dtype=torch.float64, device=self.dev)
        if self.fused is not None:
            c = self.fused.evaluate_counts().double()
            for i, k in enumerate((1, 2, 3)):
                cnt[2 * i] = c[k]
                cnt[2 * i + 1] = float((self.mask == k).sum())
        else:
            self.model.eval()
            pred = self.model(self.x, self.g, self.halo).argmax(1)
            for i, k in enumerate((1, 2, 3)):
                m = self.mask == k
                cnt[2 * i] = float((pred[m] == self.y[m]).sum())
                cnt[2 * i + 1] = float(m.sum())
        if self.world > 1 and self.emulate is None:
            dist.all_reduce(cnt)
        c = cnt.cpu().numpy()
        return {name: float(c[2 * i] / c[2 * i + 1]) if c[2 * i + 1] else float("nan")
                for i, name in enumerate(("train_acc", "val_acc", "test_acc"))}


def shard_of(gd: GraphData, rank: int, world: int):
    """This rank's rows of an in-memory graph as a ``GraphShard`` (tests / small graphs;
    large graphs are generated shard-locally by ``data.synthetic_shard``)."""
    from .data import GraphShard, shard_rows
    r0, r1, _ = shard_rows(gd.n, rank, world)
    rp = gd.rowptr[r0:r1 + 1].to(torch.int64)
    col = gd.col[int(rp[0]): int(rp[-1])]
    rp = (rp - rp[0]).to(torch.int32)
    return GraphShard(n=gd.n, r0=r0, r1=r1, rowptr=rp.contiguous(), col=col.contiguous(), x=gd.x[r0:r1],
                      y=gd.y[r0:r1], mask=gd.mask[r0:r1], n_classes=gd.n_classes,
                      n_train_global=int((gd.mask == 1).sum()), name=gd.name + "-shard%d/%d" % (rank, world))
