"""Fused GAT training epoch (GNN track, not in the reference): every dense op on
hand-written HIP kernels, no autograd, no hipBLASLt, no ATen elementwise chain.

Per layer (``gat.GATLayer`` semantics; the attention logits are linear in the
input, so they fold into the projection ``Wc = [W | W a_src | W a_dst]``):

  forward   [Wh | s_src | s_dst] = h Wc       lin_fwd (MFMA), Wh stored bf16 (the
                                              edge-gathered operand), the scores as
                                              exact fp32 planes (its ``tail`` output)
            out, lse, q = GAT aggregation     gat_fwd (online softmax); q is the
                                              LeakyReLU split that makes the row half
                                              of the backward a per-row product;
                                              layer 1 also writes h1 = bf16(dropout(
                                              elu(out + b1))) in the same kernel
            layer 2: loss, dlogits = CE(out + b2) (train rows) gat_row_ce
                      (training epochs aggregate layer 2 at the train rows only:
                      no other row's logits reach the loss -- exact)
  backward  row half (per row, no gather)     gat_rows: D = <dout, out>,
                                              d s_dst = -0.8 <dout, q>; for layer 1
                                              fused with the activation backward
                                              (dout1 = dh1 * mask * elu', db1)
            column half                       gat_col over the transposed CSR:
                                              dy = bf16([dWh | ds_src | ds_dst]) written
                                              in place (the GEMM operand)
            dWc = h^T dy                      lin_bwd_weight (split-K MFMA, fixed order)
            dh = dy Wc^T                      lin_bwd_data (MFMA; layer 2 only)
            dW, da_src, da_dst from dWc       (weight-sized tensors only)
  update    gradients summed over ranks (one all-reduce of the flat buffer), Adam
            on the flat fp32 parameter buffer (ops.adam_).

Graph-sharded runs (``halo``): layer 1 is communication-free when the trainer passes
``x_ext`` -- the static input rows of this rank's layer-1 halo, fetched once at setup --
so each rank projects ``[Wh | s_src]`` of the received rows itself and takes their
weight-gradient share as ``x_ext^T dy_ext``; only the layer-2 (training) halo moves per
epoch, plus the weight all-reduce.

Dropout is keyed by (seed, GLOBAL row, column, device step counter), so a
sharded run draws exactly the masks of a one-GPU run; together with the
rank-independent loss scale (1 / global train count) the model is the same for
any rank count.  Every op has a CPU branch (the fp32 reference of the same
bf16-stored arithmetic), so the sharded path is tested with gloo ranks on CPU.
"""
from __future__ import annotations

import math
import types
from typing import Optional

import torch

from .. import native
from ..utils.philox import model_key
from . import ops
from .linear import lin_bwd_data, lin_bwd_weight, lin_fwd


def _st(t):
    return torch._C._cuda_getCurrentRawStream(t.get_device())


def _ru8(x):
    return (x + 7) // 8 * 8


def _ptr(t):
    return t.data_ptr() if t is not None else 0


# ------------------------------------------------------------------ elementwise ops
def act_fwd(out, bias, H, p, key, step, row0=0):
    """H[:, :F] = bf16(dropout(elu(out + bias))), F = out.shape[1] (a multiple of 32).
    CPU reference: on a GPU this runs inside the layer's aggregation kernel (gat_fwd)."""
    if out.is_cuda:
        raise RuntimeError("act_fwd is the CPU reference; the GPU fuses it into gat_fwd (_agg_fwd act=...)")
    n, F = out.shape
    z = out.float() + bias.float()
    e = torch.where(z > 0, z, torch.expm1(z))
    if p > 0:
        keep = ops.dropout_keep_mask(n, F, p, key, ops._step_value(step), row0)
        e = torch.where(keep, e / (1 - p), torch.zeros_like(e))
    H[:n, :F] = e.to(H.dtype)
    return H


_BPART = {}


def _scratch(dev, shape):
    key = (dev.type, dev.index, tuple(shape))
    buf = _BPART.get(key)
    if buf is None:
        buf = _BPART[key] = torch.empty(shape, dtype=torch.float32, device=dev)
    return buf


def act_bwd(dH, out, bias, p, key, step, row0, dout, doutb, db):
    """dout = dH * mask * elu'(out + bias) (fp32, plus a bf16 copy ``doutb``), db = colsum(dout).
    CPU reference: on a GPU this runs inside the row half of the backward (gat_rows)."""
    if out.is_cuda:
        raise RuntimeError("act_bwd is the CPU reference; the GPU fuses it into gat_rows (_agg_rows act=...)")
    n, F = out.shape
    z = out.float() + bias.float()
    d = dH[:n, :F].float() * torch.where(z > 0, torch.ones_like(z), torch.exp(z))
    if p > 0:
        keep = ops.dropout_keep_mask(n, F, p, key, ops._step_value(step), row0)
        d = torch.where(keep, d / (1 - p), torch.zeros_like(d))
    dout.copy_(d)
    if doutb is not None:
        doutb.copy_(d.to(torch.bfloat16))
    db.copy_(d.sum(0))
    return dout


def row_ce(Z, bias, C, y, mask, inv_count, dZ=None, dZb=None, db=None):
    """Cross-entropy of logits ``Z[:, :C] + bias`` on the train rows (mask == 1).
    Returns [4] fp32 (sum of train NLL, correct train / valid / test); training
    (``dZ`` given): dZ = (softmax - onehot) * inv_count on train rows, 0 elsewhere
    (pad columns too), ``dZb`` its bf16 copy, ``db`` = colsum(dZ)."""
    n, ldz = Z.shape
    if Z.is_cuda:
        hip = native.hip()
        nw = hip.gnn_gat_row_ce_waves()
        spart = _scratch(Z.device, (nw, 4))
        bpart = _scratch(Z.device, (nw, C))
        stats = torch.empty(4, dtype=torch.float32, device=Z.device)
        hip.gnn_gat_row_ce(Z.data_ptr(), ldz, bias.data_ptr(), C, y.data_ptr(), mask.data_ptr(), float(inv_count),
                           _ptr(dZ), _ptr(dZb), spart.data_ptr(), bpart.data_ptr(), stats.data_ptr(), _ptr(db), n,
                           _st(Z))
        return stats
    logits = Z[:, :C].float() + bias[:C].float()
    lse = torch.logsumexp(logits, 1)
    yl = y.long()
    zy = logits.gather(1, yl[:, None])[:, 0]
    tr = mask == 1
    pred = logits.argmax(1)
    ok = pred == yl
    stats = torch.stack([(lse - zy)[tr].sum(), ok[tr].sum().float(), ok[mask == 2].sum().float(),
                         ok[mask == 3].sum().float()]).float()
    if dZ is not None or dZb is not None:
        d = torch.softmax(logits, 1)
        d[torch.arange(n), yl] -= 1.0
        d = torch.where(tr[:, None], d * inv_count, torch.zeros_like(d))
        full = torch.zeros(n, ldz, dtype=torch.float32)
        full[:, :C] = d
        if dZ is not None:
            dZ.copy_(full)
        if dZb is not None:
            dZb.copy_(full.to(torch.bfloat16))
        if db is not None:
            db[:C].copy_(d.sum(0))
    return stats


def pack_grad(dWh, ds_src, ds_dst, dy):
    """dy[:, :HF + 2K] = bf16([dWh | ds_src | ds_dst]), zero pad columns."""
    n, HF = dWh.shape
    K = ds_src.shape[1]
    if dWh.is_cuda:
        native.hip().gnn_gat_pack_grad(dWh.data_ptr(), ds_src.data_ptr(), ds_dst.data_ptr(), HF, K, dy.data_ptr(),
                                       dy.stride(0), n, _st(dWh))
        return dy
    dy.zero_()
    dy[:n, :HF + 2 * K] = torch.cat([dWh.float(), ds_src.float(), ds_dst.float()], 1).to(dy.dtype)
    return dy


# ------------------------------------------------------------------ aggregation
def _check_rows(g, Wh, s_src, s_dst, dst_rows, what):
    from .gat import _check_graph
    from ..utils import checks
    _check_graph(g, Wh, s_src, s_dst, what)
    if dst_rows is not None and checks.enabled():
        checks.rows(dst_rows, g.n, what + " dst_rows")
        checks.index(dst_rows, s_dst.shape[0], what + " dst_rows")


def _agg_fwd(Wh, s_src, s_dst, g, K, Fh, dst_rows=None, q=None, act=None):
    """out [g.n, K Fh] fp32, lse [g.n, K]: attention aggregation over ``g``; the
    destination scores of row i are ``s_dst[dst_rows[i]]`` (or ``s_dst[i]``).  GPU
    extras: ``q`` (training) receives the LeakyReLU split for the row backward;
    ``act = (bias, H, p, key, step, row0)`` writes the hidden activation
    ``H = bf16(dropout(elu(out + bias)))`` in the same kernel."""
    _check_rows(g, Wh, s_src, s_dst, dst_rows, "fused gat_fwd")
    n = g.n
    if Wh.is_cuda:
        out = torch.empty(n, K * Fh, dtype=torch.float32, device=Wh.device)
        lse = torch.empty(n, K, dtype=torch.float32, device=Wh.device)
        kw = {}
        if act is not None:
            bias, H, p, key, step, row0 = act
            sv, sp = ops._step_args(step)
            kw = dict(bias=bias.data_ptr(), H=H.data_ptr(), ldh=H.stride(0), p=float(p), k0=int(key[0]),
                      k1=int(key[1]), step=sv, stepp=sp, row0=int(row0))
        native.hip().gnn_gat_fwd(g.rowptr.data_ptr(), g.col.data_ptr(), Wh.data_ptr(), s_src.data_ptr(),
                                 s_dst.data_ptr(), out.data_ptr(), lse.data_ptr(), n, K, Fh, _st(Wh),
                                 int(Wh.dtype == torch.bfloat16), dst_rows=_ptr(dst_rows), q=_ptr(q), **kw)
        return out, lse
    from .gat import _gat_aggregate_torch
    sd = s_dst if dst_rows is None else s_dst.index_select(0, dst_rows.long())
    return _gat_aggregate_torch(Wh.float(), s_src, sd, g, K, Fh).float(), None


def _agg_rows(out, q, lse, s_dst, dst_rows, K, Fh, rstat, dout=None, dH=None, act=None, ds_dst=None, dy=None):
    """Row half of the aggregation backward (GPU, no gather): rstat [n, K, 4] =
    (s_dst, lse, D, 0) per (row, head), d s_dst = -0.8 <dout, q> into ``ds_dst`` (fp32
    [*, K]) and / or column HF + K + k of ``dy`` (bf16, row dst_rows[i] or i).  Either
    ``dout`` (bf16) is given, or ``dH`` with ``act = (dout_w, bias, db, p, key, step,
    row0)``: dout = dH * mask * elu'(out + bias) is made here, written to ``dout_w``
    (bf16), and db = colsum(dout)."""
    n = out.shape[0]
    hip = native.hip()
    kw = dict(dout_w=0, bias=0, bpart=0, db=0, p=0.0, k0=0, k1=0, step=0, stepp=0, row0=0)
    if act is not None:
        dout_w, bias, db, p, key, step, row0 = act
        sv, sp = ops._step_args(step)
        bpart = _scratch(out.device, (hip.gnn_gat_row_blocks(), K * Fh))
        kw = dict(dout_w=dout_w.data_ptr(), bias=bias.data_ptr(), bpart=bpart.data_ptr(), db=db.data_ptr(),
                  p=float(p), k0=int(key[0]), k1=int(key[1]), step=sv, stepp=sp, row0=int(row0))
        src, ldh = dH, dH.stride(0)
    else:
        src, ldh = dout, 0
    hip.gnn_gat_rows(int(act is not None), src.data_ptr(), ldh, out.data_ptr(), q.data_ptr(), lse.data_ptr(),
                     s_dst.data_ptr(), _ptr(dst_rows), rstat.data_ptr(), _ptr(ds_dst), _ptr(dy),
                     dy.stride(0) if dy is not None else 0, n=n, K=K, Fh=Fh, wbf=1, st=_st(out), **kw)


def _agg_cols(Wh, s_src, rstat, doutb, g, K, Fh, lo, hi, dWh=None, ds_src=None, dy=None):
    """Column half for source rows [lo, hi) of the transposed CSR (rows are independent,
    so a row range is a pointer offset): fp32 ``dWh`` [hi - lo, K Fh] / ``ds_src`` [hi - lo,
    K], or bf16 [dWh | ds_src] straight into ``dy`` rows [lo, hi) (GPU)."""
    rp_t, col_t = g.transposed()
    KF = K * Fh
    dyp = dy.data_ptr() + dy.element_size() * dy.stride(0) * lo if dy is not None else 0
    native.hip().gnn_gat_col(rp_t.data_ptr() + 4 * lo, col_t.data_ptr(), Wh.data_ptr() + Wh.element_size() * KF * lo,
                             s_src.data_ptr() + 4 * K * lo, rstat.data_ptr(), doutb.data_ptr(), _ptr(dWh),
                             _ptr(ds_src), dyp, dy.stride(0) if dy is not None else 0, hi - lo, K, Fh, _st(doutb), 1)


def _agg_bwd_torch(Wh, s_src, s_dst, dout, g, K, Fh):
    from .gat import _gat_aggregate_torch
    with torch.enable_grad():
        a = Wh.float().detach().requires_grad_()
        b = s_src.detach().requires_grad_()
        c = s_dst.detach().requires_grad_()
        o = _gat_aggregate_torch(a, b, c, g, K, Fh)
        return torch.autograd.grad(o, (a, b, c), dout)


def wcat(W, a_src, a_dst, out):
    """out = [W | W a_src | W a_dst] (per head: sum over the head's columns)."""
    K, Fh = a_src.shape
    Wk = W.view(-1, K, Fh)
    torch.cat([W, (Wk * a_src).sum(-1), (Wk * a_dst).sum(-1)], 1, out=out)
    return out


def wcat_bwd(dWc, W, a_src, a_dst, gW, ga_src, ga_dst):
    K, Fh = a_src.shape
    KF = K * Fh
    Wk = W.view(-1, K, Fh)
    ds, dd = dWc[:, KF:KF + K, None], dWc[:, KF + K:KF + 2 * K, None]
    gW.copy_(dWc[:, :KF] + (ds * a_src + dd * a_dst).reshape(-1, KF))
    ga_src.copy_((Wk * ds).sum(0))
    ga_dst.copy_((Wk * dd).sum(0))


class _Layer:
    tr = None                 # the train-row CSR of the last training forward, if any


class FusedGAT:
    """The fused 2-layer GAT epoch over one rank's rows (the whole graph when
    ``halo`` is None).  ``g``: GraphCSR over [own | received] source rows;
    ``x``: fp32 [nloc, F] input features (already standardised); ``row0``: the
    global id of the first own row (dropout keys); ``n_train``: GLOBAL train count.
    ``x_ext`` (sharded, optional): bf16 [n_ext, >= F] input rows of [own | received]
    (the layer-1 halo's static features): layer 1 then projects every row it reads
    itself and needs no exchange.
    Parameters are initialised exactly like ``gat.GAT(F, C, heads, head_dim, seed)``."""

    def __init__(self, x, y, mask, n_classes, g, heads=8, head_dim=32, dropout=0.5, lr=0.005, seed=0,
                 halo=None, row0=0, n_train=None, distributed=False, train_l2=None, x_ext=None,
                 train_rows_only: bool = True, l1_train_neighbours: bool = True, train_flag_fn=None):
        from .gat import GAT
        dev = x.device
        self.dev, self.g, self.halo = dev, g, halo
        self.nloc, self.F = x.shape
        self.C = int(n_classes)
        self.p, self.lr = float(dropout), float(lr)
        self.row0, self.distributed = int(row0), bool(distributed)
        self.y = y.to(torch.int32).contiguous()
        self.mask = mask.to(torch.uint8).contiguous()
        if n_train is None:
            n_train = int((self.mask == 1).sum())
        self.n_train = max(int(n_train), 1)
        bf = dict(dtype=torch.bfloat16, device=dev)
        if x_ext is not None:
            if halo is None or x_ext.shape[0] != halo.n_ext or x_ext.dtype != torch.bfloat16:
                raise ValueError("x_ext must be bf16 [halo.n_ext, >= F] rows of [own | received]")
            self.xb = x_ext
        else:
            self.xb = torch.zeros(self.nloc, _ru8(self.F), **bf)
            self.xb[:, :self.F] = x.to(torch.bfloat16)
        self.l1_local = x_ext is not None
        ref = GAT(self.F, self.C, heads, head_dim, dropout, seed)          # the init of the autograd model
        mods = [ref.l1, ref.l2]
        flat = torch.cat([t.detach().reshape(-1) for m in mods for t in (m.W, m.a_src, m.a_dst, m.bias)])
        self.params = flat.to(dev)
        self.grads = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.key = model_key(seed, "gat-dropout")
        if self.distributed:
            # replicas start from rank 0's parameters and dropout key
            kt = torch.tensor([int(self.key[0]), int(self.key[1])], dtype=torch.int64, device=dev)
            torch.distributed.broadcast(self.params, 0)
            torch.distributed.broadcast(kt, 0)
            self.key = (int(kt[0]), int(kt[1]))
        off = 0
        self.layers = []
        kin = self.F
        for li, m in enumerate(mods):
            L = _Layer()
            L.K, L.Fh = m.K, m.Fh
            L.KF = L.K * L.Fh
            L.Kin = kin
            views = []
            for t in (m.W, m.a_src, m.a_dst, m.bias):
                k = t.numel()
                views.append((self.params[off:off + k].view(t.shape), self.grads[off:off + k].view(t.shape)))
                off += k
            (L.W, L.gW), (L.a_src, L.ga_src), (L.a_dst, L.ga_dst), (L.b, L.gb) = views
            L.N = L.KF + 2 * L.K
            L.Wc = torch.zeros(kin, L.N, dtype=torch.float32, device=dev)
            L.dWc = torch.zeros_like(L.Wc)
            L.db_scratch = torch.zeros(L.N, dtype=torch.float32, device=dev)
            # layer 1 with local projection: every [own | received] row is projected here
            rows = self.xb.shape[0] if (li == 0 and self.l1_local) else self.nloc
            L.local = li == 0 and self.l1_local
            L.Wh = torch.zeros(rows, L.KF, **bf)
            L.s = torch.zeros(2, rows, L.K, dtype=torch.float32, device=dev)
            L.dy = torch.zeros(rows, _ru8(L.N), **bf)
            self.layers.append(L)
            kin = L.KF
        L1, L2 = self.layers
        self.h1 = torch.zeros(self.nloc, L1.KF, **bf)
        self.dh1 = torch.zeros(self.nloc, L1.KF, **bf)
        self.dout1b = torch.zeros(self.nloc, L1.KF, **bf)
        self.dout1 = torch.zeros(self.nloc, L1.KF, dtype=torch.float32, device=dev) if dev.type != "cuda" else None
        self.dout2 = torch.zeros(self.nloc, L2.KF, dtype=torch.float32, device=dev)
        self.dout2b = torch.zeros(self.nloc, L2.KF, **bf)
        # Training epochs aggregate layer 2 only at this rank's train rows (the only
        # logits the loss reads; the epoch's update is unchanged -- the output-node
        # pruning of DGL's last block): a CSR of those rows over the same sources.
        # Evaluation aggregates every row (train_rows_only=False: every row always).
        self._tr = None
        trows = torch.nonzero(self.mask == 1).flatten()
        if train_l2 is not None:
            # built by the sharded trainer: the train rows' CSR over a training halo of
            # its own (only the remote rows those rows read travel in training epochs);
            # a rank without train rows brings a non-train placeholder row
            trows, gT, thalo, placeholder = train_l2
            nT = trows.numel()
            self._tr = types.SimpleNamespace(
                rows=trows, rows32=trows.to(torch.int32).contiguous(), g=gT, halo=thalo, y=self.y[trows].contiguous(),
                mask=torch.zeros_like(self.mask[trows]) if placeholder else self.mask[trows].contiguous(),
                dout=torch.zeros(nT, L2.KF, dtype=torch.float32, device=dev),
                doutb=torch.zeros(nT, L2.KF, **bf))
            self.dout2 = self.dout2b = None
        elif trows.numel() and train_rows_only:
            from .gat import GraphCSR
            rp = g.rowptr.long()
            lo, deg = rp[trows], rp[trows + 1] - rp[trows]
            trp = torch.zeros(trows.numel() + 1, dtype=torch.int64, device=dev)
            trp[1:] = torch.cumsum(deg, 0)
            eid = torch.arange(int(trp[-1]), device=dev) + torch.repeat_interleave(lo - trp[:-1], deg)
            nT = trows.numel()
            self._tr = types.SimpleNamespace(
                rows=trows, rows32=trows.to(torch.int32).contiguous(),
                g=GraphCSR(trp.to(g.rowptr.dtype), g.col[eid], nT, g.n_cols), halo=halo,
                y=self.y[trows].contiguous(), mask=self.mask[trows].contiguous(),
                dout=torch.zeros(nT, L2.KF, dtype=torch.float32, device=dev),
                doutb=torch.zeros(nT, L2.KF, **bf))
            self.dout2 = self.dout2b = None          # all-row layer-2 gradients: not needed
        # ... and then layer 1 is needed only at the rows those aggregations read: the
        # rows with a train neighbour (any rank's; A is symmetric; the neighbours' train
        # flags come over the halo once).  Training epochs aggregate layer 1 over a CSR
        # whose other rows are empty (they produce out = 0, finite, read by no train row,
        # with zero gradient); evaluation aggregates every row.  The papers100M shape has
        # ~1 % train rows, so most layer-1 edges drop out.  In a dry run (emulated halo)
        # the received rows' flags come from ``train_flag_fn`` (the deterministic split of
        # any global row); without one the pruning is off.  l1_train_neighbours=False: off.
        # The decision is the same on every rank whenever there is a halo (the flag
        # exchange is collective): a rank without train rows still takes part.
        self._g1 = None
        want = (halo is not None) or (self._tr is not None)
        emulated = halo is not None and getattr(halo, "emulate", False)
        if want and l1_train_neighbours and (not emulated or train_flag_fn is not None):
            self._g1 = self._train_neighbour_graph(g, halo, train_flag_fn if emulated else None)
        self.epoch = 0
        self.last_stats = None

    def _train_neighbour_graph(self, g, halo, flag_fn=None):
        from .gat import GraphCSR
        flag = (self.mask == 1).to(torch.float32)[:, None].contiguous()
        if flag_fn is not None:                            # emulated halo: flags generated locally
            rec = flag_fn(halo.received_ids()).to(torch.float32)[:, None]
            flag = torch.cat([flag, rec.to(flag.device)], 0).contiguous()
        elif halo is not None:
            flag = halo.exchange_parts([flag])[0]          # [own | received] train flags
        tflag = flag[:, 0] > 0.5
        rp, col = g.rowptr.long(), g.col.long()
        deg = rp[1:] - rp[:-1]
        rows = torch.repeat_interleave(torch.arange(g.n, device=col.device), deg)
        hit = torch.zeros(g.n, dtype=torch.bool, device=col.device)
        hit[rows[tflag[col]]] = True
        keep = hit[rows]
        del rows
        nrp = torch.zeros(g.n + 1, dtype=torch.int64, device=col.device)
        nrp[1:] = torch.cumsum(torch.where(hit, deg, torch.zeros_like(deg)), 0)
        return GraphCSR(nrp.to(g.rowptr.dtype), g.col[keep], g.n, g.n_cols)

    @staticmethod
    def supported(F, heads, head_dim, n_classes):
        ow = _ru8(n_classes)
        g1 = head_dim // 8
        return (head_dim % 8 == 0 and (heads == 1 or (g1 & (g1 - 1)) == 0) and heads * head_dim <= 512
                and (heads * head_dim) % 32 == 0 and ow <= 256 and F <= 512)

    def _dropout_step(self):
        return self.step_t if self.dev.type == "cuda" else int(self.step_t.item())

    # ------------------------------------------------------------------ passes
    def _project_aggregate(self, L, x, K1, train, tr=None, g1=None, act=None):
        """Projection + attention aggregation; ``tr`` (train-row CSR): only at those rows;
        ``g1``: the aggregation graph instead of the full one (same rows); ``act``: the
        fused hidden activation (GPU)."""
        wcat(L.W, L.a_src, L.a_dst, L.Wc)
        lin_fwd(x, L.Wc, None, K1=K1, out=L.Wh, tail=L.s, nsplit=L.KF, tk=L.K)
        s_src, s_dst = L.s[0], L.s[1]
        halo = None if L.local else (self.halo if tr is None else tr.halo)
        if halo is not None:
            Wh_ext, s_ext = halo.exchange_parts([L.Wh, s_src])
        else:
            Wh_ext, s_ext = L.Wh, s_src
        g = self.g if g1 is None else g1
        dst_rows = None
        if tr is not None:
            g, dst_rows = tr.g, (tr.rows32 if self.dev.type == "cuda" else tr.rows)
        q = None
        if train and self.dev.type == "cuda":
            q = torch.empty(g.n, L.KF, dtype=torch.bfloat16, device=self.dev)
        out, lse = _agg_fwd(Wh_ext, s_ext, s_dst, g, L.K, L.Fh, dst_rows=dst_rows, q=q,
                            act=act if self.dev.type == "cuda" else None)
        L.saved = (Wh_ext, s_ext, s_dst, dst_rows, out, lse, q)
        L.tr, L.g_used = tr, g
        return out

    def forward(self, train: bool):
        L1, L2 = self.layers
        p = self.p if train else 0.0
        step = self._dropout_step()
        act = (L1.b, self.h1, p, self.key, step, self.row0)
        out1 = self._project_aggregate(L1, self.xb, self.F, train, g1=self._g1 if train else None, act=act)
        if self.dev.type != "cuda":
            act_fwd(out1, L1.b, self.h1, p, self.key, step, self.row0)
        tr = self._tr if train else None
        out2 = self._project_aggregate(L2, self.h1, L1.KF, train, tr)
        if tr is not None:
            stats = row_ce(out2, L2.b, self.C, tr.y, tr.mask, 1.0 / self.n_train, dZ=tr.dout,
                           dZb=tr.doutb, db=L2.gb)
        elif train:
            stats = row_ce(out2, L2.b, self.C, self.y, self.mask, 1.0 / self.n_train, dZ=self.dout2,
                           dZb=self.dout2b, db=L2.gb)
        else:
            stats = row_ce(out2, L2.b, self.C, self.y, self.mask, 1.0 / self.n_train)
        if not train:
            for L in self.layers:
                L.saved = None
        return stats

    def _layer_backward(self, L, dout, doutb, x, K1, act=None):
        """``dout`` fp32 (CPU) / ``doutb`` bf16 (GPU) gradient of the aggregation output;
        GPU layer 1: ``doutb`` is None and ``act = (dH, bias, db)`` -- the activation
        backward runs inside the row half."""
        Wh_ext, s_ext, s_dst, dst_rows, out, lse, q = L.saved
        L.saved = None
        tr, L.tr = L.tr, None
        g, K, Fh = L.g_used, L.K, L.Fh
        halo = None if L.local else (self.halo if tr is None else tr.halo)
        if not self.dev.type == "cuda":
            sd = s_dst if dst_rows is None else s_dst.index_select(0, dst_rows)
            dWh, ds_src, ds_dst = _agg_bwd_torch(Wh_ext, s_ext, sd, dout, g, K, Fh)
            del Wh_ext, s_ext
            if halo is not None:
                dWh, ds_src = halo.reduce_back([dWh, ds_src])
            if tr is not None or ds_dst.shape[0] != dWh.shape[0]:
                # the other rows' destination-score gradients are 0 (rows outside the train
                # CSR; the received rows of a locally projected layer 1)
                full = torch.zeros(dWh.shape[0], K, dtype=ds_dst.dtype, device=ds_dst.device)
                if tr is not None:
                    full.index_copy_(0, tr.rows, ds_dst)
                else:
                    full[:ds_dst.shape[0]] = ds_dst
                ds_dst = full
            pack_grad(dWh, ds_src, ds_dst, L.dy)
            del dWh, ds_src, ds_dst
        else:
            rstat = torch.empty(g.n, K, 4, dtype=torch.float32, device=self.dev)
            rargs = {}
            if act is not None:
                dH, bias, db = act
                doutb = self.dout1b
                rargs = dict(dH=dH, act=(doutb, bias, db, self.p, self.key, self._dropout_step(), self.row0))
            else:
                rargs = dict(dout=doutb)
            if halo is None:
                # dy written in place: [dWh | ds_src] by the column half, ds_dst by the row half
                _agg_rows(out, q, lse, s_dst, dst_rows, K, Fh, rstat, dy=L.dy, **rargs)
                _agg_cols(Wh_ext, s_ext, rstat, doutb, g, K, Fh, 0, g.n_cols, dy=L.dy)
            else:
                n = self.nloc
                ds_dst = torch.zeros(n, K, dtype=torch.float32, device=self.dev)
                _agg_rows(out, q, lse, s_dst, dst_rows, K, Fh, rstat, ds_dst=ds_dst, **rargs)
                dWh = torch.empty(n, L.KF, dtype=torch.float32, device=self.dev)
                ds_src = torch.empty(n, K, dtype=torch.float32, device=self.dev)
                _agg_cols(Wh_ext, s_ext, rstat, doutb, g, K, Fh, 0, n, dWh=dWh, ds_src=ds_src)

                # the received rows' gradients are made one exchange round at a time
                def produce(lo, hi):
                    a = torch.empty(hi - lo, L.KF, dtype=torch.float32, device=self.dev)
                    b = torch.empty(hi - lo, K, dtype=torch.float32, device=self.dev)
                    _agg_cols(Wh_ext, s_ext, rstat, doutb, g, K, Fh, lo, hi, dWh=a, ds_src=b)
                    return [a, b]
                halo.reduce_back_stream(produce, [dWh, ds_src], getattr(self.halo, "grad_wire", torch.float32))
                pack_grad(dWh, ds_src, ds_dst, L.dy)
                del dWh, ds_src, ds_dst
            del rstat, Wh_ext, s_ext, q
        lin_bwd_weight(x, L.dy, L.N, K1=K1, dW=L.dWc, db=L.db_scratch)
        wcat_bwd(L.dWc, L.W, L.a_src, L.a_dst, L.gW, L.ga_src, L.ga_dst)

    def backward(self):
        L1, L2 = self.layers
        out1 = L1.saved[4]
        tr = L2.tr
        if tr is not None:
            self._layer_backward(L2, tr.dout, tr.doutb, self.h1, L1.KF)
        else:
            self._layer_backward(L2, self.dout2, self.dout2b, self.h1, L1.KF)
        lin_bwd_data(L2.dy, L2.Wc, L1.KF, out1=self.dh1)
        if self.dev.type == "cuda":
            self._layer_backward(L1, None, None, self.xb, self.F, act=(self.dh1, L1.b, L1.gb))
        else:
            act_bwd(self.dh1, out1, L1.b, self.p, self.key, self._dropout_step(), self.row0, self.dout1,
                    self.dout1b, L1.gb)
            self._layer_backward(L1, self.dout1, self.dout1b, self.xb, self.F)

    def train_step(self):
        stats = self.forward(train=True)
        self.backward()
        if self.distributed:
            torch.distributed.all_reduce(self.grads)
        ops.adam_(self.params, self.grads, self.m, self.v, self.lr, self.step_t)
        self.last_stats = stats
        self.epoch += 1
        return stats[0] / self.n_train          # this rank's share of the global mean loss

    @torch.no_grad()
    def evaluate_counts(self):
        """[4] = (train NLL sum, correct train / valid / test) of this rank's rows."""
        return self.forward(train=False)

    def state_tensors(self):
        return {"params": self.params, "adam_m": self.m, "adam_v": self.v, "adam_step": self.step_t}

    def load_state_tensors(self, t):
        for name, dst in (("params", self.params), ("adam_m", self.m), ("adam_v", self.v),
                          ("adam_step", self.step_t)):
            if t[name].shape != dst.shape:
                raise ValueError("checkpoint %s has shape %s, trainer %s" % (name, tuple(t[name].shape),
                                                                              tuple(dst.shape)))
            dst.copy_(t[name].to(dst.device))

    def to_module(self):
        """The parameters as a ``gat.GAT`` module (CPU), e.g. for the autograd reference."""
        from .gat import GAT
        L1, L2 = self.layers
        m = GAT(self.F, self.C, L1.K, L1.Fh, self.p, 0)
        with torch.no_grad():
            for mod, L in ((m.l1, L1), (m.l2, L2)):
                mod.W.copy_(L.W.cpu())
                mod.a_src.copy_(L.a_src.cpu())
                mod.a_dst.copy_(L.a_dst.cpu())
                mod.bias.copy_(L.b.cpu())
        return m
