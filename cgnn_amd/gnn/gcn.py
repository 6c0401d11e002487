"""Full-graph GCN training on MI355X (GNN track, not in the reference).

Model (Kipf & Welling): ``logits = Â · (dropout(relu(Â X W1 + b1)) W2) + b2``
with ``Â = D^-1/2 (A+I) D^-1/2``, softmax cross-entropy on the train split,
Adam.  Storage bf16, accumulation fp32, master weights fp32.

One epoch = one full-graph forward + backward + optimizer step:

  1. AX   = spmm(Xs)                       Xs = D^-1/2 X  (normalised once, like a cached Â)
  2. H1   = dropout(relu(AX W1 + b1))      } one fused MFMA kernel (gnn_dense.hip): both GEMMs,
  3. Z2   = D^-1/2 (H1 W2)                 } bias, ReLU, Philox dropout, row scale; Z2 all-gathered
  4. loss, G = spmm_ce(Z2)                 aggregate + bias + log-softmax + NLL + dlogits, fused;
                                           in training only at the train rows (8 % of
                                           ogbn-products): no other row's logits reach the
                                           loss; evaluation aggregates every row.
                                           G is stored COMPACT: dL/dlogits is zero outside
                                           the train rows, so only train rows are written,
                                           to slots 0..T-1
  5. dY2  = D^-1/2 spmm_T(G)               Â symmetric; spmm_T runs over the train COLUMNS
                                           of the adjacency only (a CSR built once: 9.5 M
                                           of the 118 M entries) -- the same sums, without
                                           the 92 % of gathers that would read zero rows
  6. dH1 = dY2 W2^T, relu/dropout backward (fused); the weight gradients
     dW2 = H1^T dY2 and [dW1; db1] = [AX | 1]^T dP1 are contractions over millions
     of rows with tiny outputs, so they run as split-K batched GEMMs (row chunks
     of CHUNK rows -> one fp32 partial per chunk -> fixed-order sum); db1 comes
     for free from the ones column the layer-1 SpMM writes next to AX
  7. gradients all-reduced (RCCL), fused Adam

Multi-GPU: each rank owns a contiguous block of rows (1-D partition); the
static features are replicated (0.5 GB for ogbn-products, trivial against
288 GB of HBM), so layer 1 needs no communication.  Layer 2 in training: the
rank aggregates only its train rows, and only the remote Z2 rows THOSE read
travel -- a training halo negotiated once at setup, one all-to-all per epoch
(``_train_row_csr``; ``train_halo=False`` uses the evaluation's exchange).
Evaluation aggregates every row, with the full halo from 4 ranks on (``halo``)
and an all-gather of Z2 below that.  The backward all-gathers the compact G (train
rows only, padded to the largest rank's count: 1/12 of Z2's bytes), plus one
all-reduce of the ~40k gradient floats.  In training both exchanges run
asynchronously on RCCL's stream beside one half each of the next epoch's layer-1
SpMM (parameter-independent; rows [0, n/2) beside the forward's halo exchange,
[n/2, n) beside the backward's all-gather), and each aggregation that needs them
is then ONE pass: layer 2 over [Z2 rows | received rows] in one buffer, the
backward over the whole train-column ELL image.  (Evaluation keeps the split
local / remote aggregation through an fp32 partial.)
"""
from __future__ import annotations

import math
import types
from typing import Optional

import numpy as np
import torch

from ..parallel import dist as pdist
from ..utils.philox import model_key
from . import ops
from .data import GraphData, partition_rows


def _ru8(x):
    return (x + 7) // 8 * 8


def _ru(x, m):
    return (x + m - 1) // m * m


def _mm_f32(a, b):
    """bf16 x bf16 -> fp32 output (fp32 accumulation)."""
    if a.is_cuda:
        return torch.mm(a, b, out_dtype=torch.float32)
    return a.float() @ b.float()


CHUNK = 8192


def _tsgemm(A, B, chunk=CHUNK):
    """A^T B for tall A [M, k1], B [M, k2] (M a multiple of ``chunk``): split-K over
    row chunks as one batched GEMM with fp32 partials, then a fixed-order sum."""
    M = A.shape[0]
    S = M // chunk
    a = A.view(S, chunk, A.shape[1]).transpose(1, 2)
    b = B.view(S, chunk, B.shape[1])
    if A.is_cuda:
        part = torch.bmm(a, b, out_dtype=torch.float32)
    else:
        part = torch.bmm(a.float(), b.float())
    return part.sum(0)


class _Done:
    """Work handle of a collective that already completed."""

    @staticmethod
    def wait():
        return True


_DONE = _Done()


class GCNTrainer:
    def __init__(self, g: GraphData, hidden: int = 256, dropout: float = 0.5, lr: float = 0.01,
                 weight_decay: float = 0.0, seed: int = 0, rank: Optional[int] = None,
                 world: Optional[int] = None, fused: bool = True, align_rows: Optional[bool] = None,
                 halo: Optional[bool] = None, capture: Optional[bool] = None, reorder: bool = False,
                 align_c: Optional[bool] = None, collectives: Optional[bool] = None,
                 train_rows_only: bool = True, l1_train_neighbours: bool = True, train_halo: bool = True,
                 bwd_overlap: bool = True):
        # train_rows_only / l1_train_neighbours: training epochs aggregate layer 2 only at
        # the train rows and layer 1 only at the rows those read (the update is the same;
        # False: every row, for equivalence tests).  train_halo: a multi-rank run's
        # training epochs exchange only the remote rows the train rows read (False: the
        # evaluation's exchange).  bwd_overlap: the backward's compact-gradient all-gather
        # overlaps the rank-local edges (False: serial).  All must agree across ranks.
        # reorder=True: relabel the nodes for gather locality first (data.reorder: LP
        # clusters + Cuthill-McKee, ~4-8 s of host C++ on the ogbn-products shape, part
        # of setup); the row partition of a multi-GPU run then cuts mostly between
        # clusters, which also shrinks the layer-2 halo.  Evaluation, and training with
        # dropout 0, are invariant; with dropout > 0 the masks are keyed by the RELABELLED
        # row, so a reordered run draws other masks (equal in distribution, not bitwise).
        # ``self.new_id`` maps the caller's node ids to the trainer's rows.
        self.new_id = None
        if reorder:
            from .data import reorder as _reorder
            g, self.new_id = _reorder(g, seed=seed)
        self.rank = pdist.rank() if rank is None else rank
        self.world = pdist.world_size() if world is None else world
        # the multi-rank code paths (exchanges, split aggregations, all-reduces): on with
        # more than one rank; ``collectives=True`` forces them on a 1-rank process group
        # (tests: the async RCCL exchange / stream-wait code without a second GPU)
        self.multi = self.world > 1 if collectives is None else (
            bool(collectives) and torch.distributed.is_available() and torch.distributed.is_initialized())
        self.dev = g.rowptr.device
        dev = self.dev
        self.F, self.C, self.hidden = g.n_features, g.n_classes, hidden
        # Gathered rows padded to whole 128-byte lines (a 208-B row straddles 2-3 lines, a
        # 256-B aligned one exactly 2; measured on the ogbn-products shape: layer-1 SpMM
        # 2.42 -> 2.20 ms, 3 % per epoch).  Default (None): the features always; the
        # layer-2 rows never: since training gathers them only for the train rows, the
        # packed 96-B rows (less to write, read and exchange) measured faster on one GPU
        # too (3.564 vs 3.590 ms, profiles/r02_l2gat/ab2_*.log).
        pad_c = False if align_rows is None else bool(align_rows)
        if align_c is not None:                  # layer-2 pitch chosen separately
            pad_c = bool(align_c)
        pad_x = True if align_rows is None else bool(align_rows)
        self.ldx = _ru(self.F + 1, 64) if pad_x else _ru8(self.F + 1)    # +1: ones column of AX
        self.ldc = _ru(self.C, 64) if pad_c else _ru8(self.C)
        self.p, self.lr, self.wd = float(dropout), float(lr), float(weight_decay)
        self.key = model_key(seed, "gcn-dropout")
        r0, r1, per, rp, col = partition_rows(g, self.rank, self.world)
        if (self.world - 1) * per >= g.n:
            # every collective plan below assumes each rank owns rows (an empty rank would
            # skip the collectives its peers block in)
            raise ValueError("GCNTrainer: %d nodes over %d ranks leaves the last rank without rows"
                             % (g.n, self.world))
        self.r0, self.r1, self.per, self.nloc = r0, r1, per, r1 - r0
        self.rowptr, self.col = rp.contiguous(), col.contiguous()
        self.dinv = g.dinv[r0:r1].contiguous()
        self.y = g.y[r0:r1].contiguous()
        self.mask = g.mask[r0:r1].contiguous()
        self.n_train = int((g.mask == 1).sum())
        self.n_val = int((g.mask == 2).sum())
        self.n_test = int((g.mask == 3).sum())
        bf = dict(dtype=torch.bfloat16, device=dev)
        # replicated normalised features Xs = D^-1/2 X, padded to ldx (zeros)
        self.Xs = torch.zeros(g.n, self.ldx, **bf)
        self.Xs[:, :self.F] = (g.x * g.dinv[:, None]).to(torch.bfloat16)
        # parameters: glorot-uniform weights, zero biases (PyG GCNConv init); one flat fp32 buffer
        gen = torch.Generator().manual_seed(seed)
        n1, n2 = self.F * hidden, hidden * self.C
        self.n_params = n1 + hidden + n2 + self.C
        flat = torch.zeros(self.n_params)
        a1 = math.sqrt(6.0 / (self.F + hidden))
        a2 = math.sqrt(6.0 / (hidden + self.C))
        flat[:n1] = (torch.rand(n1, generator=gen) * 2 - 1) * a1
        flat[n1 + hidden:n1 + hidden + n2] = (torch.rand(n2, generator=gen) * 2 - 1) * a2
        self.params = flat.to(dev)
        # the flat gradient, with a 68-float tail: a training epoch's cross-entropy
        # reduction writes its loss / accuracy sums there and its per-class dlogits sums
        # straight into gb2 (one reduction, no copy; ops.spmm_ce stats_out)
        self._grads_ext = torch.zeros(self.n_params + 68, dtype=torch.float32, device=dev)
        self.grads = self._grads_ext[:self.n_params]
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        o = [0, n1, n1 + hidden, n1 + hidden + n2, self.n_params]
        self.W1 = self.params[o[0]:o[1]].view(self.F, hidden)
        self.b1 = self.params[o[1]:o[2]]
        self.W2 = self.params[o[2]:o[3]].view(hidden, self.C)
        self.b2 = self.params[o[3]:o[4]]
        self.gW1 = self.grads[o[0]:o[1]].view(self.F, hidden)
        self.gb1 = self.grads[o[1]:o[2]]
        self.gW2 = self.grads[o[2]:o[3]].view(hidden, self.C)
        self.gb2 = self.grads[o[3]:o[4]]
        c68 = torch.arange(68, dtype=torch.int64)
        self._ce_index = torch.where(c68 < 4, self.n_params + c68,
                                     torch.where(c68 < 4 + self.C, o[3] + c68 - 4, torch.full_like(c68, -1)))
        self._ce_index = self._ce_index.to(torch.int32).to(dev)
        # activations / workspaces (rows of this rank; Z2/G padded to `per` rows for all-gather;
        # AX/H1/dH1/dY2 padded with zero rows to a multiple of CHUNK for the split-K GEMMs)
        n = self.nloc
        self.npad = (n + CHUNK - 1) // CHUNK * CHUNK
        # AX (the layer-1 aggregate: written once by the SpMM, streamed by the dense
        # forward and backward, never gathered) packed to whole 16-B chunks of its F + 1
        # columns: 208-B rows for ogbn-products instead of the gathered features' 256
        self.ldax = _ru8(self.F + 1)
        self.AX = torch.zeros(self.npad, self.ldax, **bf)
        # multi-GPU: the layer-1 aggregation of the NEXT epoch is computed into a second
        # buffer while the forward all-gather of Z2 is in flight (it does not depend on the
        # parameters), then the buffers swap; every epoch still performs its own SpMM
        # (Measured, not kept: on one GPU the same double buffer filled on a side stream,
        # so the next epoch's layer-1 aggregation overlaps this epoch's dense kernels --
        # neutral, 208.2 vs 208.8 epochs/s: the SpMM's blocks occupy every CU and the dense
        # forward only starts as they drain.  Round 5: started after the dense forward,
        # beside the latency-bound layer-2 / transposed aggregations, with the epoch's chain
        # on a high-priority stream -- neutral again, 315.5 vs 315.6: the dispatcher shares
        # the CUs between the two queues regardless of priority, the transposed aggregation
        # stretched from 0.23 to 2.18 ms beside the SpMM (profiles/r05_pref).)
        self.AX_next = torch.zeros_like(self.AX) if self.multi else None
        self._ax_ready = False
        if self.multi:
            # layer-2 aggregations split into edges whose source row this rank owns
            # (computed while the all-gather of the other ranks' rows is in flight) and
            # the remaining edges (after it), summed through an fp32 partial
            self.rp_loc, self.col_loc, self.rp_rem, self.col_rem = self._split_local(r0, r1)
            self.part = torch.zeros(self.nloc, self.ldc, dtype=torch.float32, device=dev)
        # compact dL/dlogits (train rows only) and the adjacency restricted to train columns
        self.gslot, self.rp_T, self.col_T, self.maxT = self._train_columns(g, per)
        self.Gc_loc = torch.zeros(self.maxT, self.ldc, **bf)
        self.Gc = torch.zeros(self.maxT * self.world, self.ldc, **bf) if self.multi else self.Gc_loc
        # bwd_overlap (several ranks): the all-gather of the compact gradient runs while the
        # second half of the next epoch's layer-1 aggregation is computed (False: blocking,
        # the half runs after it).  The backward aggregation itself is always one pass
        # over the whole train-column adjacency once G is complete -- round 5 split it
        # into this rank's own train columns (overlapped) and the rest, through an fp32
        # partial of every row: two launches and 2 x 59 MB of partial traffic per
        # 1/8-size epoch (37.6 + 29.8 us against ~22 us unsplit, profiles/r06_multirank)
        self._bwd_overlap = self.multi and bool(bwd_overlap)
        # the train-column adjacency's rows are short (~4 entries): on the GPU the
        # backward aggregation reads them from an ELL image (ops.spmm_ell)
        self._ell_T = ops.ell_image(self.rp_T, self.col_T) if dev.type == "cuda" else None
        self.H1 = torch.zeros(self.npad, hidden, **bf)
        self.dH1 = torch.zeros(self.npad, hidden, **bf)
        self.W2b = torch.zeros(hidden, self.ldc, **bf)
        self.Z2loc = torch.zeros(per, self.ldc, **bf)
        self.dY2 = torch.zeros(self.npad, self.ldc, **bf)
        # Layer-2 source rows of other ranks: a halo exchange (all-to-all of exactly the
        # rows this rank's edges read) or an all-gather of every row.  On the synthetic
        # ogbn-products graph the halo is 97 % of the all-gather's rows at 2 ranks, 86 %
        # at 4 and 66 % at 8, so by default it is used from 4 ranks on.  Needs an
        # initialised process group (the exchange plan is negotiated at setup).
        if halo is None:
            halo = self.world >= 4
        self.halo = bool(halo) and self.multi and torch.distributed.is_initialized()
        if self.halo:
            self._setup_halo(r0, r1, per)
            self.Z2 = None
        else:
            self.Z2 = torch.zeros(per * self.world, self.ldc, **bf) if self.multi else self.Z2loc
        # Training epochs aggregate layer 2 only at the rows the loss reads (this rank's
        # train rows): the other rows' logits enter neither the loss nor any gradient, so
        # the update is the same (the output-node pruning of DGL's last message-flow
        # block); every layer-1 row and every Z2 row is still computed, and evaluate()
        # aggregates all rows (train_rows_only=False: all rows in training too).
        self._l2 = None
        # The switch must agree across ranks: the training halo is negotiated
        # collectively, so a rank without train rows takes part with a placeholder row.
        trows = torch.nonzero(self.mask == 1).flatten()
        self._train_halo = bool(train_halo)
        if train_rows_only:
            self._l2 = self._train_row_csr(trows)
        # ... and then layer 1 is needed only at the rows with a train neighbour (the
        # sources those aggregations read; 94 % of the rows, 96.7 % of the entries on the
        # ogbn-products shape): training epochs aggregate layer 1 over a CSR whose other
        # rows are empty.  Their AX rows stay finite, their H1 / Z2 rows are read by no
        # train row and their dY2 rows are exactly 0, so the update is unchanged;
        # evaluation aggregates every row (l1_train_neighbours=False: every row).
        self._l1 = None
        if self._l2 is not None and l1_train_neighbours:
            self._l1 = self._train_neighbour_csr(g)
        # several ranks: the next epoch's layer-1 aggregation (parameter-independent) runs
        # in two row halves, the first beside the forward's layer-2 exchange, the second
        # beside the backward's gradient all-gather; each half a CSR of its own (row
        # pointers rebased, the columns a view)
        self._ax_halves = None
        if self.multi:
            rp, col = self._l1 if self._l1 is not None else (self.rowptr, self.col)
            h = self.nloc // 2
            self._ax_halves = []
            for a, b in ((0, h), (h, self.nloc)):
                e0, e1 = int(rp[a]), int(rp[b])
                self._ax_halves.append((a, b, (rp[a:b + 1] - e0).contiguous(), col[e0:e1]))
        # several ranks, training halo: layer 2 in ONE pass after the exchange -- the
        # exchange lands right behind this rank's Z2 rows (Z2ext = [Z2loc | received rows])
        # and the train rows' columns index that buffer (local c -> c - r0, remote ->
        # per + its position in the plan).  Round 5 aggregated the local edges into an
        # fp32 partial while the exchange was in flight: one more launch without the
        # long-row split of spmm_ce (47.7 us against ~10 us, profiles/r06_multirank); the
        # exchange is now covered by the first half of the next epoch's layer-1 SpMM.
        self.Z2ext = None
        l2 = self._l2
        if l2 is not None and l2.plan is not None:
            R = max(sum(l2.plan.recv_splits), 1)
            self.Z2ext = torch.zeros(per + R, self.ldc, **bf)
            self.Z2loc = self.Z2ext[:per]         # (the evaluation's exchange buffers stay separate)
            l2.plan.Zrecv = self.Z2ext[per:per + R]
            c = l2.col.long()
            loc = (c >= r0) & (c < r1)
            need = l2.plan.need
            rem = torch.searchsorted(need, c).clamp_max(max(need.numel() - 1, 0))
            l2.col_ext = torch.where(loc, c - r0, per + rem).to(torch.int32).contiguous()
        self._async = None                 # collectives overlapped? (decided at first use)
        self.epoch = 0
        self.last_stats = None
        # fused MFMA dense kernels (gnn_dense.hip); shapes they do not cover fall back to
        # hipBLASLt GEMMs + the standalone epilogue kernels
        self.fused = bool(fused) and hidden % 32 == 0 and self.C <= 64
        # fully fused backward (H1 recomputed, weight gradients in the same pass): H1 is
        # then never stored and the split-K GEMMs are not needed
        self.fused_bwd = (self.fused and dev.type == "cuda" and
                          ops.fused_bwd_supported(self.F, hidden, self.C))
        self._gpart = None
        self._grad_index = None
        # the training forward's dropout masks as the fused backward reads them (1 bit per
        # element: 78 MB for ogbn-products): the backward draws no Philox of its own
        self._kimg = (ops.keep_image(self.nloc, hidden, dev)
                      if self.fused_bwd and self.p > 0 else None)
        # capture=True (one GPU, fully fused path): the whole epoch (9 kernels + Adam) is
        # captured into a hipGraph and replayed; the dropout step is read from the device
        # step counter (Adam's), so replays draw the current epoch's mask.  Off by default:
        # a 5 ms epoch of 10 launches is not launch-bound, and on the ogbn-products shape
        # the replay measured 0.4 % SLOWER than eager launches (5.16 vs 5.14 ms, 2 x 40
        # epochs each).  Multi-GPU epochs are never captured (collectives, buffer swaps).
        from ..utils.hipgraph import StepGraph
        cap_ok = dev.type == "cuda" and not self.multi and self.fused_bwd
        self._graph = StepGraph(self._train_body, enabled=bool(capture) and cap_ok, device=dev)

    def _split_local(self, r0, r1, rowptr=None, col=None):
        """(rp, col) split into the edges whose column lies in [r0, r1) (columns shifted
        by -r0) and the rest."""
        rp = (self.rowptr if rowptr is None else rowptr).long()
        col = (self.col if col is None else col).long()
        n = rp.numel() - 1
        rows = torch.repeat_interleave(torch.arange(n, device=col.device), rp[1:] - rp[:-1])
        loc = (col >= r0) & (col < r1)

        def csr(sel, shift):
            counts = torch.bincount(rows[sel], minlength=n)
            out_rp = torch.zeros(n + 1, dtype=torch.int64, device=col.device)
            out_rp[1:] = torch.cumsum(counts, 0)
            return out_rp.to(torch.int32), (col[sel] - shift).to(torch.int32)

        a, b = csr(loc, r0)
        c, d = csr(~loc, 0)
        return a, b, c, d

    def _halo_plan(self, col_rem):
        """Exchange plan of a layer-2 halo: the distinct remote source rows that the
        edges ``col_rem`` (global ids) read -- sorted, hence grouped by owner in rank
        order -- are requested from their owners once; each exchange every rank sends
        the requested rows of its Z2 with one all-to-all.  Returns the plan with
        ``col``: the edges re-indexed into the received buffer."""
        dist = torch.distributed
        dev = self.dev
        col_rem = col_rem.long()
        need = torch.unique(col_rem)                                  # sorted global ids
        recv_counts = torch.bincount(need // self.per, minlength=self.world).to(torch.int64)
        send_counts = torch.empty_like(recv_counts)
        dist.all_to_all_single(send_counts, recv_counts)
        rc, sc = [int(v) for v in recv_counts.tolist()], [int(v) for v in send_counts.tolist()]
        req = torch.empty(sum(sc), dtype=torch.int64, device=dev)
        dist.all_to_all_single(req, need, output_split_sizes=sc, input_split_sizes=rc)
        if req.numel() and (int(req.min()) < self.r0 or int(req.max()) >= self.r1):
            raise RuntimeError("halo plan: a peer requested a row this rank does not own")
        bf = dict(dtype=torch.bfloat16, device=dev)
        return types.SimpleNamespace(
            need=need, send_idx=(req - self.r0).contiguous(), recv_splits=rc, send_splits=sc,
            col=torch.searchsorted(need, col_rem).to(torch.int32).contiguous(),
            Zrecv=torch.zeros(max(sum(rc), 1), self.ldc, **bf),
            Zsend=torch.zeros(max(sum(sc), 1), self.ldc, **bf))

    def _setup_halo(self, r0, r1, per):
        """The full halo (every remote row this rank's edges read): evaluation, and
        training with train_rows_only=False."""
        self._hplan = self._halo_plan(self.col_rem)
        self.col_rem = self._hplan.col

    def _train_neighbour_csr(self, g):
        """This rank's CSR with the edge lists of rows that have no train neighbour (any
        rank's; A is symmetric) emptied."""
        rp, col = self.rowptr.long(), self.col.long()
        deg = rp[1:] - rp[:-1]
        rows = torch.repeat_interleave(torch.arange(self.nloc, device=col.device), deg)
        train = (g.mask == 1).to(col.device)
        hit = torch.zeros(self.nloc, dtype=torch.bool, device=col.device)
        hit[rows[train[col]]] = True
        keep = hit[rows]
        nrp = torch.zeros(self.nloc + 1, dtype=torch.int64, device=col.device)
        nrp[1:] = torch.cumsum(torch.where(hit, deg, torch.zeros_like(deg)), 0)
        return nrp.to(torch.int32).contiguous(), self.col[keep].contiguous()

    def _train_row_csr(self, trows):
        """Layer-2 operands of the train rows ``trows`` (local ids, ascending): their
        CSR rows, output-row scale / labels / split, the compact-gradient slot (the k-th
        train row of this rank is slot k, as in ``_train_columns``), and on several ranks
        the same local / remote edge split (remote columns re-indexed like ``col_rem``)."""
        dev = self.dev
        rp = self.rowptr.long()
        placeholder = trows.numel() == 0
        if placeholder:            # no train rows here: one edgeless, non-train row (writes nothing)
            trows = torch.zeros(1, dtype=torch.int64, device=dev)
        lo, deg = rp[trows], rp[trows + 1] - rp[trows]
        if placeholder:
            deg = torch.zeros_like(deg)
        # the long rows first (spmm_ce gives each a whole wave, ops.long_row_order); the
        # compact-gradient slot stays the row's position among the ascending train rows
        order, n_long = ops.long_row_order(deg)
        trows, lo, deg = trows[order], lo[order], deg[order]
        trp = torch.zeros(trows.numel() + 1, dtype=torch.int64, device=dev)
        trp[1:] = torch.cumsum(deg, 0)
        eid = torch.arange(int(trp[-1]), device=dev) + torch.repeat_interleave(lo - trp[:-1], deg)
        l2 = types.SimpleNamespace(
            rp=trp.to(torch.int32).contiguous(), col=self.col[eid].contiguous(),
            dinv=self.dinv[trows].contiguous(), y=self.y[trows].contiguous(),
            mask=torch.zeros_like(self.mask[trows]) if placeholder else self.mask[trows].contiguous(),
            gslot=torch.full((1,), -1, dtype=torch.int32, device=dev) if placeholder
            else order.to(torch.int32).contiguous(), n_long=n_long)
        l2.plan = None
        if self.multi:
            l2.rp_loc, l2.col_loc, l2.rp_rem, col_rem = self._split_local(self.r0, self.r1, l2.rp, l2.col)
            if torch.distributed.is_initialized() and self._train_halo:
                # a halo of its own: only the remote rows the train rows read travel in
                # training epochs (planted-community graph after the reorder: ~10 % of
                # the other ranks' rows at 8 ranks, ~40 % at 2, against 66-97 % for the
                # full halo); train_halo=False: the evaluation's exchange
                l2.plan = self._halo_plan(col_rem)
                col_rem = l2.plan.col
            elif self.halo:
                col_rem = torch.searchsorted(self._hplan.need, col_rem.long()).to(torch.int32)
            l2.col_rem = col_rem.contiguous()
            l2.part = torch.zeros(trows.numel(), self.ldc, dtype=torch.float32, device=dev)
        return l2

    def _collective(self, fn, *args):
        """``fn(*args)`` asynchronously (returns its work handle) on RCCL and on CPU
        tensors; blocking for device tensors over gloo (only the one-GPU rehearsal,
        where gloo stages them through the host anyway and nothing can overlap)."""
        if self._async is None:
            self._async = (self.dev.type == "cpu" or torch.distributed.get_backend() != "gloo")
        if self._async:
            return fn(*args, async_op=True)
        fn(*args)
        return _DONE

    def _exchange_z2(self, plan=None):
        """Start the transfer of the other ranks' layer-2 rows: the halo of ``plan``
        or, without one, the full halo (``self.halo``) or an all-gather of every row.
        Returns (work, buffer the remote edges index)."""
        if plan is None and self.halo:
            plan = self._hplan
        if plan is None:
            return self._collective(torch.distributed.all_gather_into_tensor, self.Z2, self.Z2loc), self.Z2
        S, R = sum(plan.send_splits), sum(plan.recv_splits)
        torch.index_select(self.Z2loc, 0, plan.send_idx, out=plan.Zsend[:S])
        work = self._collective(torch.distributed.all_to_all_single, plan.Zrecv[:R], plan.Zsend[:S],
                                plan.recv_splits, plan.send_splits)
        return work, plan.Zrecv

    def _train_columns(self, g: GraphData, per: int):
        """Slots of the compact gradient and the local CSR restricted to train columns.
        A train node j owned by rank r = j // per with ordinal k among that rank's train
        nodes lives in slot r * maxT + k of the all-gathered compact G (maxT = the
        largest per-rank train count); ``gslot`` maps this rank's rows to k (or -1)."""
        dev = self.col.device
        train = (g.mask == 1).to(dev)
        n = train.numel()
        owner = torch.arange(n, device=dev) // per
        t = train.to(torch.int64)
        excl = torch.cumsum(t, 0) - t                              # train nodes before j
        first = torch.arange(self.world, device=dev) * per
        base = excl[first.clamp_max(n - 1)]                        # train nodes before rank r's block
        ordinal = excl - base[owner]
        counts = torch.bincount(owner[train], minlength=self.world)
        maxT = max(int(counts.max()), 1)
        slot = torch.where(train, owner * maxT + ordinal, torch.full_like(ordinal, -1))
        gslot = torch.where(train[self.r0:self.r1], ordinal[self.r0:self.r1],
                            torch.full_like(ordinal[self.r0:self.r1], -1)).to(torch.int32).contiguous()
        col = self.col.long()
        keep = train[col]
        nloc = self.rowptr.numel() - 1
        deg = (self.rowptr[1:] - self.rowptr[:-1]).long()
        rows = torch.repeat_interleave(torch.arange(nloc, device=dev), deg)
        cnt = torch.bincount(rows[keep], minlength=nloc)
        rp = torch.zeros(nloc + 1, dtype=torch.int64, device=dev)
        rp[1:] = torch.cumsum(cnt, 0)
        col_T = slot[col[keep]].to(torch.int32).contiguous()
        return gslot, rp.to(torch.int32).contiguous(), col_T, maxT

    # ------------------------------------------------------------------ passes
    def _all_gather(self, out, inp):
        if self.multi:
            torch.distributed.all_gather_into_tensor(out, inp)

    def _aggregate_features(self, out, train: bool = False):
        rp, col = self._l1 if (train and self._l1 is not None) else (self.rowptr, self.col)
        ops.spmm(rp, col, self.Xs, self.F, rscale=self.dinv, out=out, unit_col=self.F)

    def _aggregate_half(self, k):
        """Rows of half ``k`` of the next epoch's layer-1 aggregation, into AX_next."""
        a, b, rp, col = self._ax_halves[k]
        if b > a:
            ops.spmm(rp, col, self.Xs, self.F, rscale=self.dinv[a:b], out=self.AX_next[a:b], unit_col=self.F)

    def forward(self, train: bool):
        n, F, C = self.nloc, self.F, self.C
        H1 = self.H1[:n]
        p = self.p if train else 0.0
        kimg = self._kimg if train else None
        # a prefetched AX restricted to the train-neighbour rows serves training only
        fresh = not self._ax_ready or not (train or self._l1 is None)
        self._ax_ready = False
        if fresh:
            self._aggregate_features(self.AX, train)
        if not self.fused_bwd:           # bf16 W2 of the unfused fallbacks (the fused kernels read fp32)
            self.W2b[:, :C] = self.W2.to(torch.bfloat16)
        if not (self.fused and ops.dense_fwd(self.AX, self.W1, self.b1, self.W2, self.dinv,
                                                          None if self.fused_bwd else H1,
                                                          self.Z2loc[:n], F, p, self.key, self._dropout_step(),
                                                          self.r0, kimg=kimg)):
            W1b = self.W1.to(torch.bfloat16)
            if self.AX.is_cuda:
                torch.mm(self.AX[:n, :F], W1b, out=H1)
            else:
                H1.copy_((self.AX[:n, :F].float() @ W1b.float()).to(torch.bfloat16))
            ops.bias_relu_dropout_(H1, self.b1, self.hidden, p, self.key, self.epoch, self.r0)
            y2 = _mm_f32(H1, self.W2b)
            torch.mul(y2, self.dinv[:, None], out=y2)
            self.Z2loc[:n] = y2.to(torch.bfloat16)
        l2 = self._l2 if train else None          # train rows only (see __init__)
        if self.multi and l2 is not None and l2.plan is not None:
            # training halo: the exchange fills Z2ext behind the local rows while the first
            # half of the next epoch's layer-1 aggregation runs; then one layer-2 pass
            work, _ = self._exchange_z2(l2.plan)
            self._aggregate_half(0)
            work.wait()
            rp, col, init, zsrc = l2.rp, l2.col_ext, None, self.Z2ext
        elif self.multi:
            # the Z2 exchange (up to [n, 48] bf16, 7/8 of it inbound at 8 ranks): the
            # rank-local layer-2 edges and, in training, the first half of the next epoch's
            # layer-1 aggregation run while it is in flight
            work, zsrc = self._exchange_z2(l2.plan if l2 is not None else None)
            if l2 is not None:
                ops.spmm(l2.rp_loc, l2.col_loc, self.Z2loc, C, out=l2.part, out_dtype=torch.float32)
            else:
                ops.spmm(self.rp_loc, self.col_loc, self.Z2loc, C, out=self.part, out_dtype=torch.float32)
            if train:
                self._aggregate_half(0)
            work.wait()
            if l2 is not None:
                rp, col, init = l2.rp_rem, l2.col_rem, l2.part
            else:
                rp, col, init = self.rp_rem, self.col_rem, self.part
        elif l2 is not None:
            rp, col, init, zsrc = l2.rp, l2.col, None, self.Z2
        else:
            rp, col, init, zsrc = self.rowptr, self.col, None, self.Z2
        if l2 is not None:
            dinv, y, mask, gslot = l2.dinv, l2.y, l2.mask, l2.gslot
        else:
            dinv, y, mask, gslot = self.dinv, self.y, self.mask, (self.gslot if train else None)
        fold = train and zsrc.is_cuda
        stats, _ = ops.spmm_ce(rp, col, zsrc, C, dinv, self.b2, y, mask,
                               1.0 / max(self.n_train, 1), mode=0 if train else 1,
                               G=self.Gc_loc if train else None, init=init, gslot=gslot,
                               n_long=l2.n_long if l2 is not None else 0,
                               stats_out=(self._grads_ext, self._ce_index) if fold else None)
        if fold:      # (gb2 is written; the tail holds stats[0:4], enough for every reader)
            stats = self._grads_ext[self.n_params:]
        return stats

    def backward(self, stats):
        n, F, C = self.nloc, self.F, self.C
        if self.multi:
            # the compact gradients of every rank; the second half of the next epoch's
            # layer-1 aggregation runs beside the all-gather (bwd_overlap) or after it
            if self._bwd_overlap:
                work = self._collective(torch.distributed.all_gather_into_tensor, self.Gc, self.Gc_loc)
                self._aggregate_half(1)
                work.wait()
            else:
                torch.distributed.all_gather_into_tensor(self.Gc, self.Gc_loc)
                self._aggregate_half(1)
        if self._ell_T is not None:
            ops.spmm_ell(self._ell_T, self.col_T, self.Gc, C, rscale=self.dinv, out=self.dY2)
        else:
            ops.spmm(self.rp_T, self.col_T, self.Gc, C, rscale=self.dinv, out=self.dY2)
        if not self.dY2.is_cuda:          # (GPU: written by the forward's reduction)
            self.gb2.copy_(stats[4:4 + C])
        if self.fused_bwd:
            if self._grad_index is None:
                self._grad_index = ops.fused_bwd_grad_index(
                    F, self.hidden, C, ops.fused_bwd_width(F), device=self.dev)
            _, _, _, self._gpart = ops.fused_bwd(self.AX, self.dY2, self.W1, self.b1, self.W2, n, F,
                                                 self.p, self.key, self._dropout_step(), self.r0,
                                                 self._gpart, grads=self.grads, grad_index=self._grad_index,
                                                 kimg=self._kimg)
            if self.multi:
                torch.distributed.all_reduce(self.grads)
            return
        self.gW2.copy_(_tsgemm(self.H1, self.dY2)[:, :C])
        dH1 = self.dH1[:n]
        if not (self.fused and ops.dense_bwd(self.dY2, self.W2, self.H1, dH1, self.p)):
            if dH1.is_cuda:
                torch.mm(self.dY2[:n, :C], self.W2b[:, :C].t(), out=dH1)
            else:
                dH1.copy_((self.dY2[:n, :C].float() @ self.W2b[:, :C].float().t()).to(torch.bfloat16))
            ops.relu_dropout_bwd_(dH1, self.H1[:n], self.p)
        g1 = _tsgemm(self.AX, self.dH1)               # rows 0..F-1: dW1, row F: db1 (ones column)
        self.gW1.copy_(g1[:F])
        self.gb1.copy_(g1[F])
        if self.multi:
            torch.distributed.all_reduce(self.grads)

    def _dropout_step(self):
        """The dropout step of the fused kernels: the device step counter on a GPU (equal
        to the epoch; readable by a replayed hipGraph), the epoch on the CPU."""
        return self.step_t if (self.dev.type == "cuda" and self.fused_bwd) else self.epoch

    def _train_body(self):
        stats = self.forward(train=True)
        self.backward(stats)
        ops.adam_(self.params, self.grads, self.m, self.v, self.lr, self.step_t, wd=self.wd)
        return stats

    def train_step(self):
        stats = self._graph()
        if self.AX_next is not None:
            self.AX, self.AX_next = self.AX_next, self.AX
            self._ax_ready = True
        self.last_stats = stats
        self.epoch += 1
        return stats

    @torch.no_grad()
    def evaluate(self):
        """Accuracies on train / valid / test (no dropout), reduced over ranks."""
        stats = self.forward(train=False).clone()
        if self.multi:
            torch.distributed.all_reduce(stats)
        s = stats.cpu().numpy()
        return {"train_loss": float(s[0]) / max(self.n_train, 1),
                "train_acc": float(s[1]) / max(self.n_train, 1),
                "val_acc": float(s[2]) / max(self.n_val, 1),
                "test_acc": float(s[3]) / max(self.n_test, 1)}

    # ---------------------------------------------------------------- checkpoint
    def state_tensors(self):
        """Flat fp32 parameters, Adam moments and step, dropout RNG key (identical on
        every rank; the dropout stream position is the epoch, kept in the metadata)."""
        key = torch.tensor([int(self.key[0]), int(self.key[1])], dtype=torch.int64)
        return {"params": self.params, "adam_m": self.m, "adam_v": self.v, "adam_step": self.step_t,
                "rng_key": key}

    def load_state_tensors(self, t):
        if "rng_key" in t:
            self.key = (int(t["rng_key"][0]), int(t["rng_key"][1]))
        for name, dst in (("params", self.params), ("adam_m", self.m), ("adam_v", self.v),
                          ("adam_step", self.step_t)):
            if t[name].shape != dst.shape:
                raise ValueError("checkpoint %s has shape %s, trainer %s" % (name, tuple(t[name].shape),
                                                                              tuple(dst.shape)))
            dst.copy_(t[name].to(dst.device))
        self._ax_ready = False
        self._graph.reset()          # the dropout key is a launch argument of the captured kernels

    def train_loss(self):
        s = self.last_stats.clone()
        if self.multi:
            torch.distributed.all_reduce(s)
        return float(s[0]) / max(self.n_train, 1)


def smoke_step():
    """Two tiny GCN training steps on cuda:0 through the flagship fused kernels (a
    0.1 % ogbn-products-shaped graph, hidden 256; used by __graft_entry__.smoke)."""
    from .data import synthetic
    g = synthetic("ogbn-products", seed=0, device="cuda:0", scale=0.001)
    tr = GCNTrainer(g, hidden=256, rank=0, world=1)
    assert tr.fused and tr.fused_bwd
    tr.train_step()
    tr.train_step()
    res = tr.evaluate()
    torch.cuda.synchronize()
    assert math.isfinite(res["train_loss"]), res
    return res
