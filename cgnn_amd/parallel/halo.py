"""Halo exchange for row-partitioned graphs (one process per GPU; RCCL all-to-all over
xGMI, gloo on CPUs).

Rank r owns rows [r0, r1) (blocks of ``per``) of an n-node graph and holds the CSR of
its rows with GLOBAL source ids.  Instead of all-gathering every row of the graph,
each rank receives exactly the remote source rows its edges read:

* setup (collective, once): the distinct remote ids (sorted, hence grouped by owner)
  are sent to their owners with one all-to-all; every rank learns which of its rows
  each peer reads (``send_idx``), and the CSR columns are renumbered into the
  extended row space ``[own rows | received rows]`` (``col_ext``);
* forward: all-to-alls of the requested rows, several column groups packed per row
  as raw bytes (bf16 activations and fp32 attention scores side by side, so the
  scores cross the link exactly);
* backward: the transpose -- the gradient rows of the received rows go back to their
  owners (fp32 by default) and are summed into the owner's rows peer by peer (the
  rows one peer returns are distinct, so every accumulation is deterministic).

**Bounded memory: the exchange runs in rounds.**  At the papers100M shape with
shuffled ids a rank receives ~6x its own rows (every node has ~30 neighbours), so a
one-shot exchange needs send / receive staging buffers of tens of GB per direction
(89 M rows x 708 B of fp32 layer-2 gradient = 63 GB at 8 ranks) on top of the
activations.  Every peer's slice is split into ``rounds`` equal parts (the same
count on every rank: an all-reduce MAX at setup, sized so that one round moves at
most ``chunk_bytes`` of the widest payload), and the received rows are laid out
ROUND-MAJOR in the extended row space: round t's rows from all peers are one
contiguous block ``ext_range(t)``.  So each round receives straight into its block,
and in the backward a producer can compute only that block's gradient rows
(:meth:`reduce_back_stream`, used by the fused GAT: the [n_ext, K Fh] fp32 gradient
of the received rows is never materialised).

``emulate=(rank, world)`` builds the plan of one rank of a larger job inside a single
process (no process group): the send side is a symmetric stand-in (as many rows sent
as received, to this rank's own rows), received rows are zero and returned gradients
are zero -- a dry run with every buffer, kernel and byte count of that rank (memory
and compute measurements), not its numerics.
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Sequence, Tuple

import torch


def _rows(src: torch.Tensor, dst: torch.Tensor, src_idx=None, dst_idx=None, mode: int = 0):
    """``dst[dst_idx[r] or r] (op)= src[src_idx[r] or r]`` for r < rows (= len of the index, or
    of src): mode 0 copies (same dtype, 4-byte multiple rows), 1 adds fp32 into fp32, 2 adds
    bf16 into fp32 (accumulate modes: distinct dst rows).  2-D operands with unit column
    stride (column slices of row-major buffers are fine).  GPU: one HIP launch
    (csrc/kernels/gnn_halo.hip); CPU: the same with index ops."""
    rows = (src_idx.numel() if src_idx is not None else
            dst_idx.numel() if dst_idx is not None else src.shape[0])
    if rows == 0:
        return
    from ..utils import checks
    if checks.enabled():
        checks.index(src_idx, src.shape[0], "halo rows src_idx")
        checks.index(dst_idx, dst.shape[0], "halo rows dst_idx")
        if src_idx is None:
            checks.rows(src, rows, "halo rows src")
        if dst_idx is None:
            checks.rows(dst, rows, "halo rows dst")
    if mode == 0 and (dst.shape[1] * dst.element_size()) % 4:
        # the row kernel copies whole 4-byte words: a row of odd bf16 width would lose its
        # last element on the GPU (pad the column group to 4 bytes)
        raise ValueError("halo row copy: %d-byte rows are not a multiple of 4 bytes"
                         % (dst.shape[1] * dst.element_size()))
    if dst.is_cuda:
        from .. import native
        words = dst.shape[1] if mode else dst.shape[1] * dst.element_size() // 4
        native.hip().gnn_halo_rows(src.data_ptr(), src.stride(0) * src.element_size(),
                                   src_idx.data_ptr() if src_idx is not None else 0, dst.data_ptr(),
                                   dst.stride(0) * dst.element_size(),
                                   dst_idx.data_ptr() if dst_idx is not None else 0, rows, words, mode,
                                   torch.cuda.current_stream(dst.device).cuda_stream)
        return
    v = src.index_select(0, src_idx) if src_idx is not None else src[:rows]
    if mode == 0:
        if dst_idx is not None:
            dst[dst_idx] = v
        else:
            dst[:rows] = v
    elif dst_idx is not None:
        dst.index_put_((dst_idx,), v.to(dst.dtype), accumulate=True)
    else:
        dst[:rows] += v.to(dst.dtype)


class HaloExchange:
    def __init__(self, col: torch.Tensor, r0: int, r1: int, per: int, n: int, group=None,
                 emulate: Optional[Tuple[int, int]] = None, max_row_bytes: int = 1024,
                 chunk_bytes: int = 4 << 30):
        import torch.distributed as dist
        self.group = group
        self.dev = col.device
        self.r0, self.r1, self.per, self.n = int(r0), int(r1), int(per), int(n)
        self.nloc = self.r1 - self.r0
        self.emulate = emulate is not None
        if self.emulate:
            self.rank, self.world = int(emulate[0]), int(emulate[1])
        else:
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
        c = col.long()
        local = (c >= self.r0) & (c < self.r1)
        need = torch.unique(c[~local])                               # sorted global ids = grouped by owner
        recv_counts = torch.bincount(need // self.per, minlength=self.world).to(torch.int64)
        if self.emulate:
            send_counts = recv_counts.clone()
            send_counts[self.rank] = 0
            req = self.r0 + torch.arange(int(send_counts.sum()), dtype=torch.int64, device=self.dev) % max(self.nloc, 1)
        else:
            send_counts = torch.empty_like(recv_counts)
            dist.all_to_all_single(send_counts, recv_counts, group=group)
            sc = [int(v) for v in send_counts.tolist()]
            req = torch.empty(sum(sc), dtype=torch.int64, device=self.dev)
            dist.all_to_all_single(req, need, output_split_sizes=sc,
                                   input_split_sizes=[int(v) for v in recv_counts.tolist()], group=group)
            if req.numel() and (int(req.min()) < self.r0 or int(req.max()) >= self.r1):
                raise RuntimeError("halo plan: a peer requested a row this rank does not own")
        self.recv_splits: List[int] = [int(v) for v in recv_counts.tolist()]
        self.send_splits: List[int] = [int(v) for v in send_counts.tolist()]
        self.n_recv, self.n_send = sum(self.recv_splits), sum(self.send_splits)
        self.send_idx = (req - self.r0).contiguous()
        self.need = need
        # rounds: identical on every rank
        rb = max(self.n_recv, self.n_send) * int(max_row_bytes)
        rounds = max(1, math.ceil(rb / max(int(chunk_bytes), 1)))
        if not self.emulate and dist.is_initialized():
            t = torch.tensor([rounds], dtype=torch.int64, device=self.dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            rounds = int(t.item())
        self.rounds = rounds
        # per round: the rows of every peer slice in that round (equal split of each slice)
        self._recv_r = [self._split(self.recv_splits, t) for t in range(rounds)]
        self._send_r = [self._split(self.send_splits, t) for t in range(rounds)]
        # round-major position of every needed row in the extended space
        pos = torch.empty(self.n_recv, dtype=torch.int64, device=self.dev)
        soff = [0]
        for v in self.recv_splits:
            soff.append(soff[-1] + v)
        self._ext_base = []
        base = 0
        for t in range(rounds):
            self._ext_base.append(base)
            for p, (a, b) in enumerate(self._recv_r[t]):
                if b > a:
                    pos[soff[p] + a:soff[p] + b] = torch.arange(base, base + b - a, device=self.dev)
                    base += b - a
        self._ext_base.append(base)
        self._pos = pos
        j = torch.searchsorted(need, c.clamp_min(0))
        ext = torch.where(local, c - self.r0, self.nloc + pos[j.clamp_max(max(self.n_recv - 1, 0))]
                          if self.n_recv else c - self.r0)
        self.col_ext = ext.to(torch.int32).contiguous()
        self.n_ext = self.nloc + self.n_recv
        # per round: the own rows sent (peer order) and per-peer slices of them
        self._send_idx_r = []
        off = [0]
        for v in self.send_splits:
            off.append(off[-1] + v)
        for t in range(rounds):
            parts = [self.send_idx[off[p] + a:off[p] + b] for p, (a, b) in enumerate(self._send_r[t])]
            self._send_idx_r.append(torch.cat(parts) if parts else self.send_idx[:0])

    def received_ids(self) -> torch.Tensor:
        """Global id of every received row, in extended-space order (rows nloc...)."""
        ids = torch.empty(self.n_recv, dtype=torch.int64, device=self.dev)
        ids[self._pos] = self.need
        return ids

    def _split(self, splits: Sequence[int], t: int):
        R = self.rounds
        return [(L * t // R, L * (t + 1) // R) for L in splits]

    def _sizes(self, ranges):
        return [b - a for a, b in ranges]

    def ext_range(self, t: int) -> Tuple[int, int]:
        """Rows [lo, hi) of the extended space received in round t."""
        return self.nloc + self._ext_base[t], self.nloc + self._ext_base[t + 1]

    # ------------------------------------------------------------------ packing
    @staticmethod
    def pack(parts: Sequence[torch.Tensor]) -> torch.Tensor:
        """[rows, bytes] uint8 view of column groups of any float dtype (the wire format:
        raw bytes, so every backend moves them unchanged)."""
        return torch.cat([t.contiguous().view(torch.uint8) for t in parts], 1)

    @staticmethod
    def unpack(buf: torch.Tensor, spec: Sequence[Tuple[int, torch.dtype]]) -> List[torch.Tensor]:
        out, c = [], 0
        for width, dt in spec:
            nb = width * torch.empty(0, dtype=dt).element_size()
            out.append(buf[:, c:c + nb].contiguous().view(dt))
            c += nb
        return out

    # ------------------------------------------------------------------ exchange
    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        import torch.distributed as dist
        if self.emulate:
            out.zero_()
            return
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=self.group)

    def exchange_parts(self, parts: Sequence[torch.Tensor]) -> List[torch.Tensor]:
        """Rows [own | received] of column groups ``parts`` ([nloc, w_i], any dtypes):
        one all-to-all per round, the groups packed side by side as raw bytes per row."""
        ext = []
        for p in parts:
            e = torch.empty((self.n_ext,) + tuple(p.shape[1:]), dtype=p.dtype, device=self.dev)
            e[:self.nloc] = p
            ext.append(e)
        nbytes = [p.shape[1] * p.element_size() for p in parts]
        W = sum(nbytes)
        for t in range(self.rounds):
            lo, hi = self.ext_range(t)
            idx = self._send_idx_r[t]
            send = torch.empty(idx.numel(), W, dtype=torch.uint8, device=self.dev)
            c = 0
            for p, nb in zip(parts, nbytes):                   # gather the requested rows
                _rows(p.view(torch.uint8), send[:, c:c + nb], src_idx=idx)
                c += nb
            recv = torch.empty(hi - lo, W, dtype=torch.uint8, device=self.dev)
            self._all_to_all(recv, send, self._sizes(self._recv_r[t]), self._sizes(self._send_r[t]))
            del send
            c = 0
            for e, nb in zip(ext, nbytes):                     # unpack into this round's block
                _rows(recv[:, c:c + nb], e.view(torch.uint8)[lo:hi])
                c += nb
            del recv
        return ext

    def exchange(self, payload_local: torch.Tensor) -> torch.Tensor:
        """Rows [own | received] of a packed local payload [nloc, W] (uint8)."""
        return self.exchange_parts([payload_local])[0]

    def reduce_back(self, parts: Sequence[torch.Tensor], wire_dtype: torch.dtype = torch.float32):
        """Transpose of :meth:`exchange` for gradients given as column groups [n_ext, w_i]:
        the own rows of every group plus the gradients of the rows peers read, returned
        to this rank (in ``wire_dtype``) and summed in peer order.  Returns one
        [nloc, w_i] tensor per group (in place on the own-row slices of ``parts``)."""
        def produce(lo, hi):
            return [p[lo:hi] for p in parts]
        return self.reduce_back_stream(produce, [p[:self.nloc] for p in parts], wire_dtype)

    def reduce_back_stream(self, produce: Callable[[int, int], Sequence[torch.Tensor]],
                           own: Sequence[torch.Tensor], wire_dtype: torch.dtype = torch.float32):
        """:meth:`reduce_back` with the received rows' gradients made on demand:
        ``produce(lo, hi)`` returns the gradient groups of extended rows [lo, hi) (one
        round's block); the peers' returns are added into ``own`` ([nloc, w_i], in
        place), which is returned."""
        widths = [o.shape[1] for o in own]
        for t in range(self.rounds):
            lo, hi = self.ext_range(t)
            send = torch.empty(hi - lo, sum(widths), dtype=wire_dtype, device=self.dev)
            if hi > lo:
                got = produce(lo, hi)
                c = 0
                for g, w in zip(got, widths):
                    if g.dtype == wire_dtype:
                        _rows(g, send[:, c:c + w])
                    else:
                        send[:, c:c + w].copy_(g)
                    c += w
                del got
            idx = self._send_idx_r[t]
            back = torch.empty(idx.numel(), sum(widths), dtype=wire_dtype, device=self.dev)
            self._all_to_all(back, send, self._sizes(self._send_r[t]), self._sizes(self._recv_r[t]))
            del send
            mode = 2 if wire_dtype == torch.bfloat16 else 1
            a = 0
            for p, n_p in enumerate(self._sizes(self._send_r[t])):
                if n_p:                                   # one peer's rows are distinct: no conflicts
                    rows = idx[a:a + n_p]
                    c = 0
                    for g, w in zip(own, widths):
                        if g.dtype != torch.float32:
                            g.index_put_((rows,), back[a:a + n_p, c:c + w].to(g.dtype), accumulate=True)
                        else:
                            _rows(back[a:a + n_p, c:c + w], g, dst_idx=rows, mode=mode)
                        c += w
                a += n_p
            del back
        return list(own)

    def bytes_per_exchange(self, width_bytes: int) -> Tuple[int, int]:
        """(bytes received, bytes sent) by this rank for one exchange of ``width_bytes`` rows."""
        return self.n_recv * width_bytes, self.n_send * width_bytes
