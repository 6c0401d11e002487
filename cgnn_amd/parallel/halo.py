"""Halo exchange for row-partitioned graphs (one process per GPU; RCCL all-to-all over
xGMI, gloo on CPUs).

Rank r owns rows [r0, r1) (blocks of ``per``) of an n-node graph and holds the CSR of
its rows with GLOBAL source ids.  Instead of all-gathering every row of the graph,
each rank receives exactly the remote source rows its edges read:

* setup (collective, once): the distinct remote ids (sorted, hence grouped by owner)
  are sent to their owners with one all-to-all; every rank learns which of its rows
  each peer reads (``send_idx``), and the CSR columns are renumbered into the
  extended row space ``[own rows | received rows]`` (``col_ext``);
* forward: one all-to-all of the requested rows, packed into ONE byte buffer
  (bf16 activations and fp32 columns such as GAT's attention scores side by side
  as raw bytes, so the scores cross the link exactly);
* backward: the transpose -- the gradient rows of the received rows go back to their
  owners (fp32 by default) and are summed into the owner's rows peer by peer (the
  rows one peer returns are distinct, so every accumulation is deterministic).

xGMI sizing: a full-graph epoch moves the halo twice per layer; at 8 ranks with
shuffled ids the halo is most of the graph (every node has ~30 neighbours), so the
win over an fp32 all-gather is the bf16 payload and the rows nobody reads; a
locality-preserving partition shrinks it further (``gnn.data.reorder``).

``emulate=(rank, world)`` builds the plan of one rank of a larger job inside a single
process (no process group): the exchange then leaves the received rows at zero and
returns no gradient to peers -- a dry run that has every buffer, kernel and byte
count of that rank (memory and compute measurements), not its numerics.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch


class HaloExchange:
    def __init__(self, col: torch.Tensor, r0: int, r1: int, per: int, n: int, group=None,
                 emulate: Optional[Tuple[int, int]] = None):
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
            send_counts = torch.zeros_like(recv_counts)
            req = torch.empty(0, dtype=torch.int64, device=self.dev)
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
        ext = torch.where(local, c - self.r0, self.nloc + torch.searchsorted(need, c))
        self.col_ext = ext.to(torch.int32).contiguous()
        self.n_ext = self.nloc + self.n_recv
        # peer slices of send_idx (distinct rows within one slice: deterministic accumulation)
        bounds = [0]
        for v in self.send_splits:
            bounds.append(bounds[-1] + v)
        self._slices = [(bounds[i], bounds[i + 1]) for i in range(self.world) if bounds[i + 1] > bounds[i]]

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

    def exchange(self, payload_local: torch.Tensor) -> torch.Tensor:
        """Rows [own | received] of a packed local payload [nloc, W] (uint8)."""
        W = payload_local.shape[1]
        ext = torch.empty(self.n_ext, W, dtype=payload_local.dtype, device=self.dev)
        ext[:self.nloc] = payload_local
        send = payload_local.index_select(0, self.send_idx) if self.n_send else payload_local[:0]
        self._all_to_all(ext[self.nloc:], send.contiguous(), self.recv_splits, self.send_splits)
        return ext

    def reduce_back(self, parts: Sequence[torch.Tensor], wire_dtype: torch.dtype = torch.float32):
        """Transpose of :meth:`exchange` for gradients given as column groups [n_ext, w_i]:
        the own rows of every group plus the gradients of the rows peers read, returned
        to this rank (one all-to-all of only the received rows, in ``wire_dtype``) and
        summed in peer order.  Returns one [nloc, w_i] tensor per group (in place on the
        own-row slices of ``parts``, no full-size copy)."""
        widths = [p.shape[1] for p in parts]
        send = torch.cat([p[self.nloc:].to(wire_dtype) for p in parts], 1) if self.n_recv else \
            torch.empty(0, sum(widths), dtype=wire_dtype, device=self.dev)
        back = torch.empty(self.n_send, sum(widths), dtype=wire_dtype, device=self.dev)
        self._all_to_all(back, send, self.send_splits, self.recv_splits)
        del send
        out, c = [], 0
        for p, w in zip(parts, widths):
            g = p[:self.nloc]
            for a, b in self._slices:
                g.index_put_((self.send_idx[a:b],), back[a:b, c:c + w].to(g.dtype), accumulate=True)
            out.append(g)
            c += w
        return out

    def bytes_per_exchange(self, width_bytes: int) -> Tuple[int, int]:
        """(bytes received, bytes sent) by this rank for one exchange of ``width_bytes`` rows."""
        return self.n_recv * width_bytes, self.n_send * width_bytes
