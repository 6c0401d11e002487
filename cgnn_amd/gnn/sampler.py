"""Device-resident neighbour sampling for mini-batch GNN training (GNN track,
not in the reference).

``DeviceSampler`` keeps the CSR in HBM and produces, for a batch of seed nodes,
one bipartite block per layer entirely on the GPU:

1. ``deg -> min(deg, fanout)`` counts and their prefix sum (PyTorch ops);
2. ``gnn_sample_neighbors`` (HIP, ``gnn_sampler.hip``): one thread per
   destination, Floyd's algorithm for ``fanout`` distinct picks, Philox keyed
   by (node, salt) -- the sample of a node is independent of the batch;
3. relabelling through a device map ``global id -> local id`` (a persistent
   int32 array of n entries, reset after each layer): destinations keep ids
   ``0..n_dst-1`` (they are the prefix of the sources), new sources get
   ``n_dst + rank`` in sorted-id order, so blocks are deterministic.

The host C++ sampler (``_rt.sample_neighbors``) remains for CPU training; this
one removes the host from the mini-batch loop (no sampling thread, no
host-to-device copies of blocks).  ``sample_reference`` is the same algorithm in
NumPy (tests).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from .. import native
from ..utils import philox
from ..utils.philox import model_key


def _st(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class DeviceBlock:
    """Bipartite block (GPU tensors): ``n_dst`` rows over ``n_src`` sources; the
    destinations are the first ``n_dst`` sources.  Same interface as ``sage.Block``."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, n_src: int):
        self.rowptr, self.col = rowptr, col
        self.n_dst = rowptr.numel() - 1
        self.n_src = int(n_src)
        deg = (rowptr[1:] - rowptr[:-1]).float()
        self.inv_deg = torch.where(deg > 0, 1.0 / deg.clamp_min(1), torch.zeros_like(deg))
        self._t = None

    def transposed(self):
        if self._t is None:
            from .sage import transpose_csr
            self._t = transpose_csr(self.rowptr, self.col, self.n_src)
        return self._t


class DeviceSampler:
    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, fanouts: Sequence[int], seed: int = 0):
        if not rowptr.is_cuda:
            raise ValueError("DeviceSampler needs the CSR on a GPU")
        self.rowptr, self.col = rowptr.contiguous(), col.contiguous()
        self.n = rowptr.numel() - 1
        self.fanouts = [int(f) for f in fanouts]
        if any(f > 64 or f < 1 for f in self.fanouts):
            raise ValueError("device sampler fanouts must be in 1..64")
        self.key = model_key(seed, "neighbour-sampler")
        # one spare entry (id n) absorbs the unused tail of the over-allocated pick buffer
        self.map = torch.full((self.n + 1,), -1, dtype=torch.int32, device=rowptr.device)
        self.flag = torch.zeros(self.n + 1, dtype=torch.bool, device=rowptr.device)

    def sample(self, seeds: torch.Tensor, salt: int) -> Tuple[List[DeviceBlock], torch.Tensor]:
        """Blocks ordered input layer first, and the input node ids (int64).

        One host synchronisation per layer (the number of new source nodes): the
        pick buffer is sized by the fanout bound and its unused tail points at the
        spare id n; the new sources are the set flags of a node bitmap, read back in
        increasing id order by ``nonzero`` -- a sort-free unique."""
        hip = native.hip()
        dev = self.rowptr.device
        nodes = seeds.to(device=dev, dtype=torch.int32).contiguous()
        blocks = []
        for layer, fo in enumerate(self.fanouts):
            nd = nodes.numel()
            nl = nodes.long()
            deg = self.rowptr[nl + 1] - self.rowptr[nl]
            cnt = deg.clamp(max=fo)
            optr = torch.zeros(nd + 1, dtype=torch.int32, device=dev)
            optr[1:] = torch.cumsum(cnt, 0)
            out = torch.full((max(nd * fo, 1),), self.n, dtype=torch.int32, device=dev)
            lsalt = (int(salt) * 16 + layer) & 0xFFFFFFFF
            hip.gnn_sample_neighbors(self.rowptr.data_ptr(), self.col.data_ptr(), nodes.data_ptr(), nd, fo,
                                     optr.data_ptr(), out.data_ptr(), int(self.key[0]), int(self.key[1]), lsalt,
                                     _st(nodes))
            ol = out.long()
            # relabel: destinations keep 0..nd-1, new sources follow in increasing id order
            self.flag[ol] = True
            self.flag[nl] = False
            self.flag[self.n] = False
            new = torch.nonzero(self.flag).flatten()        # the layer's one host sync
            total = int(optr[-1])                            # (queue already drained)
            self.flag[new] = False
            self.map[nl] = torch.arange(nd, dtype=torch.int32, device=dev)
            self.map[new] = torch.arange(nd, nd + new.numel(), dtype=torch.int32, device=dev)
            local = self.map[ol[:total]]
            src = torch.cat([nodes, new.to(torch.int32)])
            self.map[src.long()] = -1
            blocks.append(DeviceBlock(optr, local, src.numel()))
            nodes = src
        return blocks[::-1], nodes.long()


def sample_reference(rowptr: np.ndarray, col: np.ndarray, seeds: np.ndarray, fanouts: Sequence[int], salt: int,
                     seed: int = 0):
    """NumPy twin of ``DeviceSampler.sample`` (same draws, same relabelling);
    returns [(rowptr, local col, src nodes)] ordered from the seeds outwards."""
    k0, k1 = model_key(seed, "neighbour-sampler")
    nodes = np.asarray(seeds, dtype=np.int64)
    out_blocks = []
    for layer, fo in enumerate(fanouts):
        lsalt = (int(salt) * 16 + layer) & 0xFFFFFFFF
        rp = [0]
        picked = []
        for v in nodes:
            s, deg = int(rowptr[v]), int(rowptr[v + 1] - rowptr[v])
            if fo < 0 or deg <= fo:
                picked.extend(col[s:s + deg].tolist())
                rp.append(rp[-1] + deg)
                continue
            sel = []
            words = None
            for m, j in enumerate(range(deg - fo, deg)):
                if m % 4 == 0:
                    words = philox.philox4x32_10(np.uint32(v), np.uint32(lsalt), np.uint32(m // 4),
                                                 np.uint32(philox.RNG_SAMPLE), k0, k1)
                w = int(words[m % 4])
                t = (w * (j + 1)) >> 32
                sel.append(j if t in sel else t)
            picked.extend(int(col[s + q]) for q in sel)
            rp.append(rp[-1] + fo)
        picked = np.asarray(picked, dtype=np.int64)
        pos = {int(v): i for i, v in enumerate(nodes)}
        new = np.unique(np.asarray([p for p in picked if int(p) not in pos], dtype=np.int64))
        for i, v in enumerate(new):
            pos[int(v)] = len(nodes) + i
        local = np.asarray([pos[int(p)] for p in picked], dtype=np.int32)
        src = np.concatenate([nodes, new])
        out_blocks.append((np.asarray(rp, dtype=np.int32), local, src))
        nodes = src
    return out_blocks
