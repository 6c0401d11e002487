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

import ctypes
import weakref
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import native
from ..utils import philox
from ..utils.philox import model_key


def _st(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class DeviceBlock:
    """Bipartite block (GPU tensors): ``n_dst`` rows over ``n_src`` sources; the
    destinations are the first ``n_dst`` sources.  Same interface as ``sage.Block``.
    ``inv_deg`` / ``transposed`` may be given precomputed (the pipelined sampler
    builds both on the device)."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, n_src: int, inv_deg=None, transposed=None,
                 gcol=None):
        self.rowptr, self.col = rowptr, col
        # global ids of the sources of every edge (= ids[col] for the block's source id
        # list), when the sampler has them: the pipelined one keeps its picks
        self.gcol = gcol
        self.n_dst = rowptr.numel() - 1
        self.n_src = int(n_src)
        if inv_deg is None:
            deg = (rowptr[1:] - rowptr[:-1]).float()
            inv_deg = torch.where(deg > 0, 1.0 / deg.clamp_min(1), torch.zeros_like(deg))
        self.inv_deg = inv_deg
        self._t = transposed

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


# priority of the sampler's stream.  With two batches sampled ahead the sampling is off
# the critical path, and a normal-priority stream leaves the training kernels first
# pick of the CUs: 10.21 / 10.30 epochs/s against 10.12 / 9.99 at high priority
# (tools/ab_sage_prio.py, profiles/r05_sage/ab_sage_prio.log)
STREAM_PRIORITY = 0


class _Slot:
    """Device buffers of one in-flight mini-batch (upper-bound sizes)."""

    def __init__(self, dev, n, batch, fanouts, need_t, publish):
        i32 = dict(dtype=torch.int32, device=dev)
        self.nd_max = []
        nd = batch
        for fo in fanouts:
            self.nd_max.append(nd)
            nd = min(nd * (fo + 1), n)
        self.optr, self.inv, self.picks, self.local, self.src = [], [], [], [], []
        self.rp_t, self.col_t, self.cnt_t = [], [], []
        for l, fo in enumerate(fanouts):
            ndm = self.nd_max[l]
            smax = min(ndm * (fo + 1), n)
            self.optr.append(torch.zeros(ndm + 1, **i32))
            self.inv.append(torch.zeros(ndm, dtype=torch.float32, device=dev))
            self.picks.append(torch.zeros(max(ndm * fo, 1), **i32))
            self.local.append(torch.zeros(max(ndm * fo, 1), **i32))
            self.src.append(torch.zeros(smax, **i32))
            if need_t[l]:
                self.rp_t.append(torch.zeros(smax + 1, **i32))
                self.col_t.append(torch.zeros(max(ndm * fo, 1), **i32))
                # zero between batches: the pipeline's last kernel clears what it counted
                self.cnt_t.append(torch.zeros(smax, **i32))
            else:
                self.rp_t.append(None)
                self.col_t.append(None)
                self.cnt_t.append(None)
        self.counts = torch.zeros(2 * len(fanouts), **i32)
        self.host_ptr = 0         # device address of the mapped counts (publish), else 0
        if publish:
            # page-locked, device-mapped host memory the pipeline's last kernel writes the
            # level sizes to: no copy call per batch
            hip = native.hip()
            h, d = hip.host_mapped_alloc(4 * 2 * len(fanouts))
            weakref.finalize(self, hip.host_mapped_free, h)
            self.counts_host = torch.from_numpy(np.ctypeslib.as_array(
                (ctypes.c_int32 * (2 * len(fanouts))).from_address(h)))
            self.host_ptr = d
        else:
            self.counts_host = torch.zeros(2 * len(fanouts), dtype=torch.int32).pin_memory()
        self.done = torch.cuda.Event()      # the sampling of this slot's batch finished
        self.free = torch.cuda.Event()      # the training that read this slot finished
        self.widx = -1                      # the slot's index in the native worker
        self.keep = None                    # what a posted job refers to (events, seeds)
        self.pending = None                 # the SampledBatch last enqueued into this slot


class SampledBatch:
    """A mini-batch whose blocks are being sampled on the side stream; ``resolve()``
    waits for that work only and returns (blocks input layer first, input node ids
    int32) with host-known sizes."""

    def __init__(self, slot, fanouts, n_seeds, waiter=None):
        self.slot, self.fanouts, self.n_seeds = slot, fanouts, n_seeds
        self.waiter = waiter      # (worker handle, job sequence number): threaded sampler
        self._res = None

    def resolve(self):
        if self._res is None:
            sl = self.slot
            if self.waiter is not None:
                # the worker issued the job and its sampling finished; the current stream
                # is ordered after it
                h, seq = self.waiter
                native.hip().gnn_sw_wait(h, seq, sl.widx, torch.cuda.current_stream(sl.counts.device).cuda_stream)
            else:
                sl.done.synchronize()
            c = sl.counts_host.tolist()          # a copy: the slot is refilled later
            blocks = []
            nd = self.n_seeds
            for l in range(len(self.fanouts)):
                n_src, total = int(c[2 * l]), int(c[2 * l + 1])
                t = None
                if sl.rp_t[l] is not None:
                    t = (sl.rp_t[l][:n_src + 1], sl.col_t[l][:total])
                blocks.append(DeviceBlock(sl.optr[l][:nd + 1], sl.local[l][:total], n_src,
                                          inv_deg=sl.inv[l][:nd], transposed=t, gcol=sl.picks[l][:total]))
                nd = n_src
            self._res = (blocks[::-1], sl.src[-1][:nd])
        return self._res


class PipelinedSampler:
    """The whole multi-level sampling of a mini-batch as ONE native call
    (``gnn_sample_blocks``: 7 HIP kernels per level, 11 with the transposed CSR --
    16 before round 6 -- device-side row counts, no host synchronisation inside) on a
    side stream, over ``slots``
    buffers: batch k + 1 (and k + 2) is sampled while batch k trains.  The level
    sizes reach the host through mapped host memory a kernel writes (``publish``;
    else one pinned copy per batch).  Same draws and relabelling as
    :class:`DeviceSampler` (bitwise equal blocks); the transposed CSRs the backward
    needs (every block but the input layer's) are built on the device too,
    deterministically (histogram, scan, scatter, per-bucket sort).

    A slot waits only for the training that last read it (``consumed``) and for the
    event the caller says its seeds are ready at (``enqueue(ready=...)``), not for
    the whole main stream: with three slots, the sampling of batch k + 1 starts
    while batch k - 1 still trains, and is done before the host asks for it
    (profiles/r05_sage).

    ``threaded`` (default): a native worker thread owns the side stream and issues the
    launches (``gnn_sw_*`` in gnn_sampler.hip); the Python thread only posts the batch,
    so the ~30 sampling launches no longer add to the host time of the training loop.

    Capturing each slot's pipeline as a hipGraph (seed count and salt read on the
    device) was tried in round 5: the uncaptured launches pass the bitwise test, the
    replayed graph faulted (illegal address) on the first replay; not kept."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, fanouts: Sequence[int], batch: int, seed: int = 0,
                 slots: int = 3, publish: bool = True, threaded: bool = True):
        if not rowptr.is_cuda:
            raise ValueError("PipelinedSampler needs the CSR on a GPU")
        if slots < 2:
            raise ValueError("the pipelined sampler needs at least two slots")
        self.rowptr, self.col = rowptr.contiguous(), col.contiguous()
        self.dev = rowptr.device
        self.n = rowptr.numel() - 1
        self.fanouts = [int(f) for f in fanouts]
        if any(f > 64 or f < 1 for f in self.fanouts):
            raise ValueError("device sampler fanouts must be in 1..64")
        self.batch = int(batch)
        self.publish = bool(publish)
        self.key = model_key(seed, "neighbour-sampler")
        L = len(self.fanouts)
        need_t = [l < L - 1 for l in range(L)]
        self.slots = [_Slot(self.dev, self.n, self.batch, self.fanouts, need_t, self.publish) for _ in range(slots)]
        # padded to whole 4096-id blocks (the flag passes read 16 flags per thread)
        self.flag = torch.zeros(native.hip().gnn_sample_flag_bytes(self.n), dtype=torch.uint8, device=self.dev)
        self.map = torch.zeros(self.n + 1, dtype=torch.int32, device=self.dev)
        ns = native.hip().gnn_sample_blocks_scratch(self.n, self.fanouts, self.slots[0].nd_max)
        self.bscratch = torch.zeros(ns, dtype=torch.int32, device=self.dev)
        # stream priority (STREAM_PRIORITY; -1 = high, 0 = normal)
        self.stream = torch.cuda.Stream(device=self.dev, priority=STREAM_PRIORITY)
        self._next = 0
        self._w = None
        if threaded:
            if not self.publish:
                raise ValueError("the threaded sampler needs publish=True (no copy on its stream)")
            hip = native.hip()
            p = lambda ts: [t.data_ptr() if t is not None else 0 for t in ts]
            dev_index = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
            self._w = hip.gnn_sw_create(dev_index, self.stream.cuda_stream, self.rowptr.data_ptr(),
                                        self.col.data_ptr(), self.n, self.fanouts, self.slots[0].nd_max,
                                        self.flag.data_ptr(), self.map.data_ptr(), self.bscratch.data_ptr(),
                                        int(self.key[0]), int(self.key[1]))
            # runs before the buffers are released: joins the thread, drains the stream
            weakref.finalize(self, hip.gnn_sw_destroy, self._w)
            for sl in self.slots:
                sl.widx = hip.gnn_sw_add_slot(self._w, p(sl.optr), p(sl.inv), p(sl.picks), p(sl.local), p(sl.src),
                                              p(sl.rp_t), p(sl.col_t), p(sl.cnt_t), sl.counts.data_ptr(),
                                              sl.host_ptr)

    def enqueue(self, seeds: torch.Tensor, salt: int, ready: Optional[torch.cuda.Event] = None) -> SampledBatch:
        """Start sampling ``seeds`` (int32 device tensor, <= batch) on the side stream.
        ``ready``: an event after which the seeds are valid (default: everything enqueued
        on the current stream so far)."""
        if seeds.numel() > self.batch:
            raise ValueError("more seeds than the sampler's batch bound")
        from ..utils import checks
        if checks.enabled():
            checks.index(seeds, self.n, "sample_blocks seeds")
            checks.csr(self.rowptr, self.col, self.n, "sample_blocks graph", n_rows=self.n)
        sl = self.slots[self._next]
        if sl.pending is not None and sl.pending._res is None:
            # the slot's previous batch was never resolved: refilling it would overwrite
            # blocks a caller may still read and, in threaded mode, free the ready event
            # (sl.keep) before the worker has issued the earlier job's wait on it
            raise RuntimeError("PipelinedSampler.enqueue: more than %d batches outstanding; resolve() "
                               "the oldest before enqueueing another" % len(self.slots))
        self._next = (self._next + 1) % len(self.slots)
        main = torch.cuda.current_stream(self.dev)
        seeds = seeds.to(dtype=torch.int32).contiguous()
        if self._w is not None:
            if ready is None:
                ready = torch.cuda.Event()
                ready.record(main)
            sl.keep = (ready, seeds)          # alive until the job is issued (and resolved)
            seeds.record_stream(self.stream)
            seq = native.hip().gnn_sw_submit(self._w, sl.widx, seeds.data_ptr(), int(seeds.numel()),
                                             int(salt) & 0xFFFFFFFF, [ready.cuda_event, sl.free.cuda_event])
            sl.pending = SampledBatch(sl, self.fanouts, int(seeds.numel()), waiter=(self._w, seq))
            return sl.pending
        p = lambda ts: [t.data_ptr() if t is not None else 0 for t in ts]
        with torch.cuda.stream(self.stream):
            if ready is None:
                self.stream.wait_stream(main)
            else:
                self.stream.wait_event(ready)
            # the slot's previous batch has trained (no-op before the first record)
            self.stream.wait_event(sl.free)
            native.hip().gnn_sample_blocks(
                self.rowptr.data_ptr(), self.col.data_ptr(), self.n, seeds.data_ptr(), int(seeds.numel()),
                self.fanouts, sl.nd_max, p(sl.optr), p(sl.inv), p(sl.picks), p(sl.local), p(sl.src), p(sl.rp_t),
                p(sl.col_t), p(sl.cnt_t), sl.counts.data_ptr(), self.flag.data_ptr(), self.map.data_ptr(),
                self.bscratch.data_ptr(), int(self.key[0]), int(self.key[1]), int(salt) & 0xFFFFFFFF,
                self.stream.cuda_stream, counts_host=sl.host_ptr)
            if not self.publish:
                sl.counts_host.copy_(sl.counts, non_blocking=True)
            sl.done.record(self.stream)
            seeds.record_stream(self.stream)
        sl.pending = SampledBatch(sl, self.fanouts, int(seeds.numel()))
        return sl.pending

    def consumed(self, batch: SampledBatch):
        """Mark the end of the training that reads ``batch`` (enqueued on the current
        stream): the slot may be refilled after it."""
        main = torch.cuda.current_stream(self.dev)
        main.wait_event(batch.slot.done)
        batch.slot.free.record(main)
