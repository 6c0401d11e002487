"""Process groups, device placement and work sharding.

The reference's only parallelism is an ensemble of independent runs executed by
a joblib process pool, placed round-robin on ``/gpu:(GPU_OFFSET + run % NB_GPU)``
(GNN.py:158-163, CGNN.py:187-191).  Here the same work (runs x
candidates x pairs) is sharded two ways:

* **in-process multi-GPU**: one Python process enqueues independent model
  batches on several devices (every device has its own stream; launches are
  asynchronous hipGraph replays, so one host thread keeps 8 GPUs busy);
* **one process per GPU** (``torchrun``): every rank scores the jobs with
  ``index % world_size == rank`` and the per-job scores are combined with one
  ``all_reduce`` (each index is owned by exactly one rank, so a SUM is an
  all-gather) -- RCCL over xGMI on GPUs, gloo on CPUs.

Scores depend only on (seed, run, salt) through the counter-based RNG, never
on the rank or device, so results are identical for 1, 2, 4 or 8 GPUs.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional, Sequence

import numpy as np
import torch


def is_distributed() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    import torch.distributed as dist
    return dist.get_rank() if is_distributed() else 0


def world_size() -> int:
    import torch.distributed as dist
    return dist.get_world_size() if is_distributed() else 1


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_process_group(backend: Optional[str] = None, timeout_s: int = 1800):
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/MASTER_ADDR...).

    backend defaults to "nccl" (= RCCL on ROCm) when GPUs are visible, else gloo.
    """
    import torch.distributed as dist
    if dist.is_initialized():
        return
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local_rank() % max(torch.cuda.device_count(), 1))
    dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))


def barrier():
    import torch.distributed as dist
    if is_distributed():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def devices_for(cfg) -> List[torch.device]:
    """GPU list for in-process sharding (reference: GPU_OFFSET + run % NB_GPU)."""
    if not (cfg.gpu and torch.cuda.is_available()):
        return []
    n_avail = torch.cuda.device_count()
    if is_distributed():
        return [torch.device("cuda", torch.cuda.current_device())]
    if cfg.device_ids:
        ids = [i for i in cfg.device_ids if i < n_avail]
    else:
        ids = [i for i in range(cfg.gpu_offset, cfg.gpu_offset + max(cfg.nb_gpu, 1)) if i < n_avail]
    if not ids:
        ids = [0]
    return [torch.device("cuda", i) for i in ids]


def shard_indices(n: int) -> np.ndarray:
    """Indices of the jobs this rank computes (round-robin over ranks)."""
    return np.arange(rank(), n, world_size())


def combine_scores(n: int, idx: np.ndarray, local: np.ndarray) -> np.ndarray:
    """All-gather per-job scores: each rank contributes its shard, SUM-reduce."""
    if not is_distributed():
        out = np.full(n, np.nan)
        out[idx] = local
        return out
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    buf = torch.zeros(n, dtype=torch.float64, device=dev)
    own = torch.zeros(n, dtype=torch.float64, device=dev)
    if len(idx):
        buf[torch.as_tensor(idx, device=dev)] = torch.as_tensor(np.nan_to_num(local, nan=0.0, posinf=0.0, neginf=0.0),
                                                                 dtype=torch.float64, device=dev)
        bad = ~np.isfinite(local)
        if bad.any():
            own[torch.as_tensor(idx[bad], device=dev)] = 1.0
    dist.all_reduce(buf)
    dist.all_reduce(own)
    out = buf.cpu().numpy()
    out[own.cpu().numpy() > 0] = np.nan
    return out


def host_cpus() -> int:
    """CPUs this process may run on (its affinity set, not the machine's count)."""
    return len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 8)


def set_host_threads(n: Optional[int] = None) -> int:
    """Threads of the host C++ runtime (graph generation, reorder, partition).  Default:
    this rank's share of the node's CPUs -- torch.distributed.run pins OMP_NUM_THREADS=1,
    which would leave the setup of every rank single-threaded.  Returns the count set."""
    from .. import native
    if n is None:
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", str(world_size())))
        n = max(1, host_cpus() // max(lw, 1))
    native.rt().set_num_threads(int(n))
    return int(n)


def broadcast_host_array(arr: Optional[np.ndarray], n: int, dtype=np.int64, src: int = 0,
                         chunk_bytes: int = 256 << 20) -> np.ndarray:
    """Broadcast a 1-D host array of ``n`` elements from rank ``src`` (the other ranks
    pass None).  Over RCCL it travels through one device staging buffer of at most
    ``chunk_bytes`` (a 111 M-entry partition order is 0.9 GB); over gloo directly.
    A status word goes first: if ``src`` has no valid array (None, or the wrong shape
    -- e.g. the pass that should have produced it raised), EVERY rank raises instead
    of the others blocking in the data broadcast until the collective times out."""
    if not is_distributed():
        return np.asarray(arr)
    import torch.distributed as dist
    tdt = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32,
           np.dtype(np.float32): torch.float32}[np.dtype(dtype)]
    nccl = dist.get_backend() == "nccl"
    sdev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    ok = rank() != src or (arr is not None and np.shape(arr) == (n,))
    status = torch.tensor([1 if ok else 0], dtype=torch.int64, device=sdev)
    dist.broadcast(status, src)
    if int(status.item()) != 1:
        held = None if arr is None else np.shape(arr)
        raise RuntimeError("broadcast_host_array: source rank %d has no valid array (holds %s, expected (%d,))"
                           % (src, held if rank() == src else "?", n))
    out = np.asarray(arr, dtype=dtype) if rank() == src else np.empty(n, dtype=dtype)
    host = torch.from_numpy(out)
    if not nccl:
        dist.broadcast(host, src)
        return out
    per = max(1, chunk_bytes // out.itemsize)
    stage = torch.empty(min(per, n), dtype=tdt, device=torch.device("cuda", torch.cuda.current_device()))
    for a in range(0, n, per):
        b = min(n, a + per)
        if rank() == src:
            stage[:b - a].copy_(host[a:b])
        dist.broadcast(stage[:b - a], src)
        if rank() != src:
            host[a:b].copy_(stage[:b - a])
    torch.cuda.synchronize()
    return out

