"""Score many generative models at once.

``score_jobs`` is the single execution entry point used by every model and
search (replacing each ``Parallel(n_jobs=NB_JOBS)(delayed(run_fn)(...))`` call
site listed in SURVEY §2.5): it takes a list of independent jobs (one job =
one run of one candidate graph on one data matrix), packs them into device
batches, spreads the batches over GPUs / ranks, and returns one score per job.

Failure handling: a non-finite score is kept as NaN and dropped
by :func:`finite_mean` exactly like the reference's ``np.isfinite`` filter;
``max_retries`` (``SETTINGS.max_retries`` / the ``max_retries`` kwarg of every
model and search entry point) re-trains such a job with a fresh RNG stream, and
``CGNN_FAULT=nan@job:k[,k...]`` injects failures (first attempt only) for tests.
With ``CGNN_PROFILE=1`` every call records a ``phase`` event ``score_jobs``.
"""
from __future__ import annotations

import dataclasses
import logging
import os
import time
from typing import Hashable, List, Optional, Sequence

import numpy as np

from ..parallel import dist as pdist
from ..utils import philox
from ..utils.metrics import METRICS, timer
from .program import Program

log = logging.getLogger("cgnn_amd")


@dataclasses.dataclass
class Job:
    program: Program
    data: np.ndarray              # [d, N] float32, already subsampled
    key: tuple                    # Philox key of this model


def subsample(mat: np.ndarray, max_points: Optional[int], seed: int, *salt) -> np.ndarray:
    """Per-run random subsample of the rows of [N, d] data (CGNN.py:183-185);
    ``max_points`` None keeps every row."""
    if max_points is None or mat.shape[0] <= max_points:
        return mat
    perm = philox.numpy_rng(seed, "subsample", *salt).permutation(mat.shape[0])
    return mat[perm[:int(max_points)]]


def finite_mean(values) -> float:
    v = np.asarray(values, dtype=np.float64)
    v = v[np.isfinite(v)]
    return float(v.mean()) if v.size else float("nan")


def _fault_indices():
    spec = os.environ.get("CGNN_FAULT", "")
    if not spec.startswith("nan@job:"):
        return set()
    return {int(x) for x in spec[len("nan@job:"):].split(",") if x.strip()}


def _group_batches(jobs: Sequence[Job], batch: int, H: Optional[int] = None):
    """Group compatible jobs (same [d, N]) into batches of at most `batch`.  With ``H``
    (device batches) also by generator-kernel family (engine.batch.kernel_family of each
    program alone), and a per-sample batch whose combined inputs / program length no
    longer fit that family is split: every model trains on the kernels it would get
    alone, so its score does not depend on the batch it lands in."""
    fam = None
    if H is not None:
        from .batch import kernel_family
        cache = {}

        def fam(p):
            k = (p.n_vars, p.max_in, len(p.prog))
            if k not in cache:
                cache[k] = kernel_family(p.n_vars, H, p.max_in, len(p.prog))
            return cache[k]
    groups = {}
    for i, j in enumerate(jobs):
        key = (j.program.n_vars, j.data.shape[1]) + ((fam(j.program),) if fam else ())
        groups.setdefault(key, []).append(i)
    out = []

    def emit(idx, family):
        if family == 1 and len(idx) > 1:
            p = [jobs[i].program for i in idx]
            from .batch import kernel_family
            if kernel_family(p[0].n_vars, H, max(q.max_in for q in p), max(len(q.prog) for q in p)) != 1:
                h = len(idx) // 2
                emit(idx[:h], family)
                emit(idx[h:], family)
                return
        out.append(idx)

    for key, idx in groups.items():
        for s in range(0, len(idx), batch):
            emit(idx[s:s + batch], key[2] if fam else None)
    return out


def _run_reference(jobs: Sequence[Job], idx, cfg) -> np.ndarray:
    from .reference import ReferenceTrainer
    tr = ReferenceTrainer([jobs[i].program for i in idx], [jobs[i].data for i in idx],
                          [jobs[i].key for i in idx], cfg.h_layer_dim,
                          learning_rate=cfg.learning_rate, init_std=cfg.init_std,
                          use_fast_mmd=cfg.use_Fast_MMD, nb_vectors=cfg.nb_vectors_approx_MMD)
    return tr.run(cfg.train_epochs, cfg.test_epochs, verbose=cfg.verbose)


def _device_batch_ok(jobs: Sequence[Job], idx, cfg) -> bool:
    """Whether the device kernels cover the batch ``idx``; if not (more variables than
    the widest compiled joint, or a generator whose forward or backward state does not
    fit in LDS) log it -- the caller trains the batch on the CPU reference path."""
    from .batch import device_supported
    d = jobs[idx[0]].program.n_vars
    max_in = max(jobs[i].program.max_in for i in idx)
    prog_len = max(len(jobs[i].program.prog) for i in idx)
    if device_supported(d, cfg.h_layer_dim, max_in, prog_len, fast_mmd=bool(cfg.use_Fast_MMD)):
        return True
    log.warning("CGNN batch of %d models (%d variables, h_layer_dim=%d, %d inputs per node) "
                "is outside the device kernels; training it on the CPU reference path",
                len(idx), d, cfg.h_layer_dim, max_in)
    METRICS.record("cpu_fallback", models=len(idx), variables=d, h_layer_dim=cfg.h_layer_dim)
    return False


def _run_local(jobs: Sequence[Job], cfg) -> np.ndarray:
    import torch
    n = len(jobs)
    scores = np.full(n, np.nan)
    if n == 0:
        return scores
    devices = pdist.devices_for(cfg)
    t0 = time.perf_counter()
    if devices:
        from .batch import DeviceTrainer
        batches = []
        for idx in _group_batches(jobs, max(1, cfg.batch_models), H=cfg.h_layer_dim):
            if _device_batch_ok(jobs, idx, cfg):
                batches.append(idx)
                continue
            scores[idx] = _run_reference(jobs, idx, cfg)
        pending = []
        for b, idx in enumerate(batches):
            dev = devices[b % len(devices)]
            tr = DeviceTrainer([jobs[i].program for i in idx], [jobs[i].data for i in idx],
                               [jobs[i].key for i in idx], cfg.h_layer_dim, dev,
                               learning_rate=cfg.learning_rate, init_std=cfg.init_std,
                               use_fast_mmd=cfg.use_Fast_MMD, nb_vectors=cfg.nb_vectors_approx_MMD,
                               record_history=cfg.train_epochs if cfg.verbose else 0)
            tr.launch(cfg.train_epochs, cfg.test_epochs)
            pending.append((idx, tr))
            # bound the number of in-flight batches per device (memory)
            if len(pending) >= 4 * len(devices):
                i0, t = pending.pop(0)
                scores[i0] = t.collect()
        for idx, tr in pending:
            scores[idx] = tr.collect()
            if cfg.verbose and tr.hist_len:
                h = tr.history()
                for r in range(tr.R):
                    for it in range(0, tr.hist_len, 100):
                        log.info('Run:%d, Iter:%d, score:%s', idx[r], it, h[r, it])
    else:
        for idx in _group_batches(jobs, max(1, cfg.batch_models)):
            scores[idx] = _run_reference(jobs, idx, cfg)
    dt = time.perf_counter() - t0
    steps = n * (cfg.train_epochs + cfg.test_epochs)
    METRICS.record("score_jobs", models=n, seconds=dt, model_steps=steps,
                   steps_per_s=steps / dt if dt > 0 else 0.0, devices=len(devices) or 0)
    return scores


def is_long(job: Job, cfg) -> bool:
    """Runs with more samples than ``cfg.long_n_min`` go to the sample-sharded trainer
    (the Fourier MMD is O(N) per sample already and stays on the batched engine)."""
    return (not cfg.use_Fast_MMD) and job.data.shape[1] > int(cfg.long_n_min)


def _run_long(jobs: Sequence[Job], cfg) -> np.ndarray:
    """Long-N jobs on ``engine.sharded.SampleShardedTrainer``: EVERY rank takes part in
    every job, owning an equal block of its samples (the reference would subsample to
    1500, CGNN.py:183-185); scores come back identical on all ranks.  N is trimmed to a
    multiple of the rank count (at most world - 1 trailing samples, a warning)."""
    import torch
    from .sharded import SampleShardedTrainer, shard_range
    n = len(jobs)
    scores = np.full(n, np.nan)
    world, rank = pdist.world_size(), pdist.rank()
    devices = pdist.devices_for(cfg)
    dev = devices[0] if devices else torch.device("cpu")
    t0 = time.perf_counter()
    for idx in _group_batches(jobs, max(1, cfg.batch_models), H=cfg.h_layer_dim if devices else None):
        if devices and not _device_batch_ok(jobs, idx, cfg):
            # every rank trains the whole job on the fp64 CPU reference (same scores on
            # every rank: no exchange needed)
            scores[idx] = _run_reference(jobs, idx, cfg)
            continue
        N = jobs[idx[0]].data.shape[1]
        Nw = N - N % world
        if Nw != N:
            log.warning("long-N jobs: %d samples over %d ranks, the last %d are not used", N, world, N - Nw)
        r0, nl = shard_range(Nw, rank, world)
        tr = SampleShardedTrainer([jobs[i].program for i in idx],
                                  [np.ascontiguousarray(jobs[i].data[:, r0:r0 + nl]) for i in idx],
                                  [jobs[i].key for i in idx], cfg.h_layer_dim, dev, Nw,
                                  learning_rate=cfg.learning_rate, init_std=cfg.init_std)
        scores[idx] = tr.run(cfg.train_epochs, cfg.test_epochs)
    dt = time.perf_counter() - t0
    steps = n * (cfg.train_epochs + cfg.test_epochs)
    METRICS.record("score_jobs_long_n", models=n, seconds=dt, model_steps=steps, ranks=world,
                   steps_per_s=steps / dt if dt > 0 else 0.0)
    return scores


def score_jobs(jobs: Sequence[Job], cfg, max_retries: Optional[int] = None) -> np.ndarray:
    """One score per job (mean test-phase loss); NaN for non-finite runs."""
    with timer("score_jobs"):
        return _score_jobs(jobs, cfg, cfg.max_retries if max_retries is None else int(max_retries))


def _score_jobs(jobs: Sequence[Job], cfg, max_retries: int, ids=None) -> np.ndarray:
    # ids: the callers' job numbers of ``jobs`` (fault injection addresses those, also
    # when a mixed short / long call recurses on its short subset)
    ids = list(range(len(jobs))) if ids is None else list(ids)
    faults = _fault_indices()
    long_idx = [i for i, j in enumerate(jobs) if is_long(j, cfg)]
    if long_idx:
        # long-N jobs: every rank trains every job on its block of samples
        out = np.full(len(jobs), np.nan)
        long_set = set(long_idx)
        short_idx = [i for i in range(len(jobs)) if i not in long_set]
        if short_idx:
            out[short_idx] = _score_jobs([jobs[i] for i in short_idx], cfg, max_retries,
                                         ids=[ids[i] for i in short_idx])
        ls = _run_long([jobs[i] for i in long_idx], cfg)
        for k, i in enumerate(long_idx):
            if ids[i] in faults:
                ls[k] = np.nan
        for attempt in range(max_retries):
            bad = [k for k in range(len(long_idx)) if not np.isfinite(ls[k])]
            if not bad:
                break
            retry = [Job(jobs[long_idx[k]].program, jobs[long_idx[k]].data,
                         philox.model_key(jobs[long_idx[k]].key[0], jobs[long_idx[k]].key[1], "retry", attempt))
                     for k in bad]
            ls[bad] = _run_long(retry, cfg)
            METRICS.record("retried_runs", attempt=attempt + 1, count=len(bad),
                           recovered=int(np.isfinite(ls[bad]).sum()))
        out[long_idx] = ls
        dropped = int((~np.isfinite(ls)).sum())
        if dropped:
            METRICS.record("dropped_runs", count=dropped, total=len(long_idx))
        return out
    n = len(jobs)
    idx = pdist.shard_indices(n)
    local = _run_local([jobs[i] for i in idx], cfg) if len(idx) else np.zeros(0)
    for k, i in enumerate(idx):
        if ids[int(i)] in faults:
            local[k] = np.nan
    for attempt in range(max_retries):
        bad = [k for k in range(len(idx)) if not np.isfinite(local[k])]
        if not bad:
            break
        retry = []
        for k in bad:
            j = jobs[idx[k]]
            retry.append(Job(j.program, j.data, philox.model_key(j.key[0], j.key[1], "retry", attempt)))
        local[bad] = _run_local(retry, cfg)
        METRICS.record("retried_runs", attempt=attempt + 1, count=len(bad),
                       recovered=int(np.isfinite(local[bad]).sum()))
    scores = pdist.combine_scores(n, idx, local)
    dropped = int((~np.isfinite(scores)).sum())
    if dropped:
        METRICS.record("dropped_runs", count=dropped, total=n)
    return scores
