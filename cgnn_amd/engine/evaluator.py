"""Batched scoring of candidate causal graphs on a fixed dataset.

``GraphEvaluator(data, cfg)(graphs)`` returns, for every candidate graph, the
mean over ``nb_runs`` runs of the trained generator's test MMD -- the
quantity each ``Parallel(...)(delayed(run_cgnn_function)(...))`` site of the
reference computes for ONE graph (CGNN.py:214-217, CGNN_confounders.py:234-237).
Here all candidates x runs are one device batch.

Common random numbers (default): run r of every candidate uses the same Philox
key and the same subsample, so score differences between candidates are not
polluted by independent noise, and a candidate's score does not depend on which
other candidates share its batch (speculative evaluation stays exact).
``cfg.compat_scores``: every candidate draws runs of its own, as the reference
does (each ``Parallel(...)`` call re-seeds, CGNN.py:237-238): keys and subsamples
are keyed by the candidate's canonical edge set -- independent across candidates,
still independent of the batch.

User ``run_cgnn_function`` plug-ins (the reference's module-level TF functions) run
one call per (candidate, run) on the host; ``cfg.nb_jobs`` > 1 spreads the calls over
that many joblib worker processes, like the reference's ``Parallel(n_jobs=NB_JOBS)``
(plug-ins must be picklable, module-level callables, as there).
"""
from __future__ import annotations

import hashlib

from typing import Callable, Optional, Sequence

import numpy as np

from ..utils.metrics import METRICS
from ..utils.philox import model_key
from .program import program_for_confounders, program_for_dag
from .scorer import Job, finite_mean, score_jobs, subsample


class GraphEvaluator:
    def __init__(self, data, cfg, mode: str = "dag", nodes=None, salt: str = "cgnn",
                 legacy_fn: Optional[Callable] = None, legacy_kwargs=None):
        if mode not in ("dag", "confounders"):
            raise ValueError(mode)
        self.cfg = cfg
        self.mode = mode
        self.salt = salt
        self.data = data
        self.nodes = list(nodes) if nodes is not None else list(data.columns)
        mat = np.asarray(data[self.nodes].values, dtype=np.float32)
        self.subs = [np.ascontiguousarray(subsample(mat, cfg.max_nb_points, cfg.seed, salt, run).T)
                     for run in range(cfg.nb_runs)]
        self.keys = [model_key(cfg.seed, salt, run) for run in range(cfg.nb_runs)]
        self.legacy_fn = legacy_fn
        self.legacy_kwargs = dict(legacy_kwargs or {})
        self.n_evaluated = 0

    def program(self, graph):
        if self.mode == "confounders":
            return program_for_confounders(graph, self.cfg.h_layer_dim)
        return program_for_dag(graph, self.cfg.h_layer_dim, nodes=self.nodes)

    def penalty(self, graph) -> float:
        if self.mode == "confounders":
            return self.cfg.complexity_graph_param * graph.number_of_edges()
        return 0.0

    def candidate_salt(self, graph) -> int:
        """Stable 64-bit identity of a candidate's edge set (compat_scores keys)."""
        h = hashlib.blake2b(repr(graph.canonical_key()).encode(), digest_size=8).digest()
        return int.from_bytes(h, "little")

    def _runs(self, graph):
        """(data, key) of every run of ``graph``: shared by all candidates, or the
        candidate's own under compat_scores."""
        if not self.cfg.compat_scores:
            return list(zip(self.subs, self.keys))
        c = self.candidate_salt(graph)
        mat = np.asarray(self.data[self.nodes].values, dtype=np.float32)
        return [(np.ascontiguousarray(subsample(mat, self.cfg.max_nb_points, self.cfg.seed, self.salt, c, run).T),
                 model_key(self.cfg.seed, self.salt, c, run)) for run in range(self.cfg.nb_runs)]

    def run_scores(self, graphs: Sequence) -> np.ndarray:
        """[len(graphs), nb_runs] raw per-run scores."""
        R = self.cfg.nb_runs
        if self.legacy_fn is not None:
            calls = [(self.n_evaluated + g, graph, run) for g, graph in enumerate(graphs) for run in range(R)]
            if self.cfg.nb_jobs > 1:
                from joblib import Parallel, delayed
                vals = Parallel(n_jobs=self.cfg.nb_jobs)(
                    delayed(self.legacy_fn)(self.data, graph, idx, run, **self.legacy_kwargs)
                    for idx, graph, run in calls)
            else:
                vals = [self.legacy_fn(self.data, graph, idx, run, **self.legacy_kwargs) for idx, graph, run in calls]
            return np.asarray(vals, dtype=np.float64).reshape(len(graphs), R)
        jobs = []
        for graph in graphs:
            prog = self.program(graph)
            for data, key in self._runs(graph):
                jobs.append(Job(prog, data, key))
        return score_jobs(jobs, self.cfg).reshape(len(graphs), R)

    def __call__(self, graphs: Sequence) -> np.ndarray:
        graphs = list(graphs)
        if not graphs:
            return np.zeros(0)
        raw = self.run_scores(graphs)
        scores = np.array([finite_mean(raw[g]) + self.penalty(gr) for g, gr in enumerate(graphs)])
        self.n_evaluated += len(graphs)
        METRICS.record("candidates", count=len(graphs), total=self.n_evaluated,
                       best=float(np.nanmin(scores)) if np.isfinite(scores).any() else None)
        return scores

    def speculation_width(self) -> int:
        """How many candidates to evaluate together (fills one device batch)."""
        import torch
        from ..parallel import dist as pdist
        n_dev = max(len(pdist.devices_for(self.cfg)), 1) * pdist.world_size()
        per_batch = max(1, self.cfg.batch_models // max(self.cfg.nb_runs, 1))
        return max(1, per_batch * n_dev)
