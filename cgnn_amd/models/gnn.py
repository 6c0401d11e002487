"""Pairwise Generative Neural Network (GNN.py:32-207).

For a pair (A, B) two generative models are fitted per run: A->B generates B
from [A, noise] with A clamped to the data, B->A the reverse; each is scored
by the mean test-phase MMD.  The returned value is
``(score_BA - score_AB) / (score_BA + score_AB)`` (GNN.py:207): positive means
A causes B.

All ``nb_runs x 2`` models of *all* pairs handed to ``predict_proba_batch`` are
trained together in one device batch (the reference runs them as separate TF
sessions in a joblib pool, GNN.py:193-194).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from ..engine.program import program_for_pair
from ..engine.scorer import Job, finite_mean, score_jobs, subsample
from ..utils.metrics import timer
from ..utils.philox import model_key
from ..utils.settings import SETTINGS
from .base import Pairwise_Model


def pair_jobs(a, b, idx, cfg, salt="gnn") -> List[Job]:
    """The 2 * nb_runs jobs of one pair: job 2r is A->B of run r, 2r+1 is B->A."""
    a = np.asarray(a, dtype=np.float64).reshape(-1, 1)
    b = np.asarray(b, dtype=np.float64).reshape(-1, 1)
    m = np.hstack((a, b)).astype(np.float32)
    prog = program_for_pair(cfg.h_layer_dim)
    jobs = []
    for run in range(cfg.nb_runs):
        mm = subsample(m, cfg.max_nb_points, cfg.seed, salt, idx, run)
        jobs.append(Job(prog, np.ascontiguousarray(mm.T), model_key(cfg.seed, salt, idx, run, 0)))
        jobs.append(Job(prog, np.ascontiguousarray(mm[:, ::-1].T), model_key(cfg.seed, salt, idx, run, 1)))
    return jobs


def pair_score(run_scores: np.ndarray, compat: bool = False) -> tuple:
    """(score A->B, score B->A, (BA - AB) / (BA + AB)).  Default: the mean of the finite
    runs (the reference's graph scores filter with np.isfinite, CGNN.py:217).
    ``compat`` (``SETTINGS.compat_scores``): the reference's pairwise mean over every
    run, a non-finite one propagating (GNN.py:196-197)."""
    mean = (lambda v: float(np.mean(v))) if compat else finite_mean
    ab = mean(run_scores[0::2])
    ba = mean(run_scores[1::2])
    return ab, ba, (ba - ab) / (ba + ab)


class GNN(Pairwise_Model):
    """Shallow generative networks modelling x->y and y->x with a 1-hidden
    layer network and an MMD loss; the better fit is the causal direction."""

    def __init__(self, backend="PyTorch", **kwargs):
        super(GNN, self).__init__()
        # Every backend string maps to the single native path.
        self.backend = backend
        self.kwargs = dict(kwargs)
        self.last_run_scores = None

    def _cfg(self, kwargs):
        kw = dict(self.kwargs)
        kw.update(kwargs)
        return SETTINGS.snapshot(**kw)

    def predict_proba_batch(self, pairs, **kwargs) -> List[float]:
        cfg = self._cfg(kwargs)
        jobs, spans = [], []
        for a, b, idx in pairs:
            js = pair_jobs(a, b, idx, cfg)
            spans.append((len(jobs), len(jobs) + len(js)))
            jobs.extend(js)
        with timer("pairwise"):
            scores = score_jobs(jobs, cfg)
        out, self.last_run_scores = [], []
        for s, e in spans:
            ab, ba, p = pair_score(scores[s:e], cfg.compat_scores)
            self.last_run_scores.append((scores[s:e:2].copy(), scores[s + 1:e:2].copy()))
            if cfg.verbose:
                print("score A->B %.6g  B->A %.6g  -> %.4f" % (ab, ba, p))
            out.append(p)
        return out

    def predict_proba(self, a, b, idx=0, **kwargs):
        return self.predict_proba_batch([(a, b, idx)], **kwargs)[0]


# ---------------------------------------------------------------- plug-in API
class GNN_model(object):
    """Single pairwise model with the reference's object API (GNN_tf,
    GNN.py:32-126): ``GNN_model(N, run, pair).train(data)`` then
    ``.evaluate(data)`` -> mean MMD.  ``data[:, 0]`` is the cause."""

    def __init__(self, N, run=0, pair=0, **kwargs):
        self.cfg = SETTINGS.snapshot(**kwargs)
        self.run, self.pair, self.N = run, pair, N
        self._trained = None

    def train(self, data, verbose=True, **kwargs):
        cfg = self.cfg.replace(**{k: v for k, v in kwargs.items() if hasattr(self.cfg, k)})
        self._trained = (np.asarray(data, dtype=np.float32), cfg)

    def evaluate(self, data, verbose=True, **kwargs):
        m, cfg = self._trained if self._trained else (np.asarray(data, dtype=np.float32), self.cfg)
        cfg = cfg.replace(**{k: v for k, v in kwargs.items() if hasattr(cfg, k)}, nb_runs=1)
        job = Job(program_for_pair(cfg.h_layer_dim), np.ascontiguousarray(m.T),
                  model_key(cfg.seed, "gnn", self.pair, self.run, 0))
        return float(score_jobs([job], cfg)[0])


def run_instance(m, idx, run, **kwargs):
    """Both directions of one run of one pair -> [XY, YX] (tf_run_instance, GNN.py:135-166)."""
    cfg = SETTINGS.snapshot(**kwargs).replace(nb_runs=1)
    m = np.asarray(m, dtype=np.float32)
    m = subsample(m, cfg.max_nb_points, cfg.seed, "gnn", idx, run)
    prog = program_for_pair(cfg.h_layer_dim)
    jobs = [Job(prog, np.ascontiguousarray(m.T), model_key(cfg.seed, "gnn", idx, run, 0)),
            Job(prog, np.ascontiguousarray(m[:, ::-1].T), model_key(cfg.seed, "gnn", idx, run, 1))]
    s = score_jobs(jobs, cfg)
    return [float(s[0]), float(s[1])]
