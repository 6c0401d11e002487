"""Observability and evaluation metrics.

* ``METRICS`` -- structured JSONL event log (SURVEY §5 "Metrics / logging"):
  enabled by ``CGNN_METRICS=<path>``; every event is one JSON line with a
  timestamp.  ``METRICS.events`` also keeps them in memory for tests.
* ``timer`` -- per-phase wall-clock timings when ``CGNN_PROFILE=1``.
* causal-discovery scores: structural Hamming distance, precision/recall of
  oriented edges, pairwise sign accuracy, AUPR of a ranked edge list.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from typing import Dict, Iterable, List, Sequence, Tuple


class MetricsLog:
    def __init__(self):
        self.events: List[dict] = []
        self._lock = threading.Lock()
        self.path = os.environ.get("CGNN_METRICS")
        self.keep = int(os.environ.get("CGNN_METRICS_KEEP", "10000"))

    def record(self, event: str, **fields):
        rec = {"ts": time.time(), "event": event}
        rec.update(fields)
        with self._lock:
            self.events.append(rec)
            if len(self.events) > self.keep:
                del self.events[: len(self.events) - self.keep]
            if self.path:
                with open(self.path, "a") as f:
                    f.write(json.dumps(rec, default=float) + "\n")

    def last(self, event: str):
        for rec in reversed(self.events):
            if rec["event"] == event:
                return rec
        return None

    def clear(self):
        with self._lock:
            self.events.clear()


METRICS = MetricsLog()


@contextlib.contextmanager
def timer(name: str, sync_cuda: bool = True):
    """Record the wall time of a phase when CGNN_PROFILE=1."""
    if os.environ.get("CGNN_PROFILE") != "1":
        yield
        return
    import torch
    if sync_cuda and torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if sync_cuda and torch.cuda.is_available():
            torch.cuda.synchronize()
        METRICS.record("phase", name=name, seconds=time.perf_counter() - t0)


# ------------------------------------------------------------ causal metrics
def _edge_set(graph_or_edges) -> set:
    if hasattr(graph_or_edges, "get_list_edges"):
        return {(a, b) for a, b in graph_or_edges.get_list_edges(order_by_weight=False, return_weights=False)}
    return {(e[0], e[1]) for e in graph_or_edges}


def shd(pred, target, double_for_anticausal=False) -> int:
    """Structural Hamming distance between two directed edge sets.

    Missing / extra edges cost 1; a reversed edge costs 1 (or 2 with
    ``double_for_anticausal``, the cdt convention)."""
    P, T = _edge_set(pred), _edge_set(target)
    cost = 0
    seen = set()
    for (a, b) in P | T:
        key = frozenset((a, b))
        if key in seen:
            continue
        seen.add(key)
        in_p = {(x, y) for (x, y) in ((a, b), (b, a)) if (x, y) in P}
        in_t = {(x, y) for (x, y) in ((a, b), (b, a)) if (x, y) in T}
        if in_p == in_t:
            continue
        if in_p and in_t:
            cost += 2 if double_for_anticausal else 1
        else:
            cost += 1
    return cost


def orientation_scores(pred, target) -> Dict[str, float]:
    P, T = _edge_set(pred), _edge_set(target)
    tp = len(P & T)
    return {"tp": tp, "precision": tp / len(P) if P else 0.0,
            "recall": tp / len(T) if T else 0.0, "n_pred": len(P), "n_true": len(T)}


def sign_accuracy(predictions: Sequence[float], targets: Sequence[float]) -> float:
    ok = [(p > 0) == (t > 0) for p, t in zip(predictions, targets)]
    return sum(ok) / len(ok) if ok else 0.0


def aupr(scored_edges: Iterable[Tuple], target) -> float:
    """Average precision of edges ranked by descending score vs a target edge set."""
    T = _edge_set(target)
    ranked = sorted(scored_edges, key=lambda e: -e[2])
    hits, ap = 0, 0.0
    for k, (a, b, _) in enumerate(ranked, 1):
        if (a, b) in T:
            hits += 1
            ap += hits / k
    return ap / len(T) if T else 0.0
