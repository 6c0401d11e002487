"""Structure searches over edge orientations, scored by a GraphEvaluator.

All searches share the reference signature ``(graph, data, run_cgnn_function,
**kwargs)`` (CGNN.py:198-327).  ``run_cgnn_function`` may be one of this
package's run functions (then candidates are scored in device batches) or any
user callable ``f(data, graph, idx, run, **kwargs) -> float`` (scored one run
at a time, like the reference's joblib plug-in).

* ``hill_climbing`` (CGNN.py:198-252): edges in ascending weight order; the
  first reversal that lowers the score is accepted immediately; repeat until a
  full pass makes no improvement.  Speculative batching evaluates the next k
  admissible candidates against the current graph at once and keeps the first
  improving one in edge order -- later results are discarded because they were
  computed against a graph that has since changed, so the
  acceptance sequence equals the sequential one.
* ``exploratory_hill_climbing`` (CGNN.py:255-312, broken in the reference, B2):
  implemented as intended -- reverse a random set of edges whose size decays
  quadratically over ``nb_loops`` loops, accept if the score improves.
* ``tabu_search`` (a stub raising in the reference, B3): best-admissible-move
  search over single reversals with a tabu list, aspiration and patience.

Every search takes ``checkpoint=<path>``: its state is written atomically (JSON)
after every evaluated batch / loop / iteration, and a later call with the same
path resumes from it (EHC draws loop ``k``'s random edge set from a stream keyed
by ``k``, so a resumed run makes the same draws as an uninterrupted one).
"""
from __future__ import annotations

import copy
import logging
from typing import Callable, Optional

import numpy as np

from ..engine.evaluator import GraphEvaluator
from ..utils.checkpoint import SearchCheckpoint, graph_from_dict, graph_to_dict, key_from_json, key_to_json
from ..utils.metrics import timer
from ..utils.philox import numpy_rng
from ..utils.settings import SETTINGS

log = logging.getLogger("cgnn_amd")


def _say(cfg, msg):
    if cfg.verbose:
        print(msg)
    log.info(msg)


def make_evaluator(data, run_cgnn_function, cfg, mode="dag", nodes=None, kwargs=None, graph=None):
    native = run_cgnn_function is None or getattr(run_cgnn_function, "_cgnn_native", False)
    mode = getattr(run_cgnn_function, "_cgnn_mode", mode)
    if mode == "confounders" and graph is not None and graph.skeleton:
        nodes = graph.skeleton.get_list_nodes()
    return GraphEvaluator(data, cfg, mode=mode, nodes=nodes,
                          legacy_fn=None if native else run_cgnn_function, legacy_kwargs=kwargs)


def hill_climbing(graph, data, run_cgnn_function=None, **kwargs):
    cfg = SETTINGS.snapshot(**kwargs)
    nodes = kwargs.get("nodes") or sorted(graph.get_list_nodes(), key=repr)
    ev = kwargs.get("evaluator") or make_evaluator(data, run_cgnn_function, cfg, "dag", nodes, kwargs, graph)
    width = int(kwargs.get("speculation", 0) or ev.speculation_width())
    ck = SearchCheckpoint(kwargs.get("checkpoint"), "HC")
    state = ck.load()
    if state:
        graph, tested, globalscore = state["graph"], state["tested"], state["best"]
        loop, i, improvement = state["loop"], state["position"], state["improvement"]
        list_edges = [list(e) for e in state["list_edges"]]
        resume_pass = True
        _say(cfg, "Resuming HC at loop %d, edge %d, score %s" % (loop, i, globalscore))
    else:
        tested = {graph.canonical_key()}
        with timer("search:initial_score"):
            globalscore = float(ev([graph])[0])
        loop, i, improvement, list_edges = 0, 0, False, []
        resume_pass = False
        _say(cfg, "Graph score : " + str(globalscore))
    while True:
        if not resume_pass:
            loop += 1
            improvement = False
            list_edges = graph.get_list_edges()
            i = 0
        resume_pass = False
        while i < len(list_edges):
            batch, j = [], i
            while j < len(list_edges) and len(batch) < width:
                edge = list_edges[j]
                tg = copy.deepcopy(graph)
                tg.reverse_edge(edge[0], edge[1])
                key = tg.canonical_key()
                if tg.is_cyclic() or key in tested:
                    _say(cfg, 'No Evaluation for {}'.format([edge]))
                else:
                    batch.append((j, edge, tg, key))
                j += 1
            if not batch:
                i = j
                continue
            with timer("search:candidates"):
                scores = ev([b[2] for b in batch])
            nxt = j
            for (jj, edge, tg, key), s in zip(batch, scores):
                tested.add(key)
                _say(cfg, 'Edge {} in evaluation : score {} (best {})'.format(edge, s, globalscore))
                if s < globalscore:
                    graph.reverse_edge(edge[0], edge[1])
                    improvement = True
                    globalscore = float(s)
                    _say(cfg, 'Edge {} got reversed !'.format(edge))
                    nxt = jj + 1
                    break
            i = nxt
            ck.save(graph, tested, best=globalscore, loop=loop, position=i,
                    list_edges=[[e[0], e[1], float(e[2])] for e in list_edges], improvement=improvement)
        if not improvement:
            break
    graph.search_score = globalscore
    return graph


def exploratory_hill_climbing(graph, data, run_cgnn_function=None, **kwargs):
    cfg = SETTINGS.snapshot(**kwargs)
    nb_loops = int(kwargs.get("nb_loops", 150))
    exploration_factor = int(kwargs.get("exploration_factor", 10))
    edges0 = graph.get_list_edges()
    if exploration_factor >= len(edges0):
        exploration_factor = max(1, len(edges0) - 1)
    nodes = kwargs.get("nodes") or sorted(graph.get_list_nodes(), key=repr)
    ev = kwargs.get("evaluator") or make_evaluator(data, run_cgnn_function, cfg, "dag", nodes, kwargs, graph)
    ck = SearchCheckpoint(kwargs.get("checkpoint"), "EHC")
    state = ck.load()
    if state:
        graph, tested, globalscore, first = state["graph"], state["tested"], state["best"], state["loop"] + 1
        _say(cfg, "Resuming EHC at loop %d, score %s" % (first, globalscore))
    else:
        tested = {graph.canonical_key()}
        with timer("search:initial_score"):
            globalscore = float(ev([graph])[0])
        first = 1
        _say(cfg, "Graph score : " + str(globalscore))
    max_tries = int(kwargs.get("max_tries", 200))
    for loop in range(first, nb_loops + 1):
        rng = numpy_rng(cfg.seed, "EHC", loop)
        list_edges = graph.get_list_edges()
        m = max(int(exploration_factor * ((nb_loops - loop) / nb_loops) ** 2), 1)
        cand = None
        for _ in range(max_tries):
            sel = rng.choice(len(list_edges), size=min(m, len(list_edges)), replace=False)
            tg = copy.deepcopy(graph)
            for k in sel:
                tg.reverse_edge(list_edges[k][0], list_edges[k][1])
            key = tg.canonical_key()
            if not tg.is_cyclic() and key not in tested:
                cand = (sel, tg, key)
                break
        if cand is not None:
            sel, tg, key = cand
            tested.add(key)
            with timer("search:candidates"):
                s = float(ev([tg])[0])
            _say(cfg, 'Reversed Edges {} : score {} (best {})'.format([list_edges[k][:2] for k in sel], s,
                                                                      globalscore))
            if s < globalscore:
                for k in sel:
                    graph.reverse_edge(list_edges[k][0], list_edges[k][1])
                globalscore = s
        ck.save(graph, tested, best=globalscore, loop=loop)
    graph.search_score = globalscore
    return graph


def tabu_search(graph, data, run_cgnn_function=None, **kwargs):
    """Tabu search over single-edge reversals.

    Each iteration scores every admissible reversal of the current graph in
    one batch and moves to the best one even if it is worse (escaping local
    minima); reversing an edge makes its pair tabu for ``tabu_tenure``
    iterations unless the move beats the best score seen (aspiration).  Stops
    after ``max_iter`` iterations or ``patience`` iterations without a new best.
    """
    cfg = SETTINGS.snapshot(**kwargs)
    tenure = int(kwargs.get("tabu_tenure", 5))
    max_iter = int(kwargs.get("max_iter", 50))
    patience = int(kwargs.get("patience", 5))
    nodes = kwargs.get("nodes") or sorted(graph.get_list_nodes(), key=repr)
    ev = kwargs.get("evaluator") or make_evaluator(data, run_cgnn_function, cfg, "dag", nodes, kwargs, graph)
    ck = SearchCheckpoint(kwargs.get("checkpoint"), "tabu")
    state = ck.load()
    if state:
        current, cur_score = state["graph"], state["current_score"]
        best, best_score = graph_from_dict(state["best_graph"]), state["best"]
        tabu = {frozenset(p): int(t) for p, t in state["tabu"]}
        cache = {key_from_json(k): float(v) for k, v in state["cache"]}
        stale, first = state["stale"], state["iteration"] + 1
        _say(cfg, "Resuming tabu search at iteration %d, best %s" % (first, best_score))
    else:
        current = copy.deepcopy(graph)
        with timer("search:initial_score"):
            cur_score = float(ev([current])[0])
        best, best_score = copy.deepcopy(current), cur_score
        tabu = {}
        cache = {current.canonical_key(): cur_score}
        stale, first = 0, 0
    for it in range(first, max_iter):
        moves = []
        for a, b, w in current.get_list_edges():
            tg = copy.deepcopy(current)
            tg.reverse_edge(a, b)
            if tg.is_cyclic():
                continue
            moves.append(((a, b), tg, tg.canonical_key()))
        todo = [m for m in moves if m[2] not in cache]
        if todo:
            with timer("search:candidates"):
                res = ev([m[1] for m in todo])
            for m, s in zip(todo, res):
                cache[m[2]] = float(s)
        choice = None
        for (a, b), tg, key in sorted(moves, key=lambda m: cache[m[2]]):
            s = cache[key]
            pair = frozenset((a, b))
            if tabu.get(pair, -1) >= it and not s < best_score:
                continue
            choice = ((a, b), tg, s, pair)
            break
        if choice is None:
            break
        (a, b), current, cur_score, pair = choice
        tabu[pair] = it + tenure
        _say(cfg, "tabu iter %d: reverse %s -> score %s" % (it, (a, b), cur_score))
        done = False
        if cur_score < best_score:
            best, best_score, stale = copy.deepcopy(current), cur_score, 0
        else:
            stale += 1
            done = stale >= patience
        ck.save(current, set(), current_score=cur_score, best=best_score, best_graph=graph_to_dict(best),
                tabu=[[sorted(p, key=repr), t] for p, t in tabu.items()],
                cache=[[key_to_json(k), v] for k, v in cache.items()], stale=stale,
                iteration=max_iter if done else it)
        if done:
            break
    # write the result into the caller's graph object, like the other searches
    for a, b, w in list(graph.get_list_edges(order_by_weight=False)):
        graph.remove_edge(a, b)
    for a, b, w in best.get_list_edges(order_by_weight=False):
        graph.add(a, b, w)
    graph.search_score = best_score
    return graph
