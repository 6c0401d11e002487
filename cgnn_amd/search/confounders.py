"""Hill climbing with hidden confounders (CGNN_confounders.py:219-383).

Score = mean finite run score + ``complexity_graph_param * #edges``.  For every
skeleton edge, in skeleton order:

* oriented in the graph: try the reversal, then try removing the (possibly
  reversed) edge; an edge whose removal improves the score is labelled a
  possible confounder, otherwise its weight becomes the score increase its
  removal would cause (:262-317);
* absent (removed earlier): try adding u->v and v->u and keep the better one
  if it improves the score (:320-381).

Loop until a full pass brings no improvement.  Candidates that do not depend
on each other's outcome are scored in one batch: the reversal and the removal
of the current orientation, and the two additions.  The removal of the
*reversed* edge is scored afterwards only if the reversal was accepted.

``checkpoint=<path>``: the search state (graph, tested configurations, best
score, confounder labels, pass number and position in the skeleton) is written
atomically after every skeleton edge; a later call with the same path resumes
at the next edge (the reference's 95-candidate example run restarts from zero).
"""
from __future__ import annotations

import copy
import logging

from ..utils.checkpoint import SearchCheckpoint
from ..utils.metrics import timer
from ..utils.settings import SETTINGS
from .hill_climbing import _say, make_evaluator

log = logging.getLogger("cgnn_amd")


def hill_climbing_confounders(graph, data, run_cgnn_function=None, **kwargs):
    cfg = SETTINGS.snapshot(**kwargs)
    skel = graph.skeleton
    if not skel:
        raise ValueError("hill_climbing_confounders needs DirectedGraph(skeleton=...)")
    nodes = skel.get_list_nodes()
    ev = kwargs.get("evaluator") or make_evaluator(data, run_cgnn_function, cfg, "confounders", nodes, kwargs)
    ck = SearchCheckpoint(kwargs.get("checkpoint"), "HC-confounders")
    state = ck.load()
    skel_edges = skel.get_list_edges_without_duplicate()
    if state:
        graph, tested, globalscore = state["graph"], state["tested"], state["best"]
        confounders = {frozenset(c) for c in state["confounders"]}
        loop, start, improvement = state["loop"], state["position"], state["improvement"]
        skel = graph.skeleton
        _say(cfg, "Resuming confounder HC at pass %d, skeleton edge %d, score %s" % (loop, start, globalscore))
    else:
        tested = {graph.canonical_key()}
        with timer("search:initial_score"):
            globalscore = float(ev([graph])[0])
        _say(cfg, "Graph score : " + str(globalscore))
        confounders = set()
        loop, start, improvement = 1, 0, False
    while True:
        for pos in range(start, len(skel_edges)):
            u, v = skel_edges[pos]
            if graph.has_edge(u, v) or graph.has_edge(v, u):
                n1, n2 = (u, v) if graph.has_edge(u, v) else (v, u)
                # --- reversal and removal of the current orientation, together
                rev = copy.deepcopy(graph)
                rev.reverse_edge(n1, n2)
                rem = copy.deepcopy(graph)
                rem.remove_edge(n1, n2)
                cands = []
                rev_ok = not rev.is_cyclic() and rev.canonical_key() not in tested
                rem_ok = rem.canonical_key() not in tested
                if rev_ok:
                    cands.append(("rev", rev))
                if rem_ok:
                    cands.append(("rem", rem))
                scores = dict(zip([c[0] for c in cands], ev([c[1] for c in cands]))) if cands else {}
                if rev_ok:
                    tested.add(rev.canonical_key())
                    s = float(scores["rev"])
                    _say(cfg, "Reverse edge %s -> %s : %s (best %s)" % (n1, n2, s, globalscore))
                    if s < globalscore:
                        graph.reverse_edge(n1, n2)
                        improvement = True
                        globalscore = s
                        n1, n2 = n2, n1
                        _say(cfg, "Edge %s -> %s got reversed !" % (n2, n1))
                        # the removal candidate above removed the old orientation;
                        # removing either orientation gives the same graph
                # removal of the (possibly reversed) edge: same graph either way
                rem_key = rem.canonical_key()
                if rem_ok:
                    tested.add(rem_key)
                    s = float(scores["rem"])
                    if s < globalscore:
                        graph.remove_edge(n1, n2)
                        improvement = True
                        globalscore = s
                        confounders.add(frozenset((n1, n2)))
                        _say(cfg, "Edge %s -> %s got removed, possible confounder !" % (n1, n2))
                    else:
                        graph.set_weight(n1, n2, s - globalscore)
                        _say(cfg, "Edge %s -> %s not removed. Score edge : %s" % (n1, n2, s - globalscore))
                else:
                    _say(cfg, "Removing already evaluated for edge %s -> %s" % (n1, n2))
            else:
                a_g = copy.deepcopy(graph)
                a_g.add(u, v)
                b_g = copy.deepcopy(graph)
                b_g.add(v, u)
                cands = []
                for tag, g in (("uv", a_g), ("vu", b_g)):
                    if not g.is_cyclic() and g.canonical_key() not in tested:
                        cands.append((tag, g))
                s_uv = s_vu = 9999.0
                if cands:
                    res = dict(zip([c[0] for c in cands], ev([c[1] for c in cands])))
                    for tag, g in cands:
                        tested.add(g.canonical_key())
                    s_uv = float(res.get("uv", 9999.0))
                    s_vu = float(res.get("vu", 9999.0))
                if s_uv < globalscore and s_uv < s_vu:
                    graph.add(u, v, globalscore - s_uv)
                    globalscore = s_uv
                    improvement = True
                    confounders.discard(frozenset((u, v)))
                    _say(cfg, "Edge %s -> %s is added !" % (u, v))
                elif s_vu < globalscore and s_vu < s_uv:
                    graph.add(v, u, globalscore - s_vu)
                    globalscore = s_vu
                    improvement = True
                    confounders.discard(frozenset((u, v)))
                    _say(cfg, "Edge %s -> %s is added !" % (v, u))
                else:
                    _say(cfg, "Edge not added, possible confounder %s <-> %s" % (u, v))
                    confounders.add(frozenset((u, v)))
            ck.save(graph, tested, best=globalscore, loop=loop, position=pos + 1, improvement=improvement,
                    confounders=sorted([sorted(c, key=repr) for c in confounders], key=repr))
        if not improvement:
            break
        loop, start, improvement = loop + 1, 0, False
        ck.save(graph, tested, best=globalscore, loop=loop, position=0, improvement=False,
                confounders=sorted([sorted(c, key=repr) for c in confounders], key=repr))
    graph.search_score = globalscore
    graph.confounders = sorted(tuple(sorted(c, key=repr)) for c in confounders)
    return graph
