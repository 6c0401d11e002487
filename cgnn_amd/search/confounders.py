"""Hill climbing with hidden confounders (CGNN_confounders.py:219-383).

Score = mean finite run score + ``complexity_graph_param * #edges``.  For every
skeleton edge, in skeleton order:

* oriented in the graph: try the reversal, then try removing the (possibly
  reversed) edge; an edge whose removal improves the score is labelled a
  possible confounder, otherwise its weight becomes the score increase its
  removal would cause (:262-317);
* absent (removed earlier): try adding u->v and v->u and keep the better one
  if it improves the score (:320-381).

Loop until a full pass brings no improvement.  Speculative batching: the
candidates of the next skeleton edges (reversal + removal, or the two additions)
are built against the current graph and scored in ONE device batch (up to the
evaluator's speculation width, e.g. 256 models / 32 runs = 8 candidates); the
decisions are replayed in skeleton order and the window stops at the first
structural change.  Scores depend only on (seed, run) (common random numbers),
so the accepted sequence is exactly the sequential one.  (Removing the reversed
edge gives the same graph as removing the original orientation, so one removal
candidate covers both outcomes of the reversal test.)

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
    width = int(kwargs.get("speculation", 0) or ev.speculation_width())

    def plan(pos):
        """Candidates of skeleton edge ``pos`` against the current graph."""
        u, v = skel_edges[pos]
        it = {"pos": pos, "u": u, "v": v, "cands": []}
        if graph.has_edge(u, v) or graph.has_edge(v, u):
            n1, n2 = (u, v) if graph.has_edge(u, v) else (v, u)
            it.update(kind="present", n1=n1, n2=n2)
            rev = copy.deepcopy(graph)
            rev.reverse_edge(n1, n2)
            rem = copy.deepcopy(graph)
            rem.remove_edge(n1, n2)
            it["rev_ok"] = not rev.is_cyclic() and rev.canonical_key() not in tested
            it["rem_ok"] = rem.canonical_key() not in tested
            it["rem_key"] = rem.canonical_key()
            if it["rev_ok"]:
                it["cands"].append(["rev", rev, rev.canonical_key(), None])
            if it["rem_ok"]:
                it["cands"].append(["rem", rem, it["rem_key"], None])
        else:
            it["kind"] = "absent"
            a_g = copy.deepcopy(graph)
            a_g.add(u, v)
            b_g = copy.deepcopy(graph)
            b_g.add(v, u)
            for tag, g in (("uv", a_g), ("vu", b_g)):
                if not g.is_cyclic() and g.canonical_key() not in tested:
                    it["cands"].append([tag, g, g.canonical_key(), None])
        return it

    def process(it):
        """The reference's sequential decision for one edge (scores precomputed);
        returns whether the graph's structure changed."""
        nonlocal globalscore, improvement
        sc = {c[0]: c[3] for c in it["cands"]}
        for c in it["cands"]:
            tested.add(c[2])
        changed = False
        if it["kind"] == "present":
            n1, n2 = it["n1"], it["n2"]
            if it["rev_ok"]:
                s = float(sc["rev"])
                _say(cfg, "Reverse edge %s -> %s : %s (best %s)" % (n1, n2, s, globalscore))
                if s < globalscore:
                    graph.reverse_edge(n1, n2)
                    improvement = changed = True
                    globalscore = s
                    n1, n2 = n2, n1
                    _say(cfg, "Edge %s -> %s got reversed !" % (n2, n1))
            # removal of the (possibly reversed) edge: the same graph either way
            if it["rem_ok"]:
                s = float(sc["rem"])
                if s < globalscore:
                    graph.remove_edge(n1, n2)
                    improvement = changed = True
                    globalscore = s
                    confounders.add(frozenset((n1, n2)))
                    _say(cfg, "Edge %s -> %s got removed, possible confounder !" % (n1, n2))
                else:
                    graph.set_weight(n1, n2, s - globalscore)
                    _say(cfg, "Edge %s -> %s not removed. Score edge : %s" % (n1, n2, s - globalscore))
            else:
                _say(cfg, "Removing already evaluated for edge %s -> %s" % (n1, n2))
        else:
            u, v = it["u"], it["v"]
            s_uv = float(sc["uv"]) if "uv" in sc else 9999.0
            s_vu = float(sc["vu"]) if "vu" in sc else 9999.0
            if s_uv < globalscore and s_uv < s_vu:
                graph.add(u, v, globalscore - s_uv)
                globalscore = s_uv
                improvement = changed = True
                confounders.discard(frozenset((u, v)))
                _say(cfg, "Edge %s -> %s is added !" % (u, v))
            elif s_vu < globalscore and s_vu < s_uv:
                graph.add(v, u, globalscore - s_vu)
                globalscore = s_vu
                improvement = changed = True
                confounders.discard(frozenset((u, v)))
                _say(cfg, "Edge %s -> %s is added !" % (v, u))
            else:
                _say(cfg, "Edge not added, possible confounder %s <-> %s" % (u, v))
                confounders.add(frozenset((u, v)))
        return changed

    def save(position):
        ck.save(graph, tested, best=globalscore, loop=loop, position=position, improvement=improvement,
                confounders=sorted([sorted(c, key=repr) for c in confounders], key=repr))

    while True:
        pos = start
        while pos < len(skel_edges):
            # speculation: the candidates of the next edges against the current graph, scored
            # in one batch (scores depend on (seed, run) only, not on the batch); decisions are
            # then replayed in skeleton order, and the window ends at the first structural
            # change -- later edges' candidates were built on the old graph
            window, ncand = [], 0
            j = pos
            while j < len(skel_edges) and (not window or ncand + 2 <= width):
                it = plan(j)
                window.append(it)
                ncand += len(it["cands"])
                j += 1
            flat = [c for it in window for c in it["cands"]]
            if flat:
                with timer("search:candidates"):
                    scores = ev([c[1] for c in flat])
                for c, s_ in zip(flat, scores):
                    c[3] = s_
            for it in window:
                changed = process(it)
                pos = it["pos"] + 1
                save(pos)
                if changed:
                    break
        if not improvement:
            break
        loop, start, improvement = loop + 1, 0, False
        save(0)
    graph.search_score = globalscore
    graph.confounders = sorted(tuple(sorted(c, key=repr)) for c in confounders)
    return graph
