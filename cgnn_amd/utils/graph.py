"""Causal-graph data structures.

Behavioural parity with the reference (Code/cgnn/utils/Graph.py:29-434):

* ``Graph`` stores ``{src: {dst: weight}}`` (Graph.py:32-48) and can be built
  from an edge DataFrame (optional 3rd column = weight, Graph.py:44-61) or
  from a square adjacency DataFrame thresholded at 0.001 (Graph.py:37-43).
* ``get_list_nodes`` returns nodes in first-seen order over sources and their
  targets (Graph.py:95-110); ``get_list_edges`` sorts by ascending weight with
  the edge itself as tie-breaker (Graph.py:112-138).
* ``DirectedGraph`` adds cycle detection / enumeration, edge reversal and the
  two cycle breakers (Graph.py:198-377); ``UndirectedGraph`` is symmetric
  (Graph.py:380-434).

Deliberate fixes:

* B5  ``remove_cycles`` compares the cycle count of the *reversed* test graph
  (the reference compares ``self`` with itself and therefore always deletes);
  ``compat=True`` (or ``SETTINGS.compat_remove_cycles``) restores the
  reference behaviour.
* B6  ``remove_node`` works on Python 3.
* B13 a node that loses its last edge stays in the graph: the node registry is
  explicit, so the generative model never silently drops a variable.
* B11 ``canonical_key`` gives an order-independent hashable identity of the
  edge set, used by the searches instead of comparing dicts of lists.

Cycle detection and the DFS helpers are iterative (no recursion limit on
200+-node generator graphs).
"""
from __future__ import annotations

import copy
from collections import defaultdict
from typing import Dict, Hashable, Iterable, List, Optional, Sequence, Tuple

import numpy as np

Node = Hashable


def list_to_dict(links):
    """Convert ``[["V0","V3"], ...]`` edge names into ``{0: [3], 3: []}``.

    Parity: Graph.py:13-26 (unused by the reference itself).
    """
    dic = defaultdict(list)
    for src, dst in links:
        a, b = int(str(src)[1:]), int(str(dst)[1:])
        dic[a].append(b)
        if b not in dic:
            dic[b] = []
    return dic


class Graph(object):
    """Base class: weighted adjacency ``{src: {dst: weight}}`` + node registry."""

    def __init__(self, df=None, adjacency_matrix=False):
        self._graph: Dict[Node, Dict[Node, float]] = defaultdict(dict)
        self._nodes: Dict[Node, None] = {}
        if df is None:
            return
        connections = []
        if adjacency_matrix:
            data = np.asarray(df.values, dtype=float)
            cols = list(df.columns)
            n = data.shape[0]
            for i in range(n):
                for j in range(n):
                    if i != j and data[i, j] > 0.001:
                        connections.append([cols[i], cols[j], data[i, j]])
        else:
            for row in df.itertuples(index=False):
                connections.append(list(row))
        self.add_multiple_edges(connections)

    # ------------------------------------------------------------------ build
    def add_multiple_edges(self, connections):
        """Add ``(cause, effect[, weight])`` rows (Graph.py:50-61)."""
        for row in connections:
            row = list(row)
            if len(row) < 2:
                raise ValueError("edge rows need at least two entries: %r" % (row,))
            if len(row) == 2:
                self.add(row[0], row[1])
            else:
                self.add(row[0], row[1], row[2])

    def _register(self, *nodes):
        for n in nodes:
            if n not in self._nodes:
                self._nodes[n] = None

    def add(self, node1, node2, weight=1):
        raise NotImplementedError

    def remove_edge(self, node1, node2):
        raise NotImplementedError

    def add_node(self, node):
        """Register an isolated node (new; makes B13 explicit)."""
        self._register(node)
        return self

    # ----------------------------------------------------------------- query
    def get_parents(self, node):
        """Sources with an edge into ``node``, in source order (Graph.py:82-93)."""
        return [src for src, succ in self._graph.items() if node in succ]

    def get_children(self, node):
        return list(self._graph.get(node, {}).keys())

    def get_list_nodes(self):
        """First-seen order over sources and their targets (Graph.py:95-110),
        followed by registered nodes that currently have no edge (B13)."""
        seen: Dict[Node, None] = {}
        for src, succ in self._graph.items():
            if src not in seen:
                seen[src] = None
            for dst in succ:
                if dst not in seen:
                    seen[dst] = None
        for n in self._nodes:
            if n not in seen:
                seen[n] = None
        return list(seen)

    def _edges_and_weights(self):
        edges, weights = [], []
        for src, succ in self._graph.items():
            for dst, w in succ.items():
                edges.append([src, dst])
                weights.append(w)
        return edges, weights

    def get_list_edges(self, order_by_weight=True, descending=False, return_weights=True):
        """Edges, by default in ascending weight order (Graph.py:112-138).

        Ties are broken by the edge ``[src, dst]`` itself, as in the reference
        (``sorted(zip(weights, edges))``).
        """
        edges, weights = self._edges_and_weights()
        if order_by_weight and edges:
            order = sorted(range(len(edges)), key=lambda k: (weights[k], _sortable(edges[k])),
                           reverse=descending)
            edges = [edges[k] for k in order]
            weights = [weights[k] for k in order]
        if return_weights:
            return [[e[0], e[1], w] for e, w in zip(edges, weights)]
        return edges

    def get_adjacency_matrix(self):
        """``(matrix, nodes)`` with ``matrix[cause, effect] = weight`` (Graph.py:140-158)."""
        nodes = self.get_list_nodes()
        index = {n: k for k, n in enumerate(nodes)}
        m = np.zeros((len(nodes), len(nodes)))
        for src, dst, w in self.get_list_edges(order_by_weight=False):
            m[index[src], index[dst]] = w
        return m, nodes

    def get_dict_nw(self):
        """Unweighted ``{node: [children]}`` (Graph.py:160-174)."""
        out: Dict[Node, List[Node]] = {}
        for src, succ in self._graph.items():
            out.setdefault(src, [])
            for dst in succ:
                out[src].append(dst)
                out.setdefault(dst, [])
        return out

    def canonical_key(self) -> Tuple:
        """Order-independent identity of the (unweighted) edge set (fix for B11)."""
        return tuple(sorted((repr(s), repr(d)) for s, succ in self._graph.items() for d in succ))

    def number_of_edges(self) -> int:
        return sum(len(s) for s in self._graph.values())

    def remove_node(self, node):
        """Remove every reference to ``node`` (fixed Graph.py:176-192, B6)."""
        for src in list(self._graph):
            self._graph[src].pop(node, None)
        self._graph.pop(node, None)
        for src in [s for s, succ in self._graph.items() if not succ]:
            del self._graph[src]
        self._nodes.pop(node, None)

    def copy(self):
        return copy.deepcopy(self)

    def __eq__(self, other):
        if not isinstance(other, Graph):
            return NotImplemented
        return type(self) is type(other) and self.canonical_key() == other.canonical_key()

    def __hash__(self):
        return hash((type(self).__name__, self.canonical_key()))

    def __str__(self):
        return '{}({})'.format(self.__class__.__name__, dict(self._graph))

    __repr__ = __str__


def _sortable(edge):
    """Sort key for an edge that tolerates mixed node types."""
    try:
        (edge[0] < edge[1]) or (edge[1] < edge[0])
        return tuple(edge)
    except TypeError:
        return tuple(repr(x) for x in edge)


class DirectedGraph(Graph):
    """Directed weighted graph (Graph.py:198-377)."""

    def __init__(self, df=None, adjacency_matrix=False, skeleton=False):
        self.skeleton = skeleton
        super(DirectedGraph, self).__init__(df, adjacency_matrix)
        if skeleton:
            self._register(*skeleton.get_list_nodes())

    def add(self, node1, node2, weight=1):
        """Add or update ``node1 -> node2`` (Graph.py:206-216)."""
        self._graph[node1][node2] = weight
        self._register(node1, node2)
        return self

    def remove_edge(self, node1, node2):
        """Graph.py:284-292; the nodes stay registered (B13)."""
        del self._graph[node1][node2]
        if len(self._graph[node1]) == 0:
            del self._graph[node1]

    def reverse_edge(self, node1, node2, weight=None):
        """``node1 -> node2`` becomes ``node2 -> node1`` (Graph.py:269-282).

        As in the reference a falsy ``weight`` keeps the old weight.
        """
        if not weight:
            weight = self._graph[node1][node2]
        self.remove_edge(node1, node2)
        self.add(node2, node1, weight)

    def set_weight(self, node1, node2, weight):
        """Graph.py:353-360."""
        self._graph[node1][node2] = weight

    def has_edge(self, node1, node2) -> bool:
        return node1 in self._graph and node2 in self._graph[node1]

    # ------------------------------------------------------------- cycles
    def is_cyclic(self):
        """True iff the graph has a directed cycle (Graph.py:218-242).

        Iterative three-colour DFS, same visiting order as the reference.
        """
        g = self.get_dict_nw()
        WHITE, GREY, BLACK = 0, 1, 2
        colour = {v: WHITE for v in g}
        for root in g:
            if colour[root] != WHITE:
                continue
            stack = [(root, iter(g[root]))]
            colour[root] = GREY
            while stack:
                v, it = stack[-1]
                nxt = next(it, None)
                if nxt is None:
                    colour[v] = BLACK
                    stack.pop()
                elif colour[nxt] == GREY:
                    return True
                elif colour[nxt] == WHITE:
                    colour[nxt] = GREY
                    stack.append((nxt, iter(g[nxt])))
        return False

    def topological_order(self, nodes: Optional[Sequence[Node]] = None) -> List[Node]:
        """Kahn order that mirrors the reference's generation sweep
        (CGNN.py:63-84: repeatedly scan ``nodes`` and emit every node whose
        parents are all generated).  Raises on a cycle."""
        nodes = list(self.get_list_nodes() if nodes is None else nodes)
        parents = {v: set(self.get_parents(v)) for v in nodes}
        done: Dict[Node, None] = {}
        while len(done) < len(nodes):
            progressed = False
            for v in nodes:
                if v not in done and parents[v].issubset(done):
                    done[v] = None
                    progressed = True
            if not progressed:
                raise ValueError("graph is cyclic; no topological order")
        return list(done)

    def cycles(self):
        """Every simple cycle, as ``[start, ..., start]`` (Graph.py:244-267)."""
        g = self.get_dict_nw()

        def dfs(start, end):
            fringe = [(start, [])]
            while fringe:
                state, path = fringe.pop()
                if path and state == end:
                    yield path
                    continue
                for nxt in g[state]:
                    if nxt in path:
                        continue
                    fringe.append((nxt, path + [nxt]))

        return [[node] + path for node in g for path in dfs(node, node) if path]

    def remove_cycles(self, verbose=True, compat=None):
        """Break cycles by acting on their lowest-weight edge (Graph.py:294-322).

        For the first listed cycle, the lowest-weight edge on it is reversed if
        that strictly reduces the number of cycles, otherwise deleted.  With
        ``compat=True`` the reference's comparison (B5) is reproduced, which
        always deletes.
        """
        if compat is None:
            from .settings import SETTINGS
            compat = SETTINGS.compat_remove_cycles
        ordered = self.get_list_edges(return_weights=False)
        while self.is_cyclic():
            cc = self.cycles()
            s_cycle = cc[0]
            hops = [s_cycle[i:i + 2] for i in range(len(s_cycle) - 1)]
            r_edge = next(e for e in ordered if e in hops)
            test_graph = copy.deepcopy(self)
            test_graph.reverse_edge(r_edge[0], r_edge[1])
            n_after = len(self.cycles()) if compat else len(test_graph.cycles())
            if n_after < len(cc):
                self.reverse_edge(r_edge[0], r_edge[1])
                if verbose:
                    print('Link {} got reversed !'.format(r_edge))
            else:
                self.remove_edge(r_edge[0], r_edge[1])
                if verbose:
                    print('Link {} got deleted !'.format(r_edge))
            ordered = [e for e in self.get_list_edges(return_weights=False)]

    def remove_cycle_without_deletion(self):
        """Reverse the DFS back-edges of a snapshot (Graph.py:324-351).

        Visits vertices in the snapshot's order; every edge that closes onto
        the current DFS path is reversed in ``self``.  Always yields a DAG.
        """
        g = self.get_dict_nw()
        visited = set()
        for root in g:
            if root in visited:
                continue
            visited.add(root)
            path = {root}
            stack = [(root, iter(g.get(root, ())))]
            while stack:
                v, it = stack[-1]
                nxt = next(it, None)
                if nxt is None:
                    path.discard(v)
                    stack.pop()
                    continue
                if nxt in path:
                    self.reverse_edge(v, nxt)
                elif nxt not in visited:
                    visited.add(nxt)
                    path.add(nxt)
                    stack.append((nxt, iter(g.get(nxt, ()))))

    def get_correlation_matrix(self, sigma):
        """Identity plus ``sigma`` on skeleton edges (Graph.py:362-377)."""
        nodes = self.skeleton.get_list_nodes()
        index = {n: k for k, n in enumerate(nodes)}
        m = np.eye(len(nodes))
        for a, b in self.skeleton.get_list_edges_without_duplicate():
            m[index[a], index[b]] = sigma
            m[index[b], index[a]] = sigma
        return m


class UndirectedGraph(Graph):
    """Symmetric weighted graph (Graph.py:380-434)."""

    def __init__(self, df=None, adjacency_matrix=False):
        super(UndirectedGraph, self).__init__(df, adjacency_matrix)

    def add(self, node1, node2, weight=1):
        self._graph[node1][node2] = weight
        self._graph[node2][node1] = weight
        self._register(node1, node2)
        return self

    def remove_edge(self, node1, node2):
        del self._graph[node1][node2]
        del self._graph[node2][node1]
        if len(self._graph[node1]) == 0:
            del self._graph[node1]
        if node2 in self._graph and len(self._graph[node2]) == 0:
            del self._graph[node2]

    def get_neighbors(self, node):
        """Graph.py:413-420 (implemented through ``get_parents``)."""
        return self.get_parents(node)

    def get_list_edges_without_duplicate(self):
        """Each undirected edge once, in first-seen orientation (Graph.py:422-434)."""
        seen = set()
        out = []
        for src, succ in self._graph.items():
            for dst in succ:
                key = (dst, src)
                if key in seen:
                    continue
                seen.add((src, dst))
                out.append([src, dst])
        return out
