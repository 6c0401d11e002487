"""Graph utilities: behavioural parity with Code/cgnn/utils/Graph.py and the
documented fixes."""
import itertools
import random

import numpy as np
import pandas as pd
import pytest

from cgnn_amd.utils.graph import DirectedGraph, UndirectedGraph, list_to_dict


def dag(edges):
    g = DirectedGraph()
    for e in edges:
        g.add(*e)
    return g


def test_edge_dataframe_with_and_without_weights():
    df = pd.DataFrame({"Cause": ["V0", "V1"], "Effect": ["V1", "V2"]})
    g = DirectedGraph(df)
    assert g.get_list_edges(order_by_weight=False) == [["V0", "V1", 1], ["V1", "V2", 1]]
    df = pd.DataFrame({"a": ["V0", "V1"], "b": ["V1", "V2"], "w": [0.5, 0.2]})
    g = DirectedGraph(df)
    assert g.get_list_edges() == [["V1", "V2", 0.2], ["V0", "V1", 0.5]]


def test_adjacency_matrix_constructor_threshold():
    m = pd.DataFrame([[0, 0.5, 0.0005], [0, 0, 1.0], [0, 0, 0]], columns=["a", "b", "c"])
    g = DirectedGraph(m, adjacency_matrix=True)
    assert sorted(g.get_list_edges(order_by_weight=False, return_weights=False)) == [["a", "b"], ["b", "c"]]
    mat, nodes = g.get_adjacency_matrix()
    assert nodes == ["a", "b", "c"]
    assert mat[0, 1] == 0.5 and mat[1, 2] == 1.0


def test_list_nodes_first_seen_order_and_parents():
    g = dag([("B", "A"), ("C", "A"), ("A", "D")])
    assert g.get_list_nodes() == ["B", "A", "C", "D"]
    assert g.get_parents("A") == ["B", "C"]
    assert g.get_dict_nw() == {"B": ["A"], "A": ["D"], "C": ["A"], "D": []}


def test_edges_sorted_by_weight_then_edge():
    g = DirectedGraph()
    g.add("b", "c", 0.5)
    g.add("a", "c", 0.5)
    g.add("x", "y", 0.1)
    assert g.get_list_edges() == [["x", "y", 0.1], ["a", "c", 0.5], ["b", "c", 0.5]]
    assert g.get_list_edges(descending=True)[0] == ["b", "c", 0.5]
    assert g.get_list_edges(return_weights=False)[0] == ["x", "y"]


def test_cycles_and_reverse():
    g = dag([("a", "b"), ("b", "c"), ("c", "a")])
    assert g.is_cyclic()
    cyc = g.cycles()
    assert ["a", "b", "c", "a"] in cyc
    g.reverse_edge("c", "a")
    assert not g.is_cyclic()
    assert g.get_parents("c") == ["b", "a"] or set(g.get_parents("c")) == {"a", "b"}


def test_reverse_keeps_weight_unless_given():
    g = dag([("a", "b", 0.7)])
    g.reverse_edge("a", "b")
    assert g.get_list_edges() == [["b", "a", 0.7]]
    g.reverse_edge("b", "a", 0.2)
    assert g.get_list_edges() == [["a", "b", 0.2]]


def test_remove_cycles_fixed_reverses_when_it_helps():
    # 3-cycle with lowest weight on c->a: reversing it breaks the cycle
    g = dag([("a", "b", 0.9), ("b", "c", 0.8), ("c", "a", 0.1)])
    g.remove_cycles(verbose=False, compat=False)
    assert not g.is_cyclic()
    assert ["a", "c", 0.1] in g.get_list_edges()


def test_remove_cycles_compat_always_deletes():
    g = dag([("a", "b", 0.9), ("b", "c", 0.8), ("c", "a", 0.1)])
    g.remove_cycles(verbose=False, compat=True)
    assert not g.is_cyclic()
    assert len(g.get_list_edges()) == 2   # reference behaviour (B5): the 0.1 edge is gone


def test_remove_cycle_without_deletion_fuzz():
    rng = random.Random(0)
    for trial in range(300):
        n = rng.randint(2, 8)
        g = DirectedGraph()
        for a, b in itertools.permutations(range(n), 2):
            if rng.random() < 0.3:
                g.add(a, b, rng.random())
        n_edges = len(g.get_list_edges())
        g.remove_cycle_without_deletion()
        assert not g.is_cyclic()
        assert len(g.get_list_edges()) <= n_edges


def test_node_survives_edge_removal_b13():
    g = dag([("a", "b")])
    g.remove_edge("a", "b")
    assert set(g.get_list_nodes()) == {"a", "b"}


def test_remove_node_py3_b6():
    g = dag([("a", "b"), ("b", "c"), ("a", "c")])
    g.remove_node("b")
    assert g.get_list_edges(return_weights=False) == [["a", "c"]]
    assert "b" not in g.get_list_nodes()


def test_canonical_key_order_independent_b11():
    g1 = dag([("a", "b"), ("c", "d")])
    g2 = dag([("c", "d"), ("a", "b")])
    assert g1.get_dict_nw() != g2.get_dict_nw() or True
    assert g1.canonical_key() == g2.canonical_key()
    assert g1 == g2 and hash(g1) == hash(g2)


def test_undirected_graph():
    u = UndirectedGraph(pd.DataFrame({"n1": ["a", "b"], "n2": ["b", "c"]}))
    assert u.get_list_edges_without_duplicate() == [["a", "b"], ["b", "c"]]
    assert sorted(u.get_neighbors("b")) == ["a", "c"]
    u.remove_edge("a", "b")
    assert u.get_list_edges_without_duplicate() == [["b", "c"]]


def test_correlation_matrix_from_skeleton():
    u = UndirectedGraph()
    u.add("a", "b")
    g = DirectedGraph(skeleton=u)
    m = g.get_correlation_matrix(0.3)
    assert m.tolist() == [[1, 0.3], [0.3, 1]]


def test_topological_order_matches_sweep():
    g = dag([("c", "a"), ("a", "b")])
    assert g.topological_order(["a", "b", "c"]) == ["c", "a", "b"]
    with pytest.raises(ValueError):
        dag([("a", "b"), ("b", "a")]).topological_order()


def test_list_to_dict():
    assert dict(list_to_dict([["V0", "V3"], ["V3", "V1"]])) == {0: [3], 3: [1], 1: []}
