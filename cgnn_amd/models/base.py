"""Base classes of the causal models.

* ``GraphModel``      -- GraphModel.py:9-47: ``predict(df, graph)`` dispatches on
  the exact graph type (None / DirectedGraph / UndirectedGraph).
* ``Pairwise_Model``  -- PairwiseModel.py:11-125: ``predict_dataset`` over a
  CEPC DataFrame, ``orient_graph`` (orient every skeleton edge by the sign of
  the pairwise score, then ``remove_cycle_without_deletion``) and
  ``orient_graph_confounders`` (same, on a ``DirectedGraph(skeleton=umg)``,
  then ``remove_cycles``).

Unlike the reference these loops are *batched*: a subclass may implement
``predict_proba_batch`` and then every pair / edge of the dataset is scored
in one set of device launches.  The printout CSV keeps the reference format
(``SampleID,Predictions``), written after every batch.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import pandas as pd

from ..utils.formats import standardize, write_printout
from ..utils.graph import DirectedGraph, UndirectedGraph


class GraphModel(object):
    def __init__(self):
        super(GraphModel, self).__init__()

    def predict(self, df_data, graph=None, **kwargs):
        if graph is None:
            return self.create_graph_from_data(df_data, **kwargs)
        elif type(graph) == DirectedGraph:
            return self.orient_directed_graph(df_data, graph, **kwargs)
        elif type(graph) == UndirectedGraph:
            return self.orient_undirected_graph(df_data, graph, **kwargs)
        print('Unknown Graph type')
        raise ValueError

    def orient_undirected_graph(self, data, umg, **kwargs):
        raise NotImplementedError

    def orient_directed_graph(self, data, dag, **kwargs):
        raise NotImplementedError

    def create_graph_from_data(self, data, **kwargs):
        raise NotImplementedError


def _column(df_data, name):
    return standardize(np.asarray(df_data[name].values, dtype=np.float64))


class Pairwise_Model(object):
    def __init__(self):
        super(Pairwise_Model, self).__init__()

    def predict_proba(self, a, b, idx=0, **kwargs):
        raise NotImplementedError

    def predict_proba_batch(self, pairs, **kwargs) -> List[float]:
        """Score many ``(a, b, idx)`` pairs; default: one call per pair."""
        return [self.predict_proba(a, b, idx, **kwargs) for a, b, idx in pairs]

    def _chunk(self, **kwargs):
        return int(kwargs.get("pairs_per_batch", 0) or 0)

    def predict_dataset(self, x, printout=None, **kwargs):
        rows = list(x.itertuples(index=False))
        pairs = []
        for k, row in enumerate(rows):
            a = standardize(np.asarray(row.A, dtype=np.float64).reshape(-1, 1))
            b = standardize(np.asarray(row.B, dtype=np.float64).reshape(-1, 1))
            pairs.append((a, b, k))
        step = self._chunk(**kwargs) or len(pairs) or 1
        pred, res = [], []
        for s in range(0, len(pairs), step):
            out = self.predict_proba_batch(pairs[s:s + step], **kwargs)
            for (a, b, k), p in zip(pairs[s:s + step], out):
                pred.append(p)
                res.append([rows[k].SampleID, p])
            if printout is not None:
                write_printout(printout, res)
        return pred

    def _orient(self, df_data, umg, graph, printout, **kwargs):
        edges = umg.get_list_edges_without_duplicate()
        pairs = [(_column(df_data, a), _column(df_data, b), k) for k, (a, b) in enumerate(edges)]
        step = self._chunk(**kwargs) or len(pairs) or 1
        res = []
        for s in range(0, len(pairs), step):
            weights = self.predict_proba_batch(pairs[s:s + step], **kwargs)
            for (a, b), w in zip(edges[s:s + step], weights):
                if w > 0:
                    graph.add(a, b, w)
                else:
                    graph.add(b, a, abs(w))
                res.append([str(a) + '-' + str(b), w])
            if printout is not None:
                write_printout(printout, res)
        return graph

    def orient_graph(self, df_data, umg, printout=None, **kwargs):
        graph = self._orient(df_data, umg, DirectedGraph(), printout, **kwargs)
        for n in umg.get_list_nodes():
            graph.add_node(n)
        graph.remove_cycle_without_deletion()
        return graph

    def orient_graph_confounders(self, df_data, umg, printout=None, **kwargs):
        graph = self._orient(df_data, umg, DirectedGraph(skeleton=umg), printout, **kwargs)
        graph.remove_cycles(verbose=kwargs.get("verbose", False))
        return graph
