"""File formats: ChaLearn cause-effect pairs (CEPC) reader and CSV writers.

Parity:
  * ``CCEPC_PairsFileReader`` -- Code/cgnn/utils/Formats.py:12-53: reads
    ``SampleID,A,B`` where A and B are space-separated floats (leading and
    trailing blanks stripped) and optionally standardises each series.
  * printout / prediction CSVs -- PairwiseModel.py:51-54, 81-84 and the
    entry scripts (run_GNN_pairwise_inference.py:25-28, run_CGNN_graph.py:23-29)
    -- written byte-compatibly with pandas ``to_csv``.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import numpy as np
import pandas as pd


def standardize(x, axis=0):
    """Zero-mean unit-variance standardisation (population std), matching
    ``sklearn.preprocessing.scale``: a zero-variance column is only centred."""
    a = np.asarray(x, dtype=np.float64)
    mean = a.mean(axis=axis, keepdims=True)
    std = a.std(axis=axis, keepdims=True)
    std = np.where(std == 0.0, 1.0, std)
    return (a - mean) / std


scale_data = standardize


def _parse_series(text: str) -> np.ndarray:
    toks = str(text).split(" ")
    if toks and toks[0] == "":
        toks.pop(0)
    if toks and toks[-1] == "":
        toks.pop(-1)
    return np.array([float(t) for t in toks])


def CCEPC_PairsFileReader(filename, scale=True):
    """Read a CEPC pairs CSV into a DataFrame ``[SampleID, A, B]`` of arrays."""
    raw = pd.read_csv(filename)
    rows = []
    for rec in raw.itertuples(index=False):
        rec = rec._asdict()
        a = _parse_series(rec["A"])
        b = _parse_series(rec["B"])
        if scale:
            a = standardize(a)
            b = standardize(b)
        rows.append((rec["SampleID"], a, b))
    return pd.DataFrame(rows, columns=["SampleID", "A", "B"])


def write_cepc_pairs(filename, ids: Sequence, a_list: Sequence, b_list: Sequence):
    """Inverse of the reader: one ``' x0 x1 ...'`` string per series
    (same leading-blank layout as random_graph_generator.py:11-22)."""
    def fmt(v):
        return "".join(" " + repr(float(x)) for x in np.asarray(v).ravel())
    df = pd.DataFrame({"SampleID": list(ids),
                       "A": [fmt(a) for a in a_list],
                       "B": [fmt(b) for b in b_list]})
    df.to_csv(filename, index=False)
    return df


def write_printout(filename, records: List[Sequence]):
    """Progress log ``SampleID,Predictions`` rewritten after every item."""
    pd.DataFrame(records, columns=["SampleID", "Predictions"]).to_csv(filename, index=False)


def graph_to_dataframe(graph, descending=True):
    """``Cause,Effect,Score`` table as written by the entry scripts."""
    return pd.DataFrame(graph.get_list_edges(descending=descending),
                        columns=["Cause", "Effect", "Score"])


def read_skeleton(filename):
    """Skeleton / target CSV (2 columns, optional weight) -> UndirectedGraph."""
    from .graph import UndirectedGraph
    return UndirectedGraph(pd.read_csv(filename))


def read_target_dag(filename):
    from .graph import DirectedGraph
    return DirectedGraph(pd.read_csv(filename))
