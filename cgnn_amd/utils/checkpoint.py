"""Checkpoint / resume (new; the reference has none).

* Search state of the structure searches (current graph with weights,
  canonical keys of every tested configuration, best score, loop counters)
  is written atomically as JSON after every evaluated batch when a
  ``checkpoint=<path>`` kwarg is given; a later call with the same path
  resumes where the previous one stopped.
* Tensor checkpoints (GNN track, generator parameters) use safetensors
  (no pickle), plus a JSON sidecar for metadata.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Any, Dict, Optional

from .graph import DirectedGraph, UndirectedGraph


def graph_to_dict(g) -> Dict[str, Any]:
    d = {"type": type(g).__name__,
         "nodes": [_enc(n) for n in g.get_list_nodes()],
         "edges": [[_enc(a), _enc(b), float(w)] for a, b, w in g.get_list_edges(order_by_weight=False)]}
    if isinstance(g, DirectedGraph) and g.skeleton:
        d["skeleton"] = graph_to_dict(g.skeleton)
    return d


def graph_from_dict(d):
    if d["type"] == "UndirectedGraph":
        g = UndirectedGraph()
    else:
        skel = graph_from_dict(d["skeleton"]) if d.get("skeleton") else False
        g = DirectedGraph(skeleton=skel)
    for a, b, w in d["edges"]:
        g.add(_dec(a), _dec(b), w)
    for n in d["nodes"]:
        g.add_node(_dec(n))
    return g


def _enc(n):
    return n if isinstance(n, (str, int, float)) else repr(n)


def _dec(n):
    return n


def key_to_json(key):
    return [list(e) for e in key]


def key_from_json(k):
    return tuple(tuple(e) for e in k)


def atomic_write_json(path: str, obj: Dict[str, Any]):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".ckpt_", suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def load_json(path: Optional[str]):
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


class SearchCheckpoint:
    """Save/restore the state of a structure search."""

    def __init__(self, path: Optional[str], algorithm: str):
        self.path = path
        self.algorithm = algorithm

    def load(self):
        st = load_json(self.path)
        if st is None or st.get("algorithm") != self.algorithm:
            return None
        st["graph"] = graph_from_dict(st["graph"])
        st["tested"] = {key_from_json(k) for k in st.get("tested", [])}
        return st

    def save(self, graph, tested, **state):
        if not self.path:
            return
        obj = {"algorithm": self.algorithm, "graph": graph_to_dict(graph),
               "tested": [key_to_json(k) for k in sorted(tested)]}
        obj.update(state)
        atomic_write_json(self.path, obj)


def save_tensors(path: str, tensors: Dict[str, Any], metadata: Optional[Dict[str, str]] = None):
    from safetensors.torch import save_file
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, path,
              metadata={k: str(v) for k, v in (metadata or {}).items()})


def load_tensors(path: str, device="cpu"):
    from safetensors.torch import load_file
    return load_file(path, device=str(device))
