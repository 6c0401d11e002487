"""Reference module path ``cgnn.utils.Graph`` (utils/Graph.py)."""
from cgnn_amd.utils.graph import DirectedGraph, Graph, UndirectedGraph, list_to_dict  # noqa: F401
