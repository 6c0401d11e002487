"""Drop-in compatibility package: ``import cgnn`` exposes the reference API
(Code/cgnn/__init__.py:1-11) backed by the MI355X-native ``cgnn_amd``."""
from cgnn_amd import (SETTINGS, DirectedGraph, UndirectedGraph, CGNN, CGNN_confounders, GNN,
                      Loss, generators)
from . import utils

__all__ = ['DirectedGraph', 'UndirectedGraph', 'CGNN', 'CGNN_confounders', 'GNN']
