"""cgnn_amd -- Causal Generative Neural Networks, MI355X-native.

A from-scratch framework with the capabilities and Python API of the
reference CGNN package (pairwise orientation, skeleton orientation by
MMD-scored structure search, hidden confounders, synthetic causal data),
re-designed around batched hand-written HIP kernels for gfx950, hipGraph
replay and RCCL sharding.  A message-passing GNN track (GCN / GraphSAGE / GAT
on CSR SpMM / SDDMM kernels) lives in ``cgnn_amd.gnn``.

``import cgnn`` gives the reference-compatible surface.
"""
from .utils.settings import SETTINGS, DefaultSettings, RunConfig
from .utils.graph import DirectedGraph, UndirectedGraph
from .models.base import GraphModel, Pairwise_Model
from .models.gnn import GNN
from .models.cgnn import CGNN, CGNN_confounders
from .utils import loss as Loss
from . import generators

__version__ = "0.1.0"
__all__ = ['DirectedGraph', 'UndirectedGraph', 'CGNN', 'CGNN_confounders', 'GNN', 'SETTINGS']
