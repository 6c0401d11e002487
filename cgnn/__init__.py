"""Drop-in compatibility package: ``import cgnn`` exposes the reference API
(Code/cgnn/__init__.py:1-11) backed by the MI355X-native ``cgnn_amd``."""
# load the plug-in submodules first (cgnn.GNN / cgnn.CGNN / cgnn.CGNN_confounders
# modules, as in the reference), then bind the package names to the classes,
# exactly like the reference's ``from .CGNN import CGNN``
from . import GNN as _GNN_module, CGNN as _CGNN_module, CGNN_confounders as _CC_module  # noqa: F401
from . import utils
from cgnn_amd import (SETTINGS, DirectedGraph, UndirectedGraph, CGNN, CGNN_confounders, GNN,
                      Loss, generators)

__all__ = ['DirectedGraph', 'UndirectedGraph', 'CGNN', 'CGNN_confounders', 'GNN']
