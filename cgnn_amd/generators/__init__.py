from .random_graph_generator import RandomGraphGenerator, series_to_cepc_kag
from . import functions_default
