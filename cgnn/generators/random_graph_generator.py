"""Reference module path ``cgnn.generators.random_graph_generator``."""
from cgnn_amd.generators.random_graph_generator import RandomGraphGenerator, series_to_cepc_kag  # noqa: F401
