from .random_graph_generator import RandomGraphGenerator, series_to_cepc_kag
from . import functions_default
from .generators import (FullGraphPolynomialModel, full_graph_polynomial_generator, CGNN_generator,
                         polynomial_regressor, linear_regressor, support_vector_regressor)
