"""Reference module path ``cgnn.generators.generators`` (dead code in the reference,
SURVEY §2.6 B7; here the working re-implementations under the reference names)."""
from cgnn_amd.generators.generators import (CGNN_generator, FullGraphPolynomialModel,  # noqa: F401
                                            full_graph_polynomial_generator, linear_regressor,
                                            polynomial_regressor, support_vector_regressor)

FullGraphPolynomialModel_tf = FullGraphPolynomialModel
full_graph_polynomial_generator_tf = full_graph_polynomial_generator
CGNN_generator_tf = CGNN_generator
