"""Reference module path ``cgnn.CGNN`` (CGNN.py)."""
from cgnn_amd.models.cgnn import CGNN, CGNN_model, run_CGNN  # noqa: F401
from cgnn_amd.search.hill_climbing import (hill_climbing, exploratory_hill_climbing,  # noqa: F401
                                           tabu_search)

CGNN_tf = CGNN_model
run_CGNN_tf = run_CGNN
