"""Reference module path ``cgnn.CGNN_confounders`` (CGNN_confounders.py)."""
from functools import partial

from cgnn_amd.models.cgnn import CGNN_confounders, CGNN_model, run_CGNN_confounders  # noqa: F401
from cgnn_amd.search.confounders import hill_climbing_confounders  # noqa: F401
from cgnn_amd.search.hill_climbing import exploratory_hill_climbing, tabu_search  # noqa: F401

CGNN_confounders_tf = partial(CGNN_model, confounders=True)
run_CGNN_confounders_tf = run_CGNN_confounders
