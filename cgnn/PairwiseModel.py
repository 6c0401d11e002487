"""Reference module path ``cgnn.PairwiseModel`` (PairwiseModel.py)."""
from cgnn_amd.models.base import Pairwise_Model  # noqa: F401
