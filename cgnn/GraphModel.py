"""Reference module path ``cgnn.GraphModel`` (GraphModel.py)."""
from cgnn_amd.models.base import GraphModel  # noqa: F401
