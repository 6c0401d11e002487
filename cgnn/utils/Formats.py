"""Reference module path ``cgnn.utils.Formats`` (utils/Formats.py)."""
from cgnn_amd.utils.formats import CCEPC_PairsFileReader  # noqa: F401
