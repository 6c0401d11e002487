from cgnn_amd.utils.formats import CCEPC_PairsFileReader  # noqa: F401
from . import Formats, Graph, Loss, Settings  # noqa: F401  (reference module paths)
from cgnn_amd.utils.settings import SETTINGS  # noqa: F401
