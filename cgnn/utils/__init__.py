from cgnn_amd.utils.formats import CCEPC_PairsFileReader
from cgnn_amd.utils import loss as Loss
from cgnn_amd.utils.settings import SETTINGS
from cgnn_amd.utils import graph as Graph
