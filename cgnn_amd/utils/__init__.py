from .formats import CCEPC_PairsFileReader
