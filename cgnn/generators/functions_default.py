"""Reference module path ``cgnn.generators.functions_default``."""
from cgnn_amd.generators.functions_default import cause, effect, mechanism, noise, rand_bin  # noqa: F401
