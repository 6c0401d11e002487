"""Reference module path ``cgnn.utils.Settings`` (utils/Settings.py)."""
from cgnn_amd.utils.settings import SETTINGS, DefaultSettings  # noqa: F401
