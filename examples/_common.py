"""Shared helpers of the example scripts: locate the reference example CSVs
(tracked copies in tests/data/, else the read-only reference checkout)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def data_path(name, override=None):
    if override:
        return override
    for d in (os.path.join(ROOT, "tests", "data"), os.path.join(ROOT, ".refdata"), "/root/reference",
              os.getcwd()):
        p = os.path.join(d, name)
        if os.path.exists(p):
            return p
    raise FileNotFoundError(name)
