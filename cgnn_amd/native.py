"""Loader for the in-tree native extensions.

``hip()`` returns the HIP kernel module (``_hip``).  It is REQUIRED whenever a
tensor lives on a GPU: there is no silent PyTorch fallback on the device path,
a missing or stale extension raises :class:`NativeExtensionError`.  The CPU
path (tests, tiny problems on machines without a GPU) is the PyTorch oracle in
``engine/reference.py`` and never touches ``_hip``.

``CGNN_HIP_LIB`` / ``CGNN_RT_LIB`` point at another build of the same module
(A/B kernel benchmarking in one process environment).

``rt()`` returns the host C++ runtime (``_rt``); it is built on first use if
missing (g++ only, a few seconds).
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import threading

_lock = threading.Lock()
_mods = {}


class NativeExtensionError(RuntimeError):
    pass


def _load(name, builder):
    with _lock:
        if name in _mods:
            return _mods[name]
        import torch  # noqa: F401  -- torch's HIP runtime must be loaded first (same SONAME)
        alt = os.environ.get("CGNN%s_LIB" % name.upper())
        if alt:   # A/B benchmarking: load another build of the same module
            spec = importlib.util.spec_from_file_location("cgnn_amd." + name, alt)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            _mods[name] = mod
            return mod
        try:
            mod = importlib.import_module("cgnn_amd." + name)
        except ImportError as first:
            if os.environ.get("CGNN_NO_AUTOBUILD"):
                raise NativeExtensionError("cgnn_amd.%s is not built: %s" % (name, first))
            try:
                builder()
                importlib.invalidate_caches()
                mod = importlib.import_module("cgnn_amd." + name)
            except Exception as exc:  # pragma: no cover - build failures are loud
                raise NativeExtensionError("cannot build/load cgnn_amd.%s: %s" % (name, exc)) from exc
        _mods[name] = mod
        return mod


def rt():
    from . import _build
    return _load("_rt", lambda: _build.build_rt())


def hip():
    from . import _build
    return _load("_hip", lambda: _build.build_hip())


def hip_loaded_path():
    m = hip()
    return getattr(m, "__file__", None)


def gpu_available() -> bool:
    import torch
    return torch.cuda.is_available()
