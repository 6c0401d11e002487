"""Global configuration singleton.

Parity with the reference ``DefaultSettings`` (Code/cgnn/utils/Settings.py:9-45):
the same attribute names and defaults, and ``__slots__`` so that a typo'd
attribute raises ``AttributeError`` (Settings.py:10-23).

New (not in the reference):
  * ``seed``                 -- base key of the counter-based RNG
  * ``device_ids``           -- explicit GPU list (else GPU_OFFSET..GPU_OFFSET+NB_GPU)
  * ``compat_remove_cycles`` -- replicate the reference's always-delete behaviour
                                of ``remove_cycles``
  * ``batch_models``         -- how many independent models (runs x candidates)
                                one device launch trains together
  * ``verbose``              -- default verbosity of training / search logs
  * ``max_retries``          -- re-train a run whose score is non-finite up to this
                                many times with a fresh RNG stream before it is
                                dropped (0 = the reference's drop-only behaviour;
                                the reference re-runs only its polynomial generator,
                                generators.py:165-178)
  * ``compat_scores``        -- reference scoring statistics (default False):
                                the pairwise score averages ALL runs, a non-finite
                                one included (GNN.py:196-197, no np.isfinite
                                filter), and every HC candidate is scored by runs of
                                its own (Philox keys and subsamples keyed by the
                                candidate's edge set -- the reference re-draws per
                                candidate, CGNN.py:237-238) instead of the common
                                random numbers shared by all candidates
  * ``long_n_min``           -- runs with MORE samples than this (possible once
                                ``max_nb_points`` is raised, or ``None`` = no
                                subsampling) train on the sample-sharded long-N
                                trainer: the samples split over the ranks of the
                                process group (engine/sharded.py; default 1500, the
                                reference's cap, CGNN.py:183-185)

Every field can also be overridden from the environment as ``CGNN_<NAME>``
(e.g. ``CGNN_NB_RUNS=8``) when the singleton is created.

Unlike the reference, workers never read this module-global state: the engine
takes a frozen :class:`RunConfig` snapshot (``SETTINGS.snapshot(**kwargs)``)
and ships that to every rank ("SETTINGS is not propagated").
"""
from __future__ import annotations

import dataclasses
import os
from typing import Any, Optional, Tuple


class DefaultSettings(object):
    __slots__ = ("h_layer_dim",
                 "train_epochs",
                 "test_epochs",
                 "NB_RUNS",
                 "NB_JOBS",
                 "GPU",
                 "NB_GPU",
                 "GPU_OFFSET",
                 "learning_rate",
                 "init_weights",
                 "use_Fast_MMD",
                 "nb_vectors_approx_MMD",
                 "complexity_graph_param",
                 "max_nb_points",
                 # --- new fields ---
                 "seed",
                 "device_ids",
                 "compat_remove_cycles",
                 "batch_models",
                 "verbose",
                 "max_retries",
                 "long_n_min",
                 "compat_scores")

    def __init__(self):
        self.NB_RUNS = 32
        self.NB_JOBS = 1
        self.GPU = True
        self.NB_GPU = 1
        self.GPU_OFFSET = 0
        self.learning_rate = 0.01
        self.init_weights = 0.05
        self.max_nb_points = 1500

        # CGNN
        self.h_layer_dim = 20
        self.train_epochs = 1000
        self.test_epochs = 500
        self.use_Fast_MMD = False
        self.nb_vectors_approx_MMD = 100
        self.complexity_graph_param = 0.00005

        # new
        self.seed = 0
        self.device_ids = None
        self.compat_remove_cycles = False
        self.batch_models = 256
        self.verbose = False
        self.max_retries = 0
        self.long_n_min = 1500
        self.compat_scores = False
        self._apply_env()

    def _apply_env(self):
        for name in self.__slots__:
            key = "CGNN_" + name.upper()
            if key not in os.environ:
                continue
            raw = os.environ[key]
            cur = getattr(self, name)
            if isinstance(cur, bool):
                val: Any = raw.lower() in ("1", "true", "yes", "on")
            elif isinstance(cur, int):
                val = int(raw)
            elif isinstance(cur, float):
                val = float(raw)
            elif name == "device_ids":
                val = tuple(int(x) for x in raw.split(",") if x.strip())
            elif name == "max_nb_points" and raw.lower() in ("none", "0", ""):
                val = None
            else:
                val = raw
            setattr(self, name, val)

    def snapshot(self, **kwargs) -> "RunConfig":
        """Freeze the current settings, with per-call kwargs taking precedence.

        The kwarg keys follow the reference's ``kwargs.get(key, SETTINGS.ATTR)``
        table: e.g. ``init_std`` overrides ``init_weights`` and
        ``nb_runs`` overrides ``NB_RUNS``.
        """
        g = kwargs.get
        return RunConfig(
            nb_runs=int(g("nb_runs", self.NB_RUNS)),
            nb_jobs=int(g("nb_jobs", self.NB_JOBS)),
            gpu=bool(g("gpu", self.GPU)),
            nb_gpu=int(g("nb_gpu", self.NB_GPU)),
            gpu_offset=int(g("gpu_offset", self.GPU_OFFSET)),
            learning_rate=float(g("learning_rate", self.learning_rate)),
            init_std=float(g("init_std", self.init_weights)),
            max_nb_points=_opt_int(g("max_nb_points", self.max_nb_points)),
            h_layer_dim=int(g("h_layer_dim", self.h_layer_dim)),
            train_epochs=int(g("train_epochs", self.train_epochs)),
            test_epochs=int(g("test_epochs", self.test_epochs)),
            use_Fast_MMD=bool(g("use_Fast_MMD", self.use_Fast_MMD)),
            nb_vectors_approx_MMD=int(g("nb_vectors_approx_MMD", self.nb_vectors_approx_MMD)),
            complexity_graph_param=float(g("complexity_graph_param", self.complexity_graph_param)),
            seed=int(g("seed", self.seed)),
            device_ids=_as_tuple(g("device_ids", self.device_ids)),
            compat_remove_cycles=bool(g("compat_remove_cycles", self.compat_remove_cycles)),
            batch_models=int(g("batch_models", self.batch_models)),
            verbose=bool(g("verbose", self.verbose)),
            max_retries=int(g("max_retries", self.max_retries)),
            long_n_min=int(g("long_n_min", self.long_n_min)),
            compat_scores=bool(g("compat_scores", self.compat_scores)),
        )

    def __repr__(self):
        return "DefaultSettings(%s)" % ", ".join(
            "%s=%r" % (k, getattr(self, k)) for k in self.__slots__)


def _opt_int(v) -> Optional[int]:
    return None if v is None else int(v)


def _as_tuple(v) -> Optional[Tuple[int, ...]]:
    if v is None:
        return None
    if isinstance(v, int):
        return (v,)
    return tuple(int(x) for x in v)


@dataclasses.dataclass(frozen=True)
class RunConfig:
    """Immutable per-call configuration shipped to every worker / rank."""
    nb_runs: int = 32
    nb_jobs: int = 1
    gpu: bool = True
    nb_gpu: int = 1
    gpu_offset: int = 0
    learning_rate: float = 0.01
    init_std: float = 0.05
    max_nb_points: Optional[int] = 1500      # None: no subsampling
    h_layer_dim: int = 20
    train_epochs: int = 1000
    test_epochs: int = 500
    use_Fast_MMD: bool = False
    nb_vectors_approx_MMD: int = 100
    complexity_graph_param: float = 0.00005
    seed: int = 0
    device_ids: Optional[Tuple[int, ...]] = None
    compat_remove_cycles: bool = False
    batch_models: int = 256
    verbose: bool = False
    max_retries: int = 0
    long_n_min: int = 1500
    compat_scores: bool = False

    def replace(self, **kw) -> "RunConfig":
        return dataclasses.replace(self, **kw)


SETTINGS = DefaultSettings()
