"""Causal Generative Neural Networks on a DAG (CGNN.py:35-381) and with hidden
confounders (CGNN_confounders.py:37-512).

``CGNN.orient_directed_graph`` standardises the data and improves a DAG with a
structure search ('HC', 'EHC' or 'tabu'); ``orient_undirected_graph`` first
orients the skeleton with the pairwise GNN (CGNN.py:369-381, with the kwargs
forwarding fixed, B10).  ``CGNN_confounders`` does the same with
``hill_climbing_confounders`` on a ``DirectedGraph(skeleton=...)``.

The module-level plug-ins of the reference exist too: ``CGNN_model``
(= ``CGNN_tf``: ``train`` / ``evaluate`` / ``generate``) and ``run_CGNN``
(= ``run_CGNN_tf``: one run -> one score); both go through the batched engine
with a batch of one.
"""
from __future__ import annotations

import warnings

import numpy as np
import pandas as pd

from ..engine.program import program_for_confounders, program_for_dag
from ..engine.scorer import Job, score_jobs, subsample
from ..search.confounders import hill_climbing_confounders
from ..search.hill_climbing import exploratory_hill_climbing, hill_climbing, tabu_search
from ..utils.formats import standardize
from ..utils.philox import model_key
from ..utils.metrics import timer
from ..utils.settings import SETTINGS
from .base import GraphModel
from .gnn import GNN


def _frame_matrix(df_data, nodes):
    return np.asarray(df_data[list(nodes)].values, dtype=np.float32)


def run_CGNN(df_data, graph, idx=0, run=0, **kwargs):
    """Train + evaluate one CGNN run of ``graph`` (run_CGNN_tf, CGNN.py:163-195)."""
    cfg = SETTINGS.snapshot(**kwargs).replace(nb_runs=1)
    nodes = graph.get_list_nodes()
    m = subsample(_frame_matrix(df_data, nodes), cfg.max_nb_points, cfg.seed, "cgnn", run)
    job = Job(program_for_dag(graph, cfg.h_layer_dim, nodes), np.ascontiguousarray(m.T),
              model_key(cfg.seed, "cgnn", run))
    return float(score_jobs([job], cfg)[0])


run_CGNN._cgnn_native = True


def run_CGNN_confounders(df_data, graph, idx=0, run=0, **kwargs):
    """One run of the confounder model (run_CGNN_confounders_tf, CGNN_confounders.py:182-216,
    with the CPU-path bug B4 fixed)."""
    cfg = SETTINGS.snapshot(**kwargs).replace(nb_runs=1)
    nodes = graph.skeleton.get_list_nodes()
    m = subsample(_frame_matrix(df_data, nodes), cfg.max_nb_points, cfg.seed, "cgnn", run)
    job = Job(program_for_confounders(graph, cfg.h_layer_dim), np.ascontiguousarray(m.T),
              model_key(cfg.seed, "cgnn", run))
    return float(score_jobs([job], cfg)[0])


run_CGNN_confounders._cgnn_native = True
run_CGNN_confounders._cgnn_mode = "confounders"


class CGNN_model(object):
    """One generative model of a DAG with the reference's object API (CGNN_tf).

    ``train(data)`` fits it, ``evaluate(data)`` returns the mean test MMD,
    ``generate(data)`` returns generated samples [N, d] in
    ``graph.get_list_nodes()`` order.
    """

    def __init__(self, N, graph, run=0, idx=0, confounders=False, **kwargs):
        self.cfg = SETTINGS.snapshot(**kwargs)
        self.graph = graph
        self.run, self.idx, self.N = run, idx, N
        self.confounders = confounders
        self.nodes = graph.skeleton.get_list_nodes() if confounders else graph.get_list_nodes()
        self._trainer = None

    def _program(self):
        if self.confounders:
            return program_for_confounders(self.graph, self.cfg.h_layer_dim)
        return program_for_dag(self.graph, self.cfg.h_layer_dim, self.nodes)

    def _make(self, data, record=0):
        from ..parallel import dist as pdist
        data = np.ascontiguousarray(np.asarray(data, dtype=np.float32).T)
        key = model_key(self.cfg.seed, "cgnn", self.run)
        devs = pdist.devices_for(self.cfg)
        if devs:
            from ..engine.batch import DeviceTrainer
            return DeviceTrainer([self._program()], [data], [key], self.cfg.h_layer_dim, devs[0],
                                 learning_rate=self.cfg.learning_rate, init_std=self.cfg.init_std,
                                 use_fast_mmd=self.cfg.use_Fast_MMD,
                                 nb_vectors=self.cfg.nb_vectors_approx_MMD, record_history=record)
        from ..engine.reference import ReferenceTrainer
        return ReferenceTrainer([self._program()], [data], [key], self.cfg.h_layer_dim,
                                learning_rate=self.cfg.learning_rate, init_std=self.cfg.init_std,
                                use_fast_mmd=self.cfg.use_Fast_MMD,
                                nb_vectors=self.cfg.nb_vectors_approx_MMD)

    def _log(self, it, score):
        # the reference's progress line (CGNN.py:123-127, 147-149)
        print('Pair:{}, Run:{}, Iter:{}, score:{}'.format(self.idx, self.run, it, score))

    def train(self, data, verbose=True, **kwargs):
        """Fit the model; with ``verbose`` the training loss of every 100th iteration is
        printed as the reference does (recorded on the device, printed after the run)."""
        epochs = int(kwargs.get("train_epochs", self.cfg.train_epochs))
        self._trainer = self._make(data, record=epochs if verbose else 0)
        tr = self._trainer
        if hasattr(tr, "start"):
            tr.start()
            tr.train(epochs)
            hist = tr.history()[0] if verbose else None
        else:
            tr.train(epochs)
            hist = tr.loss_history[0][-epochs:] if verbose else None
        if verbose:
            for it in range(0, epochs, 100):
                self._log(it, float(hist[it]))

    def evaluate(self, data, verbose=True, **kwargs):
        """Mean test MMD over ``test_epochs`` evaluation steps (every 100th step's loss
        printed with ``verbose``)."""
        epochs = int(kwargs.get("test_epochs", self.cfg.test_epochs))
        if self._trainer is None:
            self.train(data, verbose)
        log = (lambda it, v: self._log(it, float(v[0]))) if verbose else None
        if hasattr(self._trainer, "start"):
            self._trainer.evaluate(epochs, log_every=100 if verbose else 0, log=log)
            self._trainer._test_epochs = max(epochs, 1)
            return float(self._trainer.collect()[0])
        return float(self._trainer.evaluate(epochs, log_every=100 if verbose else 0, log=log)[0])

    def generate(self, data, **kwargs):
        if self._trainer is None:
            self.train(data)
        tr = self._trainer
        if hasattr(tr, "start"):
            tr.evaluate(1)
            return tr.generated()[0].T
        with __import__("torch").no_grad():
            return tr.generate(0, tr.params[0]).numpy().T


class CGNN(GraphModel):
    """Generate the whole causal graph and improve the edge orientations."""

    def __init__(self, backend='PyTorch', **kwargs):
        super(CGNN, self).__init__()
        # every backend string maps to the one native path (B1)
        self.backend = backend
        self.kwargs = dict(kwargs)
        self.infer_graph = run_CGNN

    def _kw(self, kwargs):
        kw = dict(self.kwargs)
        kw.update(kwargs)
        return kw

    def create_graph_from_data(self, data, **kwargs):
        print("The CGNN model is not able (yet?) to model the graph directly from raw data")
        raise ValueError

    def orient_directed_graph(self, data, dag, alg='HC', **kwargs):
        data = pd.DataFrame(standardize(np.asarray(data.values, dtype=np.float64)), columns=data.columns)
        alg_dic = {'HC': hill_climbing, 'tabu': tabu_search, 'EHC': exploratory_hill_climbing}
        with timer("search:" + alg):
            return alg_dic[alg](dag, data, self.infer_graph, **self._kw(kwargs))

    def orient_undirected_graph(self, data, umg, **kwargs):
        warnings.warn("The pairwise GNN model is computed on each edge of the UMG "
                      "to initialize the model and start CGNN with a DAG")
        kw = self._kw(kwargs)
        gnn = GNN(backend=self.backend)
        dag = gnn.orient_graph(data, umg, printout=kw.pop("printout", None), **kw)
        return self.orient_directed_graph(data, dag, **kw)


class CGNN_confounders(CGNN):
    """CGNN with one shared noise per skeleton edge modelling hidden confounders."""

    def __init__(self, backend='PyTorch', **kwargs):
        super(CGNN_confounders, self).__init__(backend, **kwargs)
        self.infer_graph = run_CGNN_confounders

    def orient_directed_graph(self, data, dag, alg='HC', **kwargs):
        data = pd.DataFrame(standardize(np.asarray(data.values, dtype=np.float64)), columns=data.columns)
        alg_dic = {'HC': hill_climbing_confounders, 'tabu': tabu_search, 'EHC': exploratory_hill_climbing}
        with timer("search:confounders-" + alg):
            return alg_dic[alg](dag, data, self.infer_graph, **self._kw(kwargs))

    def orient_undirected_graph(self, data, umg, **kwargs):
        warnings.warn("The pairwise GNN model is computed on each edge of the UMG "
                      "to initialize the model and start CGNN with a DAG")
        kw = self._kw(kwargs)
        gnn = GNN(backend=self.backend)
        dag = gnn.orient_graph_confounders(data, umg, printout=kw.pop("printout", None), **kw)
        return self.orient_directed_graph(data, dag, **kw)
