"""Statistical integration tests on the reference's example datasets (SURVEY §4
item 4): the three entry-script workloads at the reference settings, fixed seed,
scored against the shipped ground truth.  GPU only (the CPU oracle would take
hours at these sizes); skipped when the example CSVs are not available."""
import numpy as np
import pandas as pd
import pytest

import cgnn
from cgnn_amd.utils.formats import CCEPC_PairsFileReader
from cgnn_amd.utils.metrics import orientation_scores, shd, sign_accuracy

from conftest import example, have_example

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reference_settings(monkeypatch):
    for k, v in dict(GPU=True, NB_RUNS=32, train_epochs=1000, test_epochs=500, h_layer_dim=20, seed=0).items():
        monkeypatch.setattr(cgnn.SETTINGS, k, v)
    yield


@pytest.mark.skipif(not have_example("Example_pairwise_pairs.csv"), reason="reference examples absent")
def test_pairwise_example_sign_accuracy():
    data = CCEPC_PairsFileReader(example("Example_pairwise_pairs.csv"), scale=True)
    targets = pd.read_csv(example("Example_pairwise_targets.csv"))["Target"].values
    pred = cgnn.GNN(backend="TensorFlow").predict_dataset(data, h_layer_dim=30)
    assert len(pred) == 5 and np.all(np.isfinite(pred))
    assert sign_accuracy(pred, targets) >= 0.6          # measured: 4/5


@pytest.mark.skipif(not have_example("Example_graph_numdata.csv"), reason="reference examples absent")
def test_graph_example_shd():
    data = pd.read_csv(example("Example_graph_numdata.csv"))
    umg = cgnn.UndirectedGraph(pd.read_csv(example("Example_graph_skeleton.csv")))
    target = cgnn.DirectedGraph(pd.read_csv(example("Example_graph_target.csv")))
    pdg = cgnn.GNN().orient_graph(data, umg)
    dag = cgnn.CGNN().orient_directed_graph(data, pdg)
    assert not dag.is_cyclic()
    assert len(dag.get_list_edges()) == 30
    assert shd(dag, target) <= 4                         # measured: 2
    assert orientation_scores(dag, target)["precision"] >= 0.85


@pytest.mark.skipif(not have_example("Example_graph_confounders_numdata.csv"), reason="reference examples absent")
def test_confounders_example_recovers_edges():
    data = pd.read_csv(example("Example_graph_confounders_numdata.csv"))
    umg = cgnn.UndirectedGraph(pd.read_csv(example("Example_graph_confounders_skeleton.csv")))
    target = cgnn.DirectedGraph(pd.read_csv(example("Example_graph_confounders_target.csv")))
    pdg = cgnn.GNN().orient_graph_confounders(data, umg, nb_runs=16)
    dag = cgnn.CGNN_confounders().orient_directed_graph(data, pdg, nb_runs=16)
    assert not dag.is_cyclic()
    sc = orientation_scores(dag, target)
    assert sc["precision"] >= 0.6 and sc["recall"] >= 0.6, sc   # measured (32 runs): 0.82 / 0.86
