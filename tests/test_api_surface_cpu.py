"""The drop-in ``cgnn`` package exposes every module path and public name of the
reference package (Code/cgnn), so reference user code imports
unchanged."""
import importlib

import pytest

REFERENCE_NAMES = {
    "cgnn": ["SETTINGS", "DirectedGraph", "UndirectedGraph", "CGNN", "CGNN_confounders", "GNN"],
    "cgnn.GNN": ["GNN_tf", "tf_run_instance", "tf_evalcausalscore_pairwise"],
    "cgnn.CGNN": ["CGNN_tf", "run_CGNN_tf", "hill_climbing", "exploratory_hill_climbing", "tabu_search"],
    "cgnn.CGNN_confounders": ["CGNN_confounders_tf", "run_CGNN_confounders_tf", "hill_climbing_confounders"],
    "cgnn.GraphModel": ["GraphModel"],
    "cgnn.PairwiseModel": ["Pairwise_Model"],
    "cgnn.utils": ["CCEPC_PairsFileReader"],
    "cgnn.utils.Graph": ["Graph", "DirectedGraph", "UndirectedGraph", "list_to_dict"],
    "cgnn.utils.Loss": ["MMD_loss_tf", "Fourier_MMD_Loss_tf", "MomentMatchingLoss_tf", "rp", "f1",
                        "bandwiths_gamma"],
    "cgnn.utils.Settings": ["SETTINGS", "DefaultSettings"],
    "cgnn.utils.Formats": ["CCEPC_PairsFileReader"],
    "cgnn.generators": ["RandomGraphGenerator"],
    "cgnn.generators.random_graph_generator": ["RandomGraphGenerator", "series_to_cepc_kag"],
    "cgnn.generators.functions_default": ["cause", "noise", "mechanism", "effect", "rand_bin"],
    "cgnn.generators.generators": ["FullGraphPolynomialModel_tf", "full_graph_polynomial_generator_tf",
                                   "CGNN_generator_tf", "polynomial_regressor", "linear_regressor",
                                   "support_vector_regressor"],
}


@pytest.mark.parametrize("module", sorted(REFERENCE_NAMES))
def test_reference_module_path_and_names(module):
    mod = importlib.import_module(module)
    missing = [n for n in REFERENCE_NAMES[module] if not hasattr(mod, n)]
    assert not missing, (module, missing)


def test_package_surface_matches_reference_all():
    import cgnn
    assert cgnn.__all__ == ['DirectedGraph', 'UndirectedGraph', 'CGNN', 'CGNN_confounders', 'GNN']
    # the same singleton behind every path
    from cgnn.utils.Settings import SETTINGS
    assert SETTINGS is cgnn.SETTINGS


def test_tf_evalcausalscore_pairwise_scores_one_direction():
    import numpy as np
    from cgnn.GNN import tf_evalcausalscore_pairwise, tf_run_instance
    rng = np.random.default_rng(0)
    x = rng.normal(size=(150, 2))
    kw = dict(gpu=False, train_epochs=10, test_epochs=4, h_layer_dim=8)
    s = tf_evalcausalscore_pairwise(x, 0, 0, **kw)
    xy, _ = tf_run_instance(x, 0, 0, **kw)
    assert np.isfinite(s) and s == pytest.approx(xy, rel=1e-6)      # same job as the X->Y half of a run
