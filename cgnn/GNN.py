"""Reference module path ``cgnn.GNN`` (GNN.py): plug-in names mapped onto cgnn_amd."""
from cgnn_amd.models.gnn import GNN, GNN_model, run_instance, pair_jobs  # noqa: F401

# reference names (GNN.py:32, :135); every backend maps to the native engine
GNN_tf = GNN_model
tf_run_instance = run_instance


def tf_evalcausalscore_pairwise(df, idx, run, **kwargs):
    """Score of ONE direction (column 0 -> column 1) of a pair for one run: train a
    pairwise generative model on ``df`` ([N, 2]) and return its mean test MMD
    (GNN.py:129-132); the run's noise is keyed by (seed, idx, run)."""
    import numpy as np
    from cgnn_amd.engine.program import program_for_pair
    from cgnn_amd.engine.scorer import Job, score_jobs
    from cgnn_amd.utils.philox import model_key
    from cgnn_amd.utils.settings import SETTINGS
    cfg = SETTINGS.snapshot(**kwargs).replace(nb_runs=1)
    m = np.asarray(df, dtype=np.float32)
    job = Job(program_for_pair(cfg.h_layer_dim), np.ascontiguousarray(m.T), model_key(cfg.seed, "gnn", idx, run, 0))
    return float(score_jobs([job], cfg)[0])
