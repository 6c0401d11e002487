"""Reference module path ``cgnn.GNN`` (GNN.py): plug-in names mapped onto cgnn_amd."""
from cgnn_amd.models.gnn import GNN, GNN_model, run_instance, pair_jobs  # noqa: F401

# reference names (GNN.py:32, :135); every backend maps to the native engine
GNN_tf = GNN_model
tf_run_instance = run_instance
