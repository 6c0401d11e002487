"""CGNN_CHECK on the HIP paths: every operand invariant the kernels assume holds in
whole training steps of the GNN trainers (fused GCN, L-layer GCN, fused GAT,
GraphSAGE with the pipelined sampler), and a corrupted CSR is refused before the
SpMM kernel launches."""
import pytest
import torch

from cgnn_amd.utils import checks

pytestmark = pytest.mark.gpu


@pytest.fixture
def checking(monkeypatch):
    monkeypatch.setattr(checks, "ENABLED", True)
    yield


def test_gpu_training_steps_pass_the_checks(checking):
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gat import GATTrainer
    from cgnn_amd.gnn.gcn import GCNTrainer
    from cgnn_amd.gnn.gcn_deep import DeepGCNTrainer
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-products", seed=4, device="cuda:0", scale=0.003)
    GCNTrainer(g, hidden=256, reorder=True).train_step()
    DeepGCNTrainer(g, hidden=128, layers=3, capture=False).train_step()
    GATTrainer(g, heads=4, head_dim=32, reorder=True).train_step()
    SAGETrainer(g, hidden=64, layers=3, fanouts=[10, 5, 5], batch_size=256).train_epoch()
    torch.cuda.synchronize()


def test_gpu_corrupt_csr_is_refused(checking):
    from cgnn_amd.gnn import ops
    rp = torch.tensor([0, 2, 3], dtype=torch.int32, device="cuda:0")
    col = torch.tensor([0, 1, 1 << 20], dtype=torch.int32, device="cuda:0")
    X = torch.ones(4, 8, dtype=torch.bfloat16, device="cuda:0")
    with pytest.raises(ValueError, match="column index range"):
        ops.spmm(rp, col, X, 8)
