"""CGNN_CHECK operand validation: corrupted index operands are refused before a
kernel could read out of bounds, and whole training steps pass the checks (no false
positives) on the CPU paths (the GPU test does the same on the HIP paths)."""
import pytest
import torch

from cgnn_amd.utils import checks


@pytest.fixture
def checking(monkeypatch):
    monkeypatch.setattr(checks, "ENABLED", True)
    yield


def test_corrupt_csr_and_indices_are_refused(checking):
    from cgnn_amd.gnn import ops
    from cgnn_amd.parallel.halo import _rows
    rp = torch.tensor([0, 2, 3], dtype=torch.int32)
    col = torch.tensor([0, 1, 5], dtype=torch.int32)          # 5 is past the 4 source rows
    X = torch.ones(4, 8, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="spmm"):
        ops.spmm(rp, col, X, 8)
    with pytest.raises(ValueError, match="decreases"):
        ops.spmm(torch.tensor([0, 3, 2], dtype=torch.int32), torch.tensor([0, 1, 2], dtype=torch.int32), X, 8)
    with pytest.raises(ValueError, match="ends at"):
        ops.spmm(torch.tensor([0, 1, 9], dtype=torch.int32), col, X, 8)
    with pytest.raises(ValueError, match="halo rows src_idx"):
        _rows(torch.zeros(3, 4), torch.zeros(2, 4), src_idx=torch.tensor([0, 3]))
    from cgnn_amd.gnn.linear import lin_fwd
    with pytest.raises(ValueError, match="idx1"):
        lin_fwd(torch.zeros(4, 8, dtype=torch.bfloat16), torch.zeros(8, 8), idx1=torch.tensor([0, 4], dtype=torch.int32))


def test_training_steps_pass_the_checks(checking):
    from cgnn_amd.gnn.data import synthetic
    from cgnn_amd.gnn.gat import GATTrainer
    from cgnn_amd.gnn.gcn import GCNTrainer
    from cgnn_amd.gnn.sage import SAGETrainer
    g = synthetic("ogbn-products", seed=4, scale=0.0005)
    GCNTrainer(g, hidden=32, reorder=True).train_step()
    GATTrainer(g, heads=4, head_dim=8, fused=True).train_step()
    SAGETrainer(g, hidden=32, layers=2, fanouts=[5, 5], batch_size=64).train_epoch()
