"""Loss functions (reference: Code/cgnn/utils/Loss.py).

``MMD_loss`` / ``Fourier_MMD_Loss`` / ``MomentMatchingLoss`` operate on
PyTorch tensors ``[N, d]`` (``xy_true``, ``xy_pred``) and are differentiable.
The ``*_tf`` names of the reference are aliases.  Inside the training engine
the same losses run as fused HIP kernels (csrc/kernels/cgnn_kernels.hip,
rff_kernels.hip).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..engine.reference import GAMMAS, rff_mmd_loss

bandwiths_gamma = list(GAMMAS)


def MMD_loss(xy_true, xy_pred):
    """Biased multi-kernel MMD^2 over the 7 bandwidths (Loss.py:12-32)."""
    from ..ops.mmd import mmd_loss
    return mmd_loss(torch.as_tensor(xy_pred), torch.as_tensor(xy_true))


def rp(k, s, d, generator=None, dtype=torch.float32, device=None):
    """Random projection matrix [d+1, k*len(s)]: 2*gamma*N(0,1) frequencies and
    a U(0, 2pi) phase row (Loss.py:35-37, frequency scale kept as in the reference, B12)."""
    g = generator
    blocks = [2 * si * torch.randn(k, d, generator=g, dtype=dtype, device=device) for si in s]
    ph = torch.rand(k * len(s), 1, generator=g, dtype=dtype, device=device) * (2 * np.pi)
    return torch.cat([torch.cat(blocks, 0), ph], 1).t()


def f1(x, wz, N=None):
    """cos([x, 1] @ wz) (Loss.py:39-45)."""
    ones = torch.ones(x.shape[0], 1, dtype=x.dtype, device=x.device)
    return torch.cos(torch.cat([x, ones], 1) @ wz)


def Fourier_MMD_Loss(xy_true, xy_pred, nb_vectors_approx_MMD, wz=None, generator=None):
    """Random-Fourier-feature MMD (Loss.py:47-56); frequencies drawn fresh unless given."""
    xy_true = torch.as_tensor(xy_true)
    xy_pred = torch.as_tensor(xy_pred)
    if wz is None:
        wz = rp(nb_vectors_approx_MMD, bandwiths_gamma, xy_pred.shape[1], generator,
                dtype=xy_pred.dtype, device=xy_pred.device)
    return rff_mmd_loss(xy_pred, xy_true, wz.to(xy_pred.dtype), nb_vectors_approx_MMD)


def MomentMatchingLoss(xy_true, xy_pred, nb_moment=1):
    """L2 distance of raw moments 1..nb_moment (Loss.py:61-71 with the
    off-by-one fixed, B8: the reference's default returned 0)."""
    xy_true = torch.as_tensor(xy_true)
    xy_pred = torch.as_tensor(xy_pred)
    loss = xy_pred.new_zeros(())
    for i in range(1, nb_moment + 1):
        mp = (xy_pred ** i).mean(0)
        mt = (xy_true ** i).mean(0)
        loss = loss + torch.sqrt(((mt - mp) ** 2).sum())
    return loss


MMD_loss_tf = MMD_loss
Fourier_MMD_Loss_tf = Fourier_MMD_Loss
MomentMatchingLoss_tf = MomentMatchingLoss
