"""Reference module path ``cgnn.utils.Loss`` (utils/Loss.py): the loss functions under
their reference names (PyTorch implementations; the training engine runs the fused
HIP kernels)."""
from cgnn_amd.utils.loss import (Fourier_MMD_Loss_tf, MMD_loss_tf, MomentMatchingLoss_tf,  # noqa: F401
                                 bandwiths_gamma, f1, rp)
