"""PyTorch oracle of the CGNN training semantics.

Runs on the CPU (float64 by default).  It is used

* as the numerical reference the HIP kernels are tested against, and
* as the execution path for tiny problems when no GPU is present (CI).

It consumes the same DAG programs and draws the same Philox noise as the
device path, so for equal (seed, run) both paths train the same model up to
floating-point rounding.

Semantics reproduced from the reference:
  * generator  x_v = W2^T ReLU(W1^T [x_pa, e_v, xi...] + b1) + b2  (CGNN.py:76-81)
  * loss       biased multi-bandwidth MMD^2, gammas {0.005 ... 50} (Loss.py:12-32)
               or random-Fourier-feature MMD (Loss.py:35-56)
  * optimiser  TF1 Adam, eps outside the bias correction (CGNN.py:97-99)
  * score      mean loss over test_epochs fresh-noise forward passes (CGNN.py:129-153)
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..utils import philox
from .program import Program

GAMMAS = (0.005, 0.05, 0.25, 0.5, 1.0, 5.0, 50.0)


def mmd_loss_dense(pred: torch.Tensor, true: torch.Tensor, gammas=GAMMAS) -> torch.Tensor:
    """Biased multi-kernel MMD^2 of [N,d] samples (Loss.py:12-32), exact distances."""
    n = pred.shape[0]
    x = torch.cat([pred, true], 0)
    d2 = torch.cdist(x, x).pow(2) if x.shape[1] > 0 else x.new_zeros(2 * n, 2 * n)
    s = torch.cat([x.new_full((n,), 1.0 / n), x.new_full((n,), -1.0 / n)])
    S = s[:, None] * s[None, :]
    loss = x.new_zeros(())
    for g in gammas:
        loss = loss + (S * torch.exp(-g * d2)).sum()
    return loss


def rff_frequencies(key, step: int, k: int, d: int, gammas=GAMMAS, dtype=torch.float64):
    """[d+1, 7k] frequency matrix exactly as the device draws it (Loss.py:35-37)."""
    F = k * len(gammas)
    f = np.arange(F, dtype=np.uint32)[:, None]
    dd = np.arange(d, dtype=np.uint32)[None, :]
    z = philox.normal(key[0], key[1], f, dd, step, philox.RNG_RFF_FREQ, dtype=np.float64)
    g = np.repeat(np.asarray(gammas, dtype=np.float64), k)[:, None]
    omega = 2.0 * g * z
    ph = 2.0 * np.pi * philox.uniform(key[0], key[1], f[:, 0], d, step, philox.RNG_RFF_FREQ,
                                      word=2, dtype=np.float64)
    W = np.concatenate([omega, ph[:, None]], axis=1).T    # [d+1, F]
    return torch.as_tensor(W, dtype=dtype)


def rff_mmd_loss(pred: torch.Tensor, true: torch.Tensor, W: torch.Tensor, k: int) -> torch.Tensor:
    """Fourier-feature MMD (Loss.py:39-56) for a given frequency matrix."""
    def phi(x):
        xo = torch.cat([x, x.new_ones(x.shape[0], 1)], 1)
        return math.sqrt(2.0 / k) * torch.cos(xo @ W).mean(0)
    return ((phi(true) - phi(pred)) ** 2).sum()


class ReferenceTrainer:
    """Train R generative models one after another on the CPU."""

    def __init__(self, programs: Sequence[Program], datas: Sequence[np.ndarray],
                 keys: Sequence[tuple], H: int, learning_rate=0.01, init_std=0.05,
                 use_fast_mmd=False, nb_vectors=100, dtype=torch.float64):
        self.programs = list(programs)
        self.datas = [torch.as_tensor(np.asarray(d), dtype=dtype) for d in datas]   # [d, N]
        self.keys = list(keys)
        self.H = int(H)
        self.lr = float(learning_rate)
        self.init_std = float(init_std)
        self.fast = bool(use_fast_mmd)
        self.k = int(nb_vectors)
        self.dtype = dtype
        self.params: List[torch.Tensor] = []
        self.loss_history: List[List[float]] = [[] for _ in self.programs]
        for p, key in zip(self.programs, self.keys):
            idx = np.arange(p.n_params, dtype=np.uint32)
            w = self.init_std * philox.normal(key[0], key[1], idx, 0, 0, philox.RNG_PARAM_INIT,
                                              dtype=np.float64)
            self.params.append(torch.as_tensor(w, dtype=dtype))
        self.rng_step = 0
        self.opt_step = 0

    # --------------------------------------------------------------- pieces
    row0 = 0           # global index of sample 0 (sample-sharded training, engine/sharded.py)

    def noise(self, r, a_ids, b, purpose, N):
        k0, k1 = self.keys[r]
        n = np.arange(N, dtype=np.uint32) + np.uint32(self.row0)
        return torch.as_tensor(philox.normal(k0, k1, n, b, self.rng_step, purpose, dtype=np.float64),
                               dtype=self.dtype)

    def generate(self, r, theta: torch.Tensor, step: Optional[int] = None) -> torch.Tensor:
        """Forward pass of model r -> generated matrix [d, N]."""
        if step is not None:
            saved, self.rng_step = self.rng_step, step
        prog = self.programs[r]
        data = self.datas[r]
        N = data.shape[1]
        H = self.H
        cols = [None] * prog.n_vars
        for var, kind, pars, confs, poff, nin in prog.node_records():
            if kind == 1:
                cols[var] = data[var]
                continue
            inp = [cols[p] for p in pars]
            inp.append(self.noise(r, None, var, philox.RNG_NODE_NOISE, N))
            for c in confs:
                inp.append(self.noise(r, None, c, philox.RNG_CONF_NOISE, N))
            X = torch.stack(inp, 1)                                  # [N, nin]
            W1 = theta[poff: poff + nin * H].view(nin, H)
            b1 = theta[poff + nin * H: poff + (nin + 1) * H]
            W2 = theta[poff + (nin + 1) * H: poff + (nin + 2) * H]
            b2 = theta[poff + (nin + 2) * H]
            cols[var] = torch.relu(X @ W1 + b1) @ W2 + b2
        if step is not None:
            self.rng_step = saved
        return torch.stack(cols, 0)

    def loss(self, r, theta):
        pred = self.generate(r, theta).T
        true = self.datas[r].T
        if self.fast:
            W = rff_frequencies(self.keys[r], self.rng_step, self.k, true.shape[1], dtype=self.dtype)
            return rff_mmd_loss(pred, true, W, self.k)
        return mmd_loss_dense(pred, true)

    # --------------------------------------------------------------- driver
    def train(self, epochs: int, verbose=False):
        R = len(self.programs)
        ms = [torch.zeros_like(p) for p in self.params]
        vs = [torch.zeros_like(p) for p in self.params]
        b1, b2, eps = 0.9, 0.999, 1e-8
        for it in range(epochs):
            t = self.opt_step + 1
            lr_t = self.lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
            for r in range(R):
                theta = self.params[r].clone().requires_grad_(True)
                L = self.loss(r, theta)
                (g,) = torch.autograd.grad(L, theta)
                self.loss_history[r].append(float(L.detach()))
                ms[r] = b1 * ms[r] + (1 - b1) * g
                vs[r] = b2 * vs[r] + (1 - b2) * g * g
                self.params[r] = self.params[r] - lr_t * ms[r] / (vs[r].sqrt() + eps)
                if verbose and it % 100 == 0:
                    print('Run:{}, Iter:{}, score:{}'.format(r, it, float(L)))
            self.rng_step += 1
            self.opt_step += 1

    def evaluate(self, epochs: int, log_every: int = 0, log=None) -> np.ndarray:
        """Mean test loss per model; ``log(it, losses[R])`` every ``log_every`` steps."""
        R = len(self.programs)
        acc = np.zeros(R)
        with torch.no_grad():
            for it in range(epochs):
                cur = np.array([float(self.loss(r, self.params[r])) for r in range(R)])
                acc += cur
                if log is not None and log_every > 0 and it % log_every == 0:
                    log(it, cur)
                self.rng_step += 1
        return acc / max(epochs, 1)

    def run(self, train_epochs: int, test_epochs: int, verbose=False) -> np.ndarray:
        self.train(train_epochs, verbose)
        return self.evaluate(test_epochs)
