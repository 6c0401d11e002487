"""Regression and generation models (reference: generators/generators.py, which
is dead code there -- SURVEY §2.6 B7; re-implemented to its intent).

* ``FullGraphPolynomialModel`` (generators.py:23-135): every variable, in
  topological order, is a degree-2 polynomial of [1, parents / norm, noise]
  -- one weight per product of two DISTINCT inputs, ``(p+2)(p+1)/2`` weights
  for p parents -- fitted to the data by MMD with Adam.
  ``full_graph_polynomial_generator`` returns generated samples and re-runs
  with a fresh seed when training diverges (generators.py:165-178).
* ``CGNN_generator`` (generators.py:181-213): fit a CGNN (h=3 by default) and
  return one generated sample set.
* ``polynomial_regressor`` (dead torch code in the reference, :218-264):
  degree-2 polynomial regression with optional noise input, fitted by
  moment matching of the joint (target, causes).
* ``linear_regressor`` (LassoLars, :267-282), ``support_vector_regressor``
  (RBF SVR, C=1e3, gamma=0.1, :285-297).

The MMD used for fitting is ``ops.mmd.mmd_loss``: the fused HIP kernel on GPU
tensors, the dense PyTorch formula on CPU tensors.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import pandas as pd
import torch

from ..ops.mmd import mmd_loss
from ..utils.loss import MomentMatchingLoss
from ..utils.settings import SETTINGS


def _device(gpu):
    return torch.device("cuda") if gpu and torch.cuda.is_available() else torch.device("cpu")


class FullGraphPolynomialModel(torch.nn.Module):
    def __init__(self, graph, list_nodes, init_std=None, generator=None):
        super().__init__()
        self.graph = graph
        self.nodes = list(list_nodes)
        std = SETTINGS.init_weights if init_std is None else init_std
        self.order = graph.topological_order(self.nodes)
        self.parents = {v: graph.get_parents(v) for v in self.nodes}
        self.weights = torch.nn.ParameterDict()
        for v in self.order:
            p = len(self.parents[v])
            n_w = (p + 2) * (p + 1) // 2
            self.weights[str(self.nodes.index(v))] = torch.nn.Parameter(
                torch.randn(n_w, generator=generator) * std)

    def forward(self, N, noise_gen=None):
        dev = next(self.parameters()).device
        gen = {}
        for v in self.order:
            pars = self.parents[v]
            p = len(pars)
            norm = (p + 2) * (p + 1) / 2
            inputs = [torch.ones(N, device=dev)]
            inputs += [gen[u] / norm for u in pars]
            inputs.append(torch.randn(N, device=dev, generator=noise_gen))
            w = self.weights[str(self.nodes.index(v))]
            out = torch.zeros(N, device=dev)
            k = 0
            for i in range(p + 2):
                for j in range(i + 1, p + 2):
                    out = out + w[k] * inputs[i] * inputs[j]
                    k += 1
            gen[v] = out
        return torch.stack([gen[v] for v in self.nodes], 1)


def full_graph_polynomial_generator(df_data, graph, idx=0, run=0, max_retries=5, **kwargs):
    cfg = SETTINGS.snapshot(**kwargs)
    dev = _device(cfg.gpu)
    nodes = graph.get_list_nodes()
    data = torch.as_tensor(np.asarray(df_data[nodes].values, dtype=np.float32), device=dev)
    for attempt in range(max_retries + 1):
        g = torch.Generator().manual_seed(cfg.seed * 1000003 + run * 101 + attempt)
        model = FullGraphPolynomialModel(graph, nodes, cfg.init_std, g).to(dev)
        ng = torch.Generator(device=dev).manual_seed(cfg.seed + 7 * attempt + run)
        opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate)
        loss = None
        for it in range(cfg.train_epochs):
            opt.zero_grad()
            loss = mmd_loss(model(data.shape[0], ng), data)
            loss.backward()
            opt.step()
        if loss is not None and math.isfinite(float(loss)):
            with torch.no_grad():
                return pd.DataFrame(model(data.shape[0], ng).cpu().numpy(), columns=nodes)
        if cfg.verbose:
            print('Has not converged, re-running graph inference')
    raise RuntimeError("polynomial generator did not converge")


def CGNN_generator(df_data, graph, idx=0, run=0, **kwargs):
    """Fit a CGNN on ``df_data`` (hidden width 3 unless given) and return generated data."""
    from ..models.cgnn import CGNN_model
    kwargs = dict(kwargs)
    kwargs.setdefault("h_layer_dim", 3)
    nodes = graph.get_list_nodes()
    data = np.asarray(df_data[nodes].values, dtype=np.float32)
    m = CGNN_model(data.shape[0], graph, run, idx, **kwargs)
    m.train(data)
    return pd.DataFrame(m.generate(data), columns=nodes)


def polynomial_regressor(x, target, causes, fixed_noise=False, verbose=False, degree=2, **kwargs):
    """Degree-2 polynomial of [causes, noise] fitted by 4-moment matching on
    (target, causes); returns the regenerated target [n]."""
    cfg = SETTINGS.snapshot(**kwargs)
    n = target.shape[0]
    tgt = torch.as_tensor(np.asarray(target, dtype=np.float32).reshape(n, 1))
    xs = torch.as_tensor(np.asarray(x, dtype=np.float32).reshape(n, -1)) if len(causes) else torch.zeros(n, 0)
    g = torch.Generator().manual_seed(cfg.seed)
    fixed = torch.randn(n, 1, generator=g)
    p = xs.shape[1] + 1
    n_w = (p + 1) * (p + 2) // 2
    w = torch.nn.Parameter(torch.randn(n_w, generator=g) * cfg.init_std)
    opt = torch.optim.Adam([w], lr=cfg.learning_rate)

    def model():
        e = fixed if fixed_noise else torch.randn(n, 1, generator=g)
        inp = [torch.ones(n, 1), xs, e]
        z = torch.cat(inp, 1)
        out = torch.zeros(n, 1)
        k = 0
        for i in range(z.shape[1]):
            for j in range(i, z.shape[1]):
                out = out + w[k] * z[:, i:i + 1] * z[:, j:j + 1]
                k += 1
        return out

    for epoch in range(cfg.train_epochs):
        opt.zero_grad()
        y = model()
        loss = MomentMatchingLoss(torch.cat([tgt, xs], 1), torch.cat([y, xs], 1), 4)
        loss.backward()
        opt.step()
        if verbose and epoch % 50 == 0:
            print('Epoch : {} ; Loss: {}'.format(epoch, float(loss)))
    with torch.no_grad():
        return model().numpy().ravel()


def linear_regressor(x, target, causes):
    from sklearn.linear_model import LassoLars
    if len(causes) == 0:
        x = np.random.normal(size=(target.shape[0], 1))
    lasso = LassoLars(alpha=1.)
    lasso.fit(x, target)
    return lasso.predict(x)


def support_vector_regressor(x, target, causes):
    from sklearn.svm import SVR
    svr_rbf = SVR(kernel='rbf', C=1e3, gamma=0.1)
    if len(causes) == 0:
        x = np.random.normal(size=(target.shape[0], 1))
    return svr_rbf.fit(x, target).predict(x)
