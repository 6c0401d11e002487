"""Mechanism and noise primitives of the synthetic causal generator
(reference: generators/functions_default.py:1-51, effective behaviour).

* ``cause``     U(-1, 1) samples (the reference builds a GMM and ignores it, B9)
* ``noise``     v * U(0,1) * N(0,1) +- 2
* ``mechanism`` cubic smoothing spline through ``d`` random knots spanning
                [min(x) - std, max(x) + std]
* ``effect``    standardised mechanism output
* ``rand_bin``  quantise a standardised variable into 2..19 categories
All take an optional ``rng`` (numpy Generator) for reproducibility.
"""
from __future__ import annotations

import numpy as np
from scipy.interpolate import UnivariateSpline

from ..utils.formats import standardize


def _rng(rng):
    return rng if rng is not None else np.random.default_rng()


def cause(n, k=4, p1=2, p2=2, rng=None):
    return _rng(rng).uniform(-1, 1, n)


def noise(n, v, rng=None):
    r = _rng(rng)
    return v * r.random(1) * r.standard_normal((n, 1)) + r.choice([2, -2])


def mechanism(x, d, rng=None):
    r = _rng(rng)
    x = np.asarray(x, dtype=np.float64).ravel()
    g = np.linspace(x.min() - x.std(), x.max() + x.std(), d)
    return UnivariateSpline(g, r.standard_normal(d))(x)[:, np.newaxis]


def effect(x, n, v, d=4, rng=None):
    return standardize(mechanism(np.array(x), d, rng)).ravel()


def rand_bin(x, rng=None):
    r = _rng(rng)
    num_cat = int(r.integers(2, 20))
    maxstd = 3
    x = standardize(np.asarray(x, dtype=np.float64))
    bins = np.linspace(-maxstd, maxstd, num=num_cat + 1)
    return np.digitize(x, bins) - 1
