"""Deterministic synthetic client updates for fixtures, tests and the CPU leg of
the bench (SURVEY.md §8(d) recipe).

X = scale * N(0,1) + a drift shared by every client (drift * N(0,1) per
coordinate).  Optional Byzantine rows 0..byz-1 sit at -10x the benign mean
(plus small noise), or are all one identical vector (the ``xie`` attack shape,
reference src/attack.py:362-372), which exercises exact-zero distances.
"""
from __future__ import annotations

import numpy as np

CONVNET_MNIST_SHAPES = [(30, 1, 5, 5), (30,), (30, 30, 5, 5), (30,), (200, 1470), (200,), (10, 200), (10,)]
"""Parameter shapes of the reference's MNIST ConvNet (src/networks.py:36-61 with
the kernel/filters/fc config of src/simulate.py:96): d_total = 319,520."""


def make_rows(n, d, seed, byz=0, identical_byz=False, scale=0.01, drift=0.001, dtype=np.float32):
    rng = np.random.default_rng(seed)
    common = drift * rng.standard_normal(d)
    x = (scale * rng.standard_normal((n, d)) + common).astype(dtype)
    if byz:
        benign = x[byz:].astype(np.float64).mean(axis=0)
        if identical_byz:
            x[:byz] = (-10.0 * benign).astype(dtype)[None, :]
        else:
            x[:byz] = (-10.0 * benign + 0.1 * scale * rng.standard_normal((byz, d))).astype(dtype)
    return x


def make_clients(n, shape, seed, **kw):
    d = int(np.prod(shape))
    x = make_rows(n, d, seed, **kw)
    return [x[i].reshape(shape) for i in range(n)]


def make_convnet_round(n, seed, **kw):
    """Per-layer client lists for one FL round with the ConvNet shapes:
    returns layers[l] = list of n arrays of CONVNET_MNIST_SHAPES[l]."""
    layers = []
    for li, shp in enumerate(CONVNET_MNIST_SHAPES):
        layers.append(make_clients(n, shp, seed * 131 + li, **kw))
    return layers
