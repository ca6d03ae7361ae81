"""GPU parity at BASELINE.json's full sizes through a size-independent property:
every coordinate is aggregated independently, so the device result over the
whole N x d matrix must equal the oracle's on ANY subset of columns.  Checked
bit-exactly on 4096 random columns plus the first and last 300 (block tails),
with NaN / +-inf / tie columns planted among them.

Sizes: N=128 and N=100 at d=1e8 (configs C2/north star: 51.2 GB resident),
N=512 at d=1.25e7 (the per-GPU shard of config C5)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import srfl_loader

srfl_loader.load()
from srfl_amd import engine  # noqa: E402
from oracle import dba_np as odba  # noqa: E402
from oracle import robust_np as orc  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _matrix(n, d, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    X = torch.empty((n, d), dtype=torch.float32, device=DEV)
    step = max(1, int(2e9 // (4 * d)))
    for r in range(0, n, step):
        X[r:r + step].normal_(0.0, 0.01, generator=g)
    return X


def _columns(d, seed):
    rng = np.random.default_rng(seed)
    cols = np.unique(np.concatenate([np.arange(300), np.arange(d - 300, d),
                                     rng.integers(0, d, 4096)]))
    return cols


def _plant(X, cols, rng):
    """NaNs, infinities and ties in some of the checked columns."""
    n = X.shape[0]
    pick = rng.choice(cols, 24, replace=False)
    for k, c in enumerate(pick):
        c = int(c)
        if k % 4 == 0:
            X[rng.integers(0, n), c] = float("nan")
        elif k % 4 == 1:
            X[rng.integers(0, n, 3), c] = float("nan")
        elif k % 4 == 2:
            X[rng.integers(0, n), c] = float("inf")
            X[rng.integers(0, n), c] = float("-inf")
        else:
            X[:, c] = X[0, c]


def _host_cols(X, cols):
    idx = torch.from_numpy(cols).to(DEV)
    return X.index_select(1, idx).cpu().numpy()


@pytest.fixture(scope="module")
def big():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    X = _matrix(128, 100_000_000, 11)
    cols = _columns(X.shape[1], 5)
    _plant(X, cols, np.random.default_rng(9))
    torch.cuda.synchronize()
    yield X, cols, _host_cols(X, cols)
    del X
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [128, 100])
def test_trimmed_mean_full_size(big, n):
    X, cols, h = big
    out = engine.trimmed_mean(X[:n])
    got = out[torch.from_numpy(cols).to(DEV)].cpu().numpy()
    np.testing.assert_array_equal(got, orc.trimmed_mean(list(h[:n])))


@pytest.mark.parametrize("n", [128, 100])
def test_median_full_size(big, n):
    X, cols, h = big
    got = engine.median(X[:n])[torch.from_numpy(cols).to(DEV)].cpu().numpy()
    np.testing.assert_array_equal(got, orc.median(list(h[:n])))


def test_average_and_lower_median_full_size(big):
    X, cols, h = big
    sel = torch.from_numpy(cols).to(DEV)
    np.testing.assert_array_equal(engine.average(X)[sel].cpu().numpy(), orc.average(list(h)))
    np.testing.assert_array_equal(engine.order_stat(X, 63)[sel].cpu().numpy(), odba.median(h))


def test_n512_shard_full_size():
    X = _matrix(512, 12_500_000, 12)
    cols = _columns(X.shape[1], 6)
    _plant(X, cols, np.random.default_rng(10))
    h = _host_cols(X, cols)
    sel = torch.from_numpy(cols).to(DEV)
    np.testing.assert_array_equal(engine.trimmed_mean(X)[sel].cpu().numpy(), orc.trimmed_mean(list(h)))
    np.testing.assert_array_equal(engine.median(X)[sel].cpu().numpy(), orc.median(list(h)))
    del X
    torch.cuda.empty_cache()
