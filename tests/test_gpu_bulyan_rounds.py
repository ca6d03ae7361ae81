"""Bulyan's median / trimmed-mean selection: engine.bulyan (all rounds in one
sra_bulyan_f32 call) against the per-round C ABI a sharded layer uses
(sra_bulyan_round_f32 + sra_bulyan_pick, reached through shard.bulyan with no
process group): the same selection and the same float64 result bit for bit --
ragged tiles, tied values, signed zeros, infinities, every P bucket of the row
count (src/robust_estimator.py:297-332)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import gpu_available
from synth import make_rows

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from srfl_amd import engine, shard


def _both(x, f, mode):
    X = torch.from_numpy(x).cuda()
    d = int(X.shape[1])
    want = shard.bulyan(shard.engine_ops(), X, d, f, mode)
    got, sel = engine.bulyan(X, f, mode, selected=True)
    torch.cuda.synchronize()
    return got, want


@pytest.mark.parametrize("mode", ["median", "trimmedmean"])
@pytest.mark.parametrize("n,f,d", [(5, 1, 300), (16, 3, 257), (17, 4, 1000), (33, 8, 513), (64, 10, 4097),
                                   (100, 20, 3000), (113, 20, 777), (127, 30, 256), (128, 20, 20_000),
                                   (128, 5, 1)])
def test_rank_rounds_equal_sorting_rounds(mode, n, f, d):
    x = make_rows(n, d, seed=n * 7 + f + d, byz=min(f, n // 4))
    got, want = _both(x, f, mode)
    assert torch.equal(got, want)


@pytest.mark.parametrize("mode", ["median", "trimmedmean"])
def test_rank_rounds_ties_zeros_infinities(mode):
    rng = np.random.default_rng(3)
    n, d, f = 96, 2000, 15
    x = rng.integers(-3, 4, size=(n, d)).astype(np.float32) * np.float32(0.25)   # heavy ties
    x[rng.random((n, d)) < 0.05] = -0.0
    x[5, 10:20] = np.inf
    x[7, 15:30] = -np.inf
    x[30:40] = x[0]                                                           # identical clients
    got, want = _both(x, f, mode)
    assert torch.equal(got.nan_to_num(), want.nan_to_num())
    assert torch.equal(torch.isnan(got), torch.isnan(want))


def test_rank_rounds_nan_trimmedmean():
    """A NaN coordinate: NaN ranks last; the trimmed window reaches it only once
    enough clients are gone -- same aggregates and picks as the sorting rounds."""
    x = make_rows(60, 1500, seed=44, byz=6)
    x[3, 100] = np.nan
    x[9, 100] = np.nan
    got, want = _both(x, 10, "trimmedmean")
    assert torch.equal(got.nan_to_num(), want.nan_to_num())
    assert torch.equal(torch.isnan(got), torch.isnan(want))


def test_rank_rounds_nan_median_raises():
    x = make_rows(40, 500, seed=45, byz=4)
    x[2, 7] = np.nan
    with pytest.raises(AssertionError):
        engine.bulyan(torch.from_numpy(x).cuda(), 5, "median")
