"""Reproducibility of the centred Gram and everything picked from it.

Round 5 found that a diagonal tile's (i, j) / (j, i) pair had two writers, so G
differed from call to call in ~1 % of entries (fixed in csrc/gram.hip).  The
sharded Krum (one reduce of per-rank Grams), the Bulyan-Krum order and the
two-rank shard test all assume a reproducible G, so this pins it: every Gram
path (the LDS-DMA pipe at N = 128, the pair Gram at N = 300, the bucket Gram
of mom_krum) called three times must give bitwise equal, bitwise symmetric
results, and so must the Krum order and the Bulyan-Krum selection built on
them.  Reference: src/robust_estimator.py:242 -- each unordered pair has one
distance."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import gpu_available
from synth import make_rows

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from srfl_amd import engine


def _three(fn):
    out = [fn() for _ in range(3)]
    torch.cuda.synchronize()
    return out


def _assert_bitwise_equal_sym(gs):
    a = gs[0].cpu().numpy().view(np.uint64)
    for g in gs[1:]:
        np.testing.assert_array_equal(g.cpu().numpy().view(np.uint64), a)
    np.testing.assert_array_equal(a, a.T)


@pytest.mark.parametrize("n,d", [(128, 1 << 20), (128, 1_000_003), (300, 200_000), (64, 70_001)])
def test_gram_reproducible_and_symmetric(n, d):
    X = torch.from_numpy(make_rows(n, d, seed=n + d, byz=n // 6)).cuda()
    _assert_bitwise_equal_sym(_three(lambda: engine.gram(X)))


@pytest.mark.parametrize("n,bs", [(512, 3), (128, 4), (100, 3)])
def test_bucket_gram_reproducible_and_symmetric(n, bs):
    X = torch.from_numpy(make_rows(n, 300_000, seed=n, byz=n // 6)).cuda()
    _assert_bitwise_equal_sym(_three(lambda: engine.gram_buckets(X, bs)))


def test_krum_order_and_bulyan_krum_reproducible():
    X = torch.from_numpy(make_rows(128, 1 << 20, seed=5, byz=20)).cuda()
    orders = _three(lambda: engine.krum_select(X, 20, rounds=88, scores=True))
    for o, s in orders[1:]:
        assert torch.equal(o, orders[0][0])
        assert torch.equal(s.view(torch.int32), orders[0][1].view(torch.int32))
    sels = _three(lambda: engine.bulyan(X, 20, "krum", selected=True))
    for agg, sel in sels[1:]:
        assert torch.equal(sel, sels[0][1])
        assert torch.equal(agg.view(torch.int64), sels[0][0].view(torch.int64))
    moms = _three(lambda: engine.mom_krum(X, 5, 3))
    for row, order in moms[1:]:
        assert torch.equal(order, moms[0][1])
        assert torch.equal(row.view(torch.int32), moms[0][0].view(torch.int32))
