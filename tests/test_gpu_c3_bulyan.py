"""Config C3 at full size: Bulyan median / trimmed mean at N=128, f=20,
d=1e7 (theta=88, beta=48), reference src/robust_estimator.py:277-332.

The rounds are driven through the per-round C ABI (sra_bulyan_round_f32 +
sra_bulyan_pick, the calls sra_bulyan_f32 itself makes) so every round can be
checked on its own:
  * the round's aggregate, bit-exactly against the oracle's np.median /
    trimmed_mean of the clients still in the set, on a column sample
    (coordinates are independent, so a column subset is a full check of those
    columns);
  * the device's fp64 distance of every remaining client against an
    independent torch float64 distance over all 1e7 coordinates (rel 1e-8:
    fp32 sums over 64-coordinate tiles, fp64 across the 156,250 tiles; the
    reference's own fp32 BLAS norms are good to ~1e-6),
    and the removed client against the argmin of the independent distances
    (first index, as the reference's strict `<` scan; a near-tie within 1e-8
    would accept either side and is counted);
  * the per-coordinate stage of the one-shot sra_bulyan_f32 against the
    left-first restatement on sampled columns of the selected aggregates, and
    the one-shot result equal to the stage over the driven rounds' aggregates
    (same selection)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import srfl_loader

srfl_loader.load()
from srfl_amd import engine  # noqa: E402
from oracle import robust_np as orc  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N, F, D = 128, 20, 10_000_000


def _matrix(seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    X = torch.empty((N, D), dtype=torch.float32, device=DEV)
    X.normal_(0.0, 0.01, generator=g)
    # Byzantine-like rows: shifted and scaled differently, so the rounds remove
    # a mix of outliers and benign clients
    X[:F] += 0.004
    X[F:F + 5] *= 1.7
    return X


def _columns(seed):
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([np.arange(200), np.arange(D - 200, D), rng.integers(0, D, 1800)]))


def _ref_dist(X, rows_l, agg):
    idx = torch.tensor(rows_l, dtype=torch.long, device=DEV)
    out = torch.zeros(len(rows_l), dtype=torch.float64, device=DEV)
    step = 1 << 20
    for c0 in range(0, D, step):
        c1 = min(D, c0 + step)
        diff = X[idx, c0:c1].double() - agg[c0:c1].double()
        out += (diff * diff).sum(dim=1)
    return out


@pytest.mark.parametrize("mode", ["trimmedmean", "median"])
def test_c3_bulyan_rounds_fullsize(mode):
    X = _matrix(31 if mode == "median" else 32)
    theta = N - 2 * F
    beta = theta - 2 * F
    cols = _columns(5)
    Xc = X[:, torch.from_numpy(cols).to(DEV)].cpu().numpy()
    rows = torch.arange(N, dtype=torch.int32, device=DEV)
    nxt = torch.empty_like(rows)
    S = torch.empty((theta, D), dtype=torch.float32, device=DEV)
    dist = torch.empty(N, dtype=torch.float64, device=DEV)
    alive = list(range(N))
    near_ties = 0
    for t in range(theta):
        nr = N - t
        engine.bulyan_round(X, rows, nr, mode, S[t], dist)
        sub = Xc[alive]
        want = orc.median(sub) if mode == "median" else orc.trimmed_mean(list(sub))
        got = S[t, torch.from_numpy(cols).to(DEV)].cpu().numpy()
        np.testing.assert_array_equal(got, np.asarray(want, dtype=np.float32), err_msg="round %d aggregate" % t)
        ref = _ref_dist(X, alive, S[t]).cpu().numpy()
        dv = dist[:nr].cpu().numpy()
        np.testing.assert_allclose(dv, ref, rtol=1e-8, err_msg="round %d distances" % t)
        engine.bulyan_pick(dist, rows, nr, nxt)
        rows, nxt = nxt, rows
        removed = sorted(set(alive) - set(rows[:nr - 1].cpu().tolist()))
        assert len(removed) == 1
        pos = alive.index(removed[0])
        best = int(np.argmin(ref))
        if pos != best:
            # only a near-tie of the independent distances may flip the pick
            assert abs(ref[pos] - ref[best]) <= 1e-8 * ref[best], (t, pos, best, ref[pos], ref[best])
            near_ties += 1
        alive.pop(pos)
    assert near_ties <= 2
    # the one-shot op makes the same selection: its result is the stage over S
    one = engine.bulyan(X, F, mode)
    stage = engine.bulyan_stage(S, beta)
    torch.testing.assert_close(one, stage, rtol=0, atol=0)
    Sc = S[:, torch.from_numpy(cols).to(DEV)].double().cpu().numpy()
    want = np.array([orc.bulyan_one_coordinate_leftfirst(Sc[:, j], beta) for j in range(len(cols))])
    np.testing.assert_allclose(one[torch.from_numpy(cols).to(DEV)].cpu().numpy(), want, rtol=1e-12, atol=1e-15)
