"""Property tests of the aggregators on the device, with
hypothesis drawing shapes, seeds, offsets and outlier scales:

* translation equivariance: agg(X + c 1^T) = agg(X) + c for every coordinate-
  wise rule, Krum / Bulyan-Krum pick the same clients, the spectral filters
  move with the data.  Inputs are integer-valued fp32 (|x| <= 2^10) so that
  X + c is exact; median and the Krum/Bulyan picks are then bit-exact, and the
  rules that divide (trimmed mean, average, filters) agree to a few ulps at
  the magnitude of c;
* permutation invariance of the coordinate-wise rules (the column's multiset
  is all that matters);
* robustness: f clients scaled away by 1e3-1e6 are never picked by Krum,
  never selected by Bulyan-Krum, and move neither the coordinate-wise rules
  nor the filters' outputs out of the honest clients' range.
The reference functions these properties belong to: robust_estimator.py
:144-208 (filters), :220-232 (median, trimmed mean), :234-257 (Krum family),
:259-332 (Bulyan); average simulate.py:235-244."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import gpu_available

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from srfl_amd import engine

SETTINGS = dict(max_examples=12, deadline=None, derandomize=True)


def _ints(seed, n, d, lim=1024):
    rng = np.random.default_rng(seed)
    return rng.integers(-lim, lim + 1, size=(n, d)).astype(np.float32)


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


@settings(**SETTINGS)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(3, 140), d=st.integers(1, 700),
       c=st.integers(-2**12, 2**12))
def test_coordinatewise_translation_equivariance(seed, n, d, c):
    x = _ints(seed, n, d)
    X, Xc = _dev(x), _dev(x + np.float32(c))
    np.testing.assert_array_equal(engine.median(Xc).cpu().numpy(),
                                  engine.median(X).cpu().numpy() + np.float32(c))
    # the rules that divide round (S + k c) / k once and S / k + c twice: a few
    # ulps at the magnitude of c (numpy's own trimmed mean differs the same way)
    tol = 4.0 * float(np.spacing(np.float32(1.0))) * (abs(c) + 1024.0)
    for fn in (engine.trimmed_mean, engine.average):
        got = fn(Xc).cpu().numpy().astype(np.float64)
        want = fn(X).cpu().numpy().astype(np.float64) + c
        np.testing.assert_allclose(got, want, rtol=0, atol=tol, err_msg=fn.__name__)


@settings(**SETTINGS)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(2, 140), d=st.integers(1, 500))
def test_coordinatewise_permutation_invariance(seed, n, d):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, d)) * 10 ** rng.uniform(-3, 3)).astype(np.float32)
    perm = rng.permutation(n)
    X, Xp = _dev(x), _dev(x[perm])
    for fn in (engine.median, engine.trimmed_mean):
        np.testing.assert_array_equal(fn(X).cpu().numpy(), fn(Xp).cpu().numpy())


@settings(**SETTINGS)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(8, 100), d=st.integers(4, 2000),
       c=st.integers(-2**10, 2**10))
def test_krum_translation_invariance(seed, n, d, c):
    """Same pick (or, on a near-tie, two picks whose scores agree to fp32 rounding:
    the centring mean of X + c rounds differently from mean(X) + c)."""
    f = max(1, n // 5)
    x = _ints(seed, n, d)
    o1, s1 = engine.krum_select(_dev(x), f, 1)
    o2, s2 = engine.krum_select(_dev(x + np.float32(c)), f, 1)
    i1, i2 = int(o1[0]), int(o2[0])
    s1, s2 = s1.cpu().numpy(), s2.cpu().numpy()
    np.testing.assert_allclose(s2, s1, rtol=1e-5)
    assert i1 == i2 or abs(float(s1[i1]) - float(s1[i2])) <= 1e-5 * abs(float(s1[i1]))


@settings(**SETTINGS)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(10, 128), d=st.integers(8, 3000),
       scale=st.sampled_from([1e3, 1e4, 1e6]))
def test_krum_rejects_scaled_away_outliers(seed, n, d, scale):
    rng = np.random.default_rng(seed)
    f = max(1, n // 5)
    x = (0.01 * rng.standard_normal((n, d))).astype(np.float32)
    bad = rng.choice(n, size=f, replace=False)
    x[bad] *= np.float32(scale)
    _, idx = engine.krum(_dev(x), f)
    assert int(idx) not in set(bad.tolist())


@settings(**SETTINGS)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(12, 64), d=st.integers(4, 600),
       scale=st.sampled_from([1e3, 1e5]))
def test_bulyan_krum_never_selects_outliers(seed, n, d, scale):
    rng = np.random.default_rng(seed)
    f = max(1, (n - 3) // 4)
    x = (0.01 * rng.standard_normal((n, d))).astype(np.float32)
    bad = rng.choice(n, size=f, replace=False)
    x[bad] *= np.float32(scale)
    X = _dev(x)
    out, sel = engine.bulyan(X, f, "krum", selected=True)
    assert not (set(sel.cpu().numpy()[: n - 2 * f].tolist()) & set(bad.tolist()))
    good = np.delete(x, bad, axis=0)
    o = out.cpu().numpy()
    assert np.all(o >= good.min(0) - 1e-6) and np.all(o <= good.max(0) + 1e-6)


@settings(**SETTINGS)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(10, 128), d=st.integers(1, 700),
       scale=st.sampled_from([1e3, 1e6]))
def test_coordinatewise_bounded_by_honest_range(seed, n, d, scale):
    """With f < int(0.1 n) + 1 ... the trimmed mean (b = int(0.1 n) >= f) and the
    median stay inside the honest clients' per-coordinate range."""
    rng = np.random.default_rng(seed)
    f = max(1, int(0.1 * n))
    x = (0.01 * rng.standard_normal((n, d))).astype(np.float32)
    bad = rng.choice(n, size=f, replace=False)
    x[bad] = np.float32(scale) * np.sign(rng.standard_normal((f, d))).astype(np.float32)
    good = np.delete(x, bad, axis=0)
    X = _dev(x)
    for fn in (engine.median, engine.trimmed_mean):
        o = fn(X).cpu().numpy()
        assert np.all(o >= good.min(0)) and np.all(o <= good.max(0)), fn.__name__


@settings(max_examples=6, deadline=None, derandomize=True)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(16, 64), k=st.integers(20, 200),
       c=st.integers(-2**8, 2**8))
def test_filters_translation_equivariance(seed, n, k, c):
    """The filters work on the centred covariance: a common offset moves the
    output by that offset.  The chunk Gram's centring mean of X + c rounds
    differently from mean(X) + c (~1 ulp of c), and the filter iterations
    amplify that perturbation, hence the tolerance."""
    x = _ints(seed, n, k, lim=256) / np.float32(256.0)
    X, Xc = _dev(x), _dev(x + np.float32(c))
    for fn in (engine.filter_l2, engine.ex_noregret):
        a = fn(X, 0.2, 1e-5, 20, 1000).cpu().numpy()
        b = fn(Xc, 0.2, 1e-5, 20, 1000).cpu().numpy()
        np.testing.assert_allclose(b - c, a, rtol=0, atol=1e-6 * (abs(c) + 1.0))


@settings(max_examples=6, deadline=None, derandomize=True)
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(24, 100), k=st.integers(50, 400),
       scale=st.sampled_from([1e2, 1e4]))
def test_filterl2_discounts_scaled_away_outliers(seed, n, k, scale):
    """f = int(0.1 n) clients far out along one direction: filterL2 removes them
    first (their tau dominates), so the output lands within the honest clients'
    range and near their mean."""
    rng = np.random.default_rng(seed)
    f = max(1, int(0.1 * n))
    x = (0.01 * rng.standard_normal((n, k))).astype(np.float32)
    bad = rng.choice(n, size=f, replace=False)
    direction = rng.standard_normal(k).astype(np.float32)
    x[bad] = np.float32(0.01 * scale) * direction[None, :] + x[bad]
    good = np.delete(x, bad, axis=0)
    o = engine.filter_l2(_dev(x), 0.2, 1e-5, 20, 1000).cpu().numpy()
    assert np.all(o >= good.min(0)) and np.all(o <= good.max(0))
    assert np.abs(o - good.mean(0)).max() < 0.5 * np.abs(good).max()
