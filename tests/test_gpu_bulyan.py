"""GPU parity of Bulyan (k4) in all three selection modes against the golden
fixtures and the oracle.

The selection (which clients / aggregates enter the per-coordinate stage), the
Bulyan median pick (numpy's fp64 pairwise tie-break for even theta) and the
beta-window are discrete decisions reproduced exactly; the final fp64 mean is
summed in the same (distance) order with numpy's pairwise scheme, so the
result matches to fp64 rounding (rtol 1e-12)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import fixtures, gpu_available
from oracle import robust_np as orc
from synth import make_rows

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from srfl_amd import engine, robust_estimator as gre

BY = fixtures(func="bulyan")


def _leftfirst_and_ties(xs, f, mode):
    """The defined-tie restatement of the per-coordinate stage over the
    oracle's (bit-exact) selection, plus the coordinates where the reference's
    own result depends on numpy's unstable argsort."""
    rows = [np.asarray(r).ravel() for r in xs]
    sel, _ = orc.bulyan_select(rows, f, mode)
    S = np.array([np.asarray(g, dtype=np.float64).ravel() for g in sel])
    beta = S.shape[0] - 2 * f
    want = np.array([orc.bulyan_one_coordinate_leftfirst(S[:, j], beta) for j in range(S.shape[1])])
    ties = np.array([orc.bulyan_boundary_tie(S[:, j], beta) for j in range(S.shape[1])])
    return want, ties


@pytest.mark.parametrize("rec", BY, ids=[r["name"] for r in BY])
def test_golden_bulyan(rec):
    xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
    p = rec["params"]
    if "error" in rec:
        # IndexError (theta <= 0, :327) or AssertionError (median mode with a
        # NaN client: no strict minimum distance, :308)
        with pytest.raises({"IndexError": IndexError, "AssertionError": AssertionError}[rec["error"]]):
            gre.bulyan(xs, p["f"], p["aggsubfunc"])
        return
    got = gre.bulyan(xs, p["f"], p["aggsubfunc"])
    assert got.dtype == np.float64 and got.shape == rec["out"].shape
    want, ties = _leftfirst_and_ties(xs, p["f"], p["aggsubfunc"])
    # 1. exactly the defined (left-first) tie rule everywhere
    np.testing.assert_allclose(got.ravel(), want, rtol=1e-12, atol=1e-15)
    # 2. the reference itself wherever its argsort order is not tie-dependent
    ok = ~ties
    np.testing.assert_allclose(got.ravel()[ok], rec["out"].ravel()[ok], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("mode", ["krum", "median", "trimmedmean"])
@pytest.mark.parametrize("n,f", [(128, 20), (100, 20), (64, 10), (37, 8), (100, 30), (30, 8), (16, 3)])
def test_bulyan_against_oracle(mode, n, f):
    x = make_rows(n, 1500, seed=77 + n + f, byz=f)
    want, _ = _leftfirst_and_ties(list(x), f, mode)
    got = engine.bulyan(torch.from_numpy(x).cuda(), f, mode).cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)


def test_bulyan_krum_selection_matches_oracle():
    x = make_rows(60, 4000, seed=11, byz=12, identical_byz=True)
    rows = [r for r in x]
    _, removed = orc.bulyan_select(rows, 12, "krum")
    _, sel = engine.bulyan(torch.from_numpy(x).cuda(), 12, "krum", selected=True)
    assert sel.cpu().tolist() == removed


def test_bulyan_even_theta_tiebreak_dense_ties():
    # integer-valued data: many exact ties in distances and values
    rng = np.random.default_rng(5)
    x = rng.integers(-4, 5, size=(48, 700)).astype(np.float32)
    for mode in ("krum", "median", "trimmedmean"):
        want, _ = _leftfirst_and_ties(list(x), 10, mode)
        got = engine.bulyan(torch.from_numpy(x).cuda(), 10, mode).cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("mode", ["krum", "median", "trimmedmean"])
def test_bulyan_wide_magnitude_columns(mode):
    """Columns whose values span more than fp64 can sum exactly (1e-2 beside
    1e-12 and 1e-30) take the listed-column path: numpy's pairwise totals for
    the centre and the argsort-order walk for the window."""
    rng = np.random.default_rng(17)
    x = (0.01 * rng.standard_normal((40, 600))).astype(np.float32)
    cols = rng.choice(600, 200, replace=False)
    for c in cols:
        rows = rng.choice(40, 3, replace=False)
        x[rows[0], c] *= 1e-10
        x[rows[1], c] *= 1e-28
    want, _ = _leftfirst_and_ties(list(x), 8, mode)
    got = engine.bulyan(torch.from_numpy(x).cuda(), 8, mode).cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15, equal_nan=True)


@pytest.mark.parametrize("theta,beta", [(88, 48), (22, 4), (31, 5), (16, -8), (10, -10), (128, 40), (7, 7)])
def test_stage_f32_columns(theta, beta):
    """The per-coordinate stage alone (sra_bulyan_stage_f32) on float32 rows:
    plain columns, wide-magnitude columns (listed path), NaN / inf columns
    (the generic stage), duplicate-heavy columns, against the left-first
    restatement of robust_estimator.py:259-275."""
    rng = np.random.default_rng(theta * 7 + beta)
    d = 900
    S = (0.01 * rng.standard_normal((theta, d))).astype(np.float32)
    S[:, 100:200] = rng.integers(-3, 4, size=(theta, 100)).astype(np.float32)   # ties
    for c in range(200, 300):
        r = rng.choice(theta, 2, replace=False)
        S[r[0], c] *= 1e-12
        S[r[1], c] *= 1e-30
    S[rng.integers(0, theta), 300] = np.nan
    S[rng.integers(0, theta), 301] = np.inf
    S[rng.integers(0, theta), 302] = -np.inf
    S[:2, 303] = np.inf
    S[:, 304] = 0.0
    got = engine.bulyan_stage(torch.from_numpy(S).cuda(), beta).cpu().numpy()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = np.array([orc.bulyan_one_coordinate_leftfirst(S[:, j].astype(np.float64), beta) for j in range(d)])
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15, equal_nan=True)


def test_scalar_helpers_match_reference():
    """Drop-in bulyan_median / bulyan_one_coordinate (robust_estimator.py:259-275)
    against the live-reference fixture (float64 in, numpy scalars out)."""
    import os
    import warnings
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "bulyan_coord.npz"))
    offs = np.concatenate([[0], np.cumsum(z["lens"])])
    for c in range(len(z["lens"])):
        a = z["values"][offs[c]:offs[c + 1]]
        beta = int(z["betas"][c])
        m, row = gre.bulyan_median(a)
        assert int(m) == int(z["median_index"][c])
        np.testing.assert_array_equal(row, z["rows"][offs[c]:offs[c + 1]])
        got = gre.bulyan_one_coordinate(a, beta)
        assert isinstance(got, np.float64)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            want = orc.bulyan_one_coordinate_leftfirst(a, beta)
        np.testing.assert_allclose(got, want, rtol=1e-15, atol=0)
        if not orc.bulyan_boundary_tie(a, beta):
            np.testing.assert_allclose(got, z["one"][c], rtol=1e-15, atol=0)


@pytest.mark.parametrize("mode", ["median", "trimmedmean"])
@pytest.mark.parametrize("n,f", [(129, 20), (200, 20), (256, 30), (512, 20)])
def test_bulyan_many_clients(mode, n, f):
    """More than 128 clients (the reference has no limit): rounds with more
    than 128 remaining clients take the LDS k-select + distance passes, the
    later ones the fused register pass; theta > 128 takes the LDS stage."""
    d = 400 if n <= 256 else 200
    x = make_rows(n, d, seed=91 + n + f, byz=f)
    want, _ = _leftfirst_and_ties(list(x), f, mode)
    got = engine.bulyan(torch.from_numpy(x).cuda(), f, mode).cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("theta,beta", [(160, 80), (129, 1), (300, -40), (472, 392), (511, 100)])
def test_stage_f32_many_rows(theta, beta):
    """The per-coordinate stage for theta > 128 (LDS sort, the same exact-span
    window path, the stage by definition for NaN / inf / wide columns)."""
    rng = np.random.default_rng(theta + 3 * beta)
    d = 260
    S = (0.01 * rng.standard_normal((theta, d))).astype(np.float32)
    S[:, 60:100] = rng.integers(-3, 4, size=(theta, 40)).astype(np.float32)
    for c in range(100, 140):
        r = rng.choice(theta, 2, replace=False)
        S[r[0], c] *= 1e-12
        S[r[1], c] *= 1e-30
    S[rng.integers(0, theta), 140] = np.nan
    S[rng.integers(0, theta), 141] = np.inf
    S[rng.integers(0, theta), 142] = -np.inf
    S[:2, 143] = np.inf
    S[:, 144] = 0.0
    got = engine.bulyan_stage(torch.from_numpy(S).cuda(), beta).cpu().numpy()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = np.array([orc.bulyan_one_coordinate_leftfirst(S[:, j].astype(np.float64), beta) for j in range(d)])
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15, equal_nan=True)


@pytest.mark.parametrize("mode,n,f", [("median", 600, 40), ("trimmedmean", 600, 40), ("median", 1100, 60),
                                      ("trimmedmean", 1100, 60), ("krum", 600, 40)])
def test_bulyan_beyond_512_clients(mode, n, f):
    """No client ceiling the reference lacks (robust_estimator.py:277-332):
    rounds with more than 512 remaining clients take the LDS k-select with
    row groups of 1024 for the distances, Bulyan-Krum the N > 512 Krum rounds,
    and theta = 520 / 980 the stage with a 32-coordinate LDS tile."""
    x = make_rows(n, 120, seed=7 + n + f, byz=f)
    want, _ = _leftfirst_and_ties(list(x), f, mode)
    got = engine.bulyan(torch.from_numpy(x).cuda(), f, mode).cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("theta,beta", [(600, 200), (1030, 900), (2100, 37)])
def test_stage_f32_beyond_512_rows(theta, beta):
    """The stage for theta > 512 (16- and 32-coordinate LDS tiles; the stage
    by definition for NaN / inf / wide columns with fewer lanes per block)."""
    rng = np.random.default_rng(theta + beta)
    d = 70
    S = (0.01 * rng.standard_normal((theta, d))).astype(np.float32)
    S[:, 10:20] = rng.integers(-3, 4, size=(theta, 10)).astype(np.float32)
    for c in range(20, 30):
        r = rng.choice(theta, 2, replace=False)
        S[r[0], c] *= 1e-12
        S[r[1], c] *= 1e-30
    S[rng.integers(0, theta), 30] = np.nan
    S[rng.integers(0, theta), 31] = np.inf
    S[:2, 32] = -np.inf
    S[:, 33] = 0.0
    got = engine.bulyan_stage(torch.from_numpy(S).cuda(), beta).cpu().numpy()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = np.array([orc.bulyan_one_coordinate_leftfirst(S[:, j].astype(np.float64), beta) for j in range(d)])
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15, equal_nan=True)


@pytest.mark.parametrize("theta,beta", [(700, 300), (2000, 1500)])
def test_scalar_helpers_beyond_512(theta, beta):
    """The drop-in's bulyan_median / bulyan_one_coordinate (robust_estimator.py:
    259-275) on arrays longer than 512 (rank slots in dynamic LDS, fewer lanes
    per block), against the oracle's restatement."""
    import warnings
    a = np.random.default_rng(theta).standard_normal(theta)
    m, row = gre.bulyan_median(a)
    wm, wrow = orc.bulyan_median(a)
    assert int(m) == int(wm)
    np.testing.assert_array_equal(row, wrow)
    got = gre.bulyan_one_coordinate(a, beta)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = orc.bulyan_one_coordinate_leftfirst(a, beta)
    np.testing.assert_allclose(got, want, rtol=1e-15, atol=0)
