"""Pin the CPU oracle (oracle/robust_np.py) against the golden fixtures that
tests/golden/gen_fixtures.py generated from the live reference.

Bit-exact where the restatement follows the reference's evaluation order
(average, median, trimmed_mean, krum scores/index, bulyan); the spectral
filters evaluate the weighted covariance with one GEMM instead of the
reference's stacked outer products, so they are pinned at fp64 rounding level.
"""
from __future__ import annotations

import json
import os
import warnings

import numpy as np
import pytest

from conftest import fixtures, GOLDEN, TRACE_OF, assert_chunks_within_bound
from oracle import robust_np as orc
from synth import make_convnet_round

CALL = {
    "median": lambda xs, p: orc.median(xs),
    "trimmed_mean": lambda xs, p: orc.trimmed_mean(xs, p.get("beta", 0.1)),
    "krum": lambda xs, p: orc.krum(xs, p["f"]),
    "krum_": lambda xs, p: orc.krum_(xs, p["f"]),
    "mom_krum": lambda xs, p: orc.mom_krum(xs, p["f"]),
    "bulyan": lambda xs, p: orc.bulyan(xs, p["f"], p["aggsubfunc"]),
    "filterL2": lambda xs, p: orc.filterL2(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]),
    "ex_noregret": lambda xs, p: orc.ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]),
    "mom_filterL2": lambda xs, p: orc.mom_filterL2(xs, p["eps"], p["sigma"], p["expansion"], p["itv"], p["delta"]),
    "mom_ex_noregret": lambda xs, p: orc.mom_ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"], p["delta"]),
}
EXACT = {"median", "trimmed_mean", "krum", "krum_", "mom_krum", "bulyan"}

CASES = fixtures()
# the full-size C4 / C5 fixtures through the primal oracle take minutes each:
# marked slow (their decisions are pinned by test_filter_trace_oracle.py's
# client-space oracle on every run)
_SLOW = {"filterL2_n128_c4", "ex_noregret_n128_c4", "mom_filterL2_n512_c5"}
CASE_PARAMS = [pytest.param(r, marks=pytest.mark.slow) if r["name"] in _SLOW else r for r in CASES]


@pytest.mark.parametrize("rec", CASE_PARAMS, ids=[r["name"] for r in CASES])
def test_oracle_matches_reference(rec):
    xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
    call = CALL[rec["func"]]
    if "error" in rec:
        exc = {"IndexError": IndexError, "ValueError": ValueError, "TypeError": TypeError,
               "AssertionError": AssertionError}[rec["error"]]
        with pytest.raises(exc), warnings.catch_warnings():
            warnings.simplefilter("ignore")
            call(xs, rec["params"])
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        got = call(xs, rec["params"])
    if isinstance(got, tuple):
        got, idx = got
        assert idx == int(rec["index"])
    got = np.asarray(got)
    want = rec["out"]
    assert got.shape == want.shape
    if rec["func"] in EXACT or rec["name"] == "ex_noregret_none_exit":
        # (ex_noregret_none_exit: the reference's projection is infeasible and the
        # next, unweighted iteration exits early with the fp32 mean, :65-72, 99)
        np.testing.assert_array_equal(got, want)
        if rec["func"] != "krum_":
            assert got.dtype == want.dtype
    elif rec["name"] in TRACE_OF:
        # 50 iterations, 30 of them on benign clients only: the reweighting
        # c *= 1 - tau/tau_max carries fp64 rounding to 1e-6 .. 1e-3 of max|out|
        # with identical decisions; per-chunk bound = 3x the farthest of three
        # independent oracle evaluations (tests/golden/add_trace_bounds.py).
        # The default (gemm) order is one of those three, so this value check is
        # consistency only; the oracle's C4/C5 parity proper is pinned by
        # test_filter_trace_oracle.py, which requires the reference's decision
        # trace exactly (every chunk, iteration count included).
        assert_chunks_within_bound(got, rec)
    else:
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12)


def test_oracle_c1_convnet_round():
    z = np.load(os.path.join(GOLDEN, "c1_convnet_n100.npz"))
    layers = make_convnet_round(int(z["n"]), int(z["seed"]))
    cs = [float(np.sum(np.stack(l).astype(np.float64))) for l in layers]
    np.testing.assert_array_equal(np.array(cs), z["x_checksum"])
    med = np.concatenate([orc.median(l).ravel() for l in layers])
    tm = np.concatenate([orc.trimmed_mean(l).ravel() for l in layers])
    np.testing.assert_array_equal(med, z["median"])
    np.testing.assert_array_equal(tm, z["trimmedmean"])
    assert json.loads(str(z["shapes"]))[4] == [200, 1470]


def test_leftfirst_bulyan_rule_equals_reference_off_ties():
    """The defined tie rule (oracle.bulyan_one_coordinate_leftfirst, which the
    GPU kernel implements) reproduces the reference bit for bit on every
    coordinate whose beta-nearest set is not tie-ambiguous."""
    from conftest import fixtures
    n_tie = 0
    for rec in fixtures(func="bulyan"):
        if "error" in rec:
            continue
        xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
        p = rec["params"]
        rows = [np.asarray(r).ravel() for r in xs]
        sel, _ = orc.bulyan_select(rows, p["f"], p["aggsubfunc"])
        S = np.array([np.asarray(g, dtype=np.float64).ravel() for g in sel])
        beta = S.shape[0] - 2 * p["f"]
        for j in range(S.shape[1]):
            tie = orc.bulyan_boundary_tie(S[:, j], beta)
            n_tie += tie
            if not tie:
                got = orc.bulyan_one_coordinate_leftfirst(S[:, j], beta)
                want = rec["out"].ravel()[j]
                assert got == want or abs(got - want) <= 1e-15 or (np.isnan(got) and np.isnan(want))
    assert n_tie > 0   # the median-mode fixtures do contain such ties


def _coord_cases():
    z = np.load(os.path.join(GOLDEN, "bulyan_coord.npz"))
    vals, lens = z["values"], z["lens"]
    offs = np.concatenate([[0], np.cumsum(lens)])
    for c in range(len(lens)):
        yield (vals[offs[c]:offs[c + 1]], int(z["betas"][c]), int(z["median_index"][c]),
               z["rows"][offs[c]:offs[c + 1]], float(z["one"][c]))


def test_oracle_bulyan_scalar_helpers():
    """robust_estimator.bulyan_median / bulyan_one_coordinate (:259-275) on
    arrays with odd/even theta, ties, NaN (argmin -> 0), inf and negative beta."""
    n_tie = 0
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for a, beta, mi, row, one in _coord_cases():
            m, r = orc.bulyan_median(a)
            assert m == mi
            np.testing.assert_array_equal(np.where(np.arange(len(a)) == m, 0.0, r), row)
            got = orc.bulyan_one_coordinate_leftfirst(a, beta)
            if orc.bulyan_boundary_tie(a, beta):
                n_tie += 1
                continue
            assert got == one or abs(got - one) <= 1e-15 * max(1.0, abs(one)) or (np.isnan(got) and np.isnan(one))
    assert n_tie > 0


def test_projection_infeasible_only_when_cap_reaches_one():
    """robust_estimator.py:78-99: let I be the last candidate with clip_I =
    1 - (I+1) cap > 0.  Then clip_{I+1} <= 0 gives clip_I <= cap, and the
    rescaled largest remaining weight is c_max clip_I / S_rest <= clip_I <= cap:
    candidate I always passes the :92 test.  So projected_c is None exactly when
    no candidate has clip > 0, i.e. cap = 1 / ((1 - eps) n') >= 1 -- fixed for
    the chunk, so the None happens at iteration 0 or never, and the unweighted
    iteration after it sees iteration 0's covariance (in fp32).  This is why the
    None-then-exit outcome only exists inside the fp32 window that
    ex_noregret_none_below / ex_noregret_exit_above bracket (DESIGN.md
    section 4).  Checked here on weights spread over 12 orders of magnitude."""
    import warnings
    from oracle import robust_np as orc
    rng = np.random.default_rng(7)
    warnings.simplefilter("ignore")
    for _ in range(3000):
        n = int(rng.integers(2, 40))
        eps = float(rng.uniform(0.0, 0.6))
        c = np.exp(rng.uniform(-28.0, 0.0, n)) * (rng.uniform() if rng.uniform() < 0.5 else 1.0)
        got = orc.kl_capped_projection(c, eps)
        cap = 1.0 / (1 - eps) / n
        if cap < 1.0 - 1e-12:
            assert got is not None, (n, eps)
            assert got.max() <= cap * (1 + 1e-12) and abs(got.sum() - 1.0) < 1e-9
        elif cap >= 1.0:
            assert got is None
