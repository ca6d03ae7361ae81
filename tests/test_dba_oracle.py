"""CPU: the DBA-harness oracle (oracle/dba_np.py) against golden fixtures from
the live src/DBA/helper.py methods (tests/golden/gen_dba_fixtures.py)."""
from __future__ import annotations

import os
import random
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from dba_cases import CASES, DBA_LAYERS, case_params, case_rows, case_seed, fixture_path  # noqa: E402
from oracle import dba_np as od  # noqa: E402

SEG = np.cumsum([0] + [int(np.prod(s)) for _, s in DBA_LAYERS])
# torch.mean / torch.norm reduce in an order of their own: fp32 results agree to a few ulp
ATOL32 = 1e-8


def fx(name):
    return dict(np.load(fixture_path(name)))


@pytest.mark.parametrize("name", ["median_n24", "median_n25"])
def test_lower_median_bit_exact(name):
    x, _ = case_rows(name)
    np.testing.assert_array_equal(od.median(x), fx(name)["out_0"])


@pytest.mark.parametrize("name", ["momkrum_n24_f5", "momkrum_n25_f5"])
def test_mom_krum_aliased_bucket_bit_exact(name):
    x, _ = case_rows(name)
    np.testing.assert_array_equal(od.mom_krum(x), fx(name)["out_0"])


@pytest.mark.parametrize("name", ["krum_n24_f5", "krum_n25_f0"])
def test_krum_per_layer(name):
    x, _ = case_rows(name)
    out, _ = od.krum(x, SEG, CASES[name][1]["f"])
    np.testing.assert_array_equal(out, fx(name)["out_0"])


@pytest.mark.parametrize("name", ["mean_n24", "trimmedmean_n24_b02", "trimmedmean_n25_b01"])
def test_means(name):
    x, _ = case_rows(name)
    got = od.fed_avg(x) if CASES[name][0] == "fed_avg" else od.trimmed_mean(x, CASES[name][1]["beta"])
    np.testing.assert_allclose(got, fx(name)["out_0"], rtol=0, atol=ATOL32)


def _near(cand, ref, atol, rtol):
    """Per coordinate: some candidate equals ref within tolerance (NaN matches NaN:
    keep = 0 when beta <= -theta is the mean of an empty slice)."""
    close = np.abs(cand - ref[None, :]) <= atol + rtol * np.abs(ref)
    both_nan = np.isnan(cand) & np.isnan(ref)[None, :]
    return (close | both_nan).any(axis=0)


@pytest.mark.parametrize("name", ["bulyankrum_n24_f5", "bulyankrum_n25_f2", "bulyanmedian_n25_f5",
                                  "bulyanmedian_n24_f5", "bulyantrimmed_n25_f5", "bulyankrum_n30_f8_negbeta",
                                  "bulyanmedian_n30_f8_negbeta", "bulyantrimmed_n40_f12_negbeta",
                                  "bulyanmedian_n30_f10_negbeta", "bulyantrimmed_nan_n24_f5",
                                  "bulyankrum_nan_n24_f5"])
def test_bulyan_one_of_two_medians(name):
    method, kw, *_ = CASES[name]
    mode = {"bulyan_krum": "krum", "bulyan_median": "median", "bulyan_trimmed_mean": "trimmedmean"}[method]
    x, _ = case_rows(name)
    cand = od.bulyan_candidates(x, SEG, kw["f"], mode)
    ref = fx(name)["out_0"].astype(np.float64)
    got = od.bulyan(x, SEG, kw["f"], mode)
    # NaN client picked first by Krum (helper.py:982): NaN in the reference and the oracle alike
    nan_pick = np.isnan(ref) & np.isnan(got)
    assert np.array_equal(np.isnan(ref), np.isnan(got))
    ok = _near(cand, ref, 1e-7, 2e-6) | nan_pick
    assert ok.all(), np.nonzero(~ok)
    # the shared fp64 stage lands on one of the candidates too
    assert (_near(cand, got, 1e-12, 1e-12) | nan_pick).all()


def test_bulyan_median_nan_asserts():
    """helper.py:1047: a NaN coordinate propagates through torch.median; no
    finite distance, ``assert min_index != None`` fails in the reference and the oracle."""
    assert str(fx("bulyanmedian_nan_n24_f5")["error"]) == "AssertionError"
    x, _ = case_rows("bulyanmedian_nan_n24_f5")
    with pytest.raises(AssertionError):
        od.bulyan(x, SEG, 5, "median")


def test_filterl2():
    x, _ = case_rows("filterl2_n24")
    kw = CASES["filterl2_n24"][1]
    got = od.filterl2(x, SEG, kw["sigma"], kw["expansion"])
    np.testing.assert_allclose(got, fx("filterl2_n24")["out_0"], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("name", ["exnoregret_n24", "exnoregret_n24_sqrt"])
def test_ex_noregret(name):
    x, _ = case_rows(name)
    kw = CASES[name][1]
    got = od.ex_noregret(x, SEG, kw["eps"], kw["sigma"], kw["expansion"], kw["itv"])
    np.testing.assert_allclose(got, fx(name)["out_0"], rtol=1e-5, atol=1e-8)


def test_history_two_rounds():
    f = fx("history_n24")
    prev = None
    for rnd in range(2):
        x, _ = case_rows("history_n24", rnd)
        clipped, agg = od.history(x, prev, SEG)
        np.testing.assert_allclose(clipped, f["clipped_%d" % rnd], rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(agg, f["out_%d" % rnd], rtol=1e-5, atol=1e-8)
        prev = f["out_%d" % rnd]


def test_bucketing_two_rounds():
    f = fx("bucketing_n100")
    prev = None
    for rnd in range(2):
        x, _ = case_rows("bucketing_n100", rnd)
        random.seed(case_seed("bucketing_n100") + rnd)
        _, agg = od.bucketing(x, prev, SEG, random)
        np.testing.assert_allclose(agg, f["out_%d" % rnd], rtol=1e-5, atol=1e-8)
        prev = f["out_%d" % rnd]


@pytest.mark.parametrize("name", ["mean_sharded_n100", "median_sharded_n100"])
def test_sharded(name):
    x, _ = case_rows(name)
    random.seed(case_seed(name))
    s = od.sharding(x, random)
    got = od.fed_avg(s) if CASES[name][0] == "fed_avg" else od.median(s)
    np.testing.assert_allclose(got, fx(name)["out_0"], rtol=0, atol=ATOL32)


def test_sharding_too_few_clients_raises():
    assert str(fx("sharding_n25")["error"]) == "IndexError"
    x, _ = case_rows("sharding_n25")
    with pytest.raises(IndexError):
        od.sharding(x, random.Random(0))


def test_geometric_median():
    f = fx("geomed_n24")
    x, ns = case_rows("geomed_n24")
    med, calls, wv, dist = od.geometric_median(x, ns, SEG, maxiter=4)
    np.testing.assert_allclose(med, f["out_0"], rtol=1e-5, atol=1e-8)
    assert calls == int(f["calls_0"])
    np.testing.assert_allclose(wv, f["wv_0"], rtol=1e-5)
    np.testing.assert_allclose(dist, f["dist_0"], rtol=1e-5)


@pytest.mark.parametrize("name", ["foolsgold_n24", "foolsgold_mem_n24"])
def test_foolsgold_weights(name):
    f = fx(name)
    memory = {}
    for rnd in range(2):
        assert str(f["error_%d" % rnd]) == "NameError"   # helper.py:1417 ``alpha(base)``
        x, _ = case_rows(name, rnd)
        g = od.foolsgold_features(x, SEG, memory, list(range(x.shape[0])), case_params(name)["fg_use_memory"])
        np.testing.assert_allclose(np.array([memory[i] for i in range(x.shape[0])]), f["memory_%d" % rnd],
                                   rtol=1e-15)
        wv, alpha = od.foolsgold_weights(g)
        np.testing.assert_allclose(wv, f["wv_%d" % rnd], rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(alpha, f["alpha_%d" % rnd], rtol=1e-12, atol=1e-14)
