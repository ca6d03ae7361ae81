"""GPU parity of the DBA harness's aggregators (srfl_amd.dba)
against the live reference's outputs (tests/golden/dba_*.npz) and the CPU
oracle (oracle/dba_np.py), plus unit tests of the k10 kernels.

Bars: bit-exact for the lower median, the per-layer Krum pick, mom_krum's
aliased bucket, the shard averages and the k10 kernels against numpy with the
same fp32 operation order; torch.mean-based means within a few fp32 ulp
(atol 1e-8 at |x| ~ 1e-2); Bulyan equal to one of the two exact-tie answers
(DBA's fp32 stage decides an even theta's tie by rounding) to rtol 2e-6;
filters / history / bucketing / geometric median rtol 1e-5 (fp64 device
arithmetic vs the reference's fp32 torch)."""
from __future__ import annotations

import collections
import random

import numpy as np
import pytest
import torch

from dba_cases import CASES, DBA_LAYERS, case_params, case_rows, case_seed, fixture_path
from oracle import dba_np as od

import srfl_loader

srfl_loader.load()
from srfl_amd import dba, engine  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SEG = np.cumsum([0] + [int(np.prod(s)) for _, s in DBA_LAYERS])
ATOL32 = 1e-8


class _Model:
    def __init__(self):
        self._sd = collections.OrderedDict((k, torch.zeros(s, device=DEV)) for k, s in DBA_LAYERS)

    def state_dict(self):
        return self._sd


def _updates(x, ns, device=DEV):
    ups = collections.OrderedDict()
    for i in range(x.shape[0]):
        d, o = {}, 0
        for k, s in DBA_LAYERS:
            n = int(np.prod(s))
            d[k] = torch.from_numpy(x[i, o:o + n].reshape(s).copy()).to(device)
            o += n
        ups[i] = (int(ns[i]), d)
    return ups


def _flat(sd):
    return np.concatenate([sd[k].detach().cpu().reshape(-1).double().numpy() for k, _ in DBA_LAYERS])


def _run(name, rnd=0, helper=None, device=DEV):
    method, kw, *_ = CASES[name]
    h = helper or dba.HelperAggregation(case_params(name))
    x, ns = case_rows(name, rnd)
    ups = _updates(x, ns, device)
    m = _Model()
    random.seed(case_seed(name) + rnd)
    res = getattr(h, method)(m, ups, **kw)
    torch.cuda.synchronize()
    return _flat(m.state_dict()), res, ups, h


def fx(name):
    return dict(np.load(fixture_path(name)))


# --------------------------------------------------------------- end to end
@pytest.mark.parametrize("name", ["median_n24", "median_n25", "momkrum_n24_f5", "momkrum_n25_f5", "krum_n24_f5",
                                  "krum_n25_f0"])
def test_bit_exact_methods(name):
    got, *_ = _run(name)
    np.testing.assert_array_equal(got.astype(np.float32), fx(name)["out_0"])


@pytest.mark.parametrize("device", [DEV, "cpu"])
def test_median_host_inputs(device):
    got, *_ = _run("median_n24", device=device)
    np.testing.assert_array_equal(got.astype(np.float32), fx("median_n24")["out_0"])


@pytest.mark.parametrize("name", ["mean_n24", "trimmedmean_n24_b02", "trimmedmean_n25_b01", "mean_sharded_n100",
                                  "median_sharded_n100"])
def test_means(name):
    got, *_ = _run(name)
    np.testing.assert_allclose(got, fx(name)["out_0"], rtol=0, atol=ATOL32)


def test_sharded_median_matches_oracle_bit_exact():
    name = "median_sharded_n100"
    got, *_ = _run(name)
    x, _ = case_rows(name)
    random.seed(case_seed(name))
    np.testing.assert_array_equal(got.astype(np.float32), od.median(od.sharding(x, random)))


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
def test_bulyan(name):
    method, kw, *_ = CASES[name]
    mode = {"bulyan_krum": "krum", "bulyan_median": "median", "bulyan_trimmed_mean": "trimmedmean"}[method]
    got, *_ = _run(name)
    x, _ = case_rows(name)
    # the device shares the oracle's fp64 per-coordinate stage
    np.testing.assert_allclose(got, od.bulyan(x, SEG, kw["f"], mode).astype(np.float32), rtol=0, atol=0)
    cand = od.bulyan_candidates(x, SEG, kw["f"], mode)
    ref = fx(name)["out_0"].astype(np.float64)
    # a NaN client Krum picks first (np.argmin of a NaN score, helper.py:982) puts NaN among each of its
    # coordinates' selected values: NaN there in the reference and on the device (the candidates skip it)
    nan_pick = np.isnan(ref) & np.isnan(got)
    assert np.array_equal(np.isnan(ref), np.isnan(got))
    assert (_near(cand, ref, 1e-7, 2e-6) | nan_pick).all()
    assert (_near(cand, got.astype(np.float64), 1e-7, 2e-6) | nan_pick).all()


def test_bulyan_median_nan_raises():
    """helper.py:1047: torch.median propagates the NaN client's coordinate, every
    distance of the round is NaN, ``assert min_index != None`` fails."""
    assert str(fx("bulyanmedian_nan_n24_f5")["error"]) == "AssertionError"
    with pytest.raises(AssertionError):
        _run("bulyanmedian_nan_n24_f5")
    x, _ = case_rows("bulyanmedian_nan_n24_f5")
    with pytest.raises(AssertionError):
        od.bulyan(x, SEG, 5, "median")


def test_bulyan_krum_f1_rejected_and_theta():
    x, ns = case_rows("bulyankrum_n25_f2")
    h = dba.HelperAggregation(case_params("bulyankrum_n25_f2"))
    with pytest.raises(ValueError):
        h.bulyan_krum(_Model(), _updates(x, ns), f=1)
    with pytest.raises(RuntimeError):
        h.bulyan_median(_Model(), _updates(x, ns), f=13)


def test_filterl2():
    got, *_ = _run("filterl2_n24")
    np.testing.assert_allclose(got, fx("filterl2_n24")["out_0"], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("name", ["exnoregret_n24", "exnoregret_n24_sqrt"])
def test_ex_noregret(name):
    got, *_ = _run(name)
    np.testing.assert_allclose(got, fx(name)["out_0"], rtol=1e-5, atol=1e-8)


def test_history_two_rounds_and_write_back():
    f = fx("history_n24")
    h = None
    for rnd in range(2):
        got, _, ups, h = _run("history_n24", rnd, helper=h)
        np.testing.assert_allclose(got, f["out_%d" % rnd], rtol=1e-5, atol=1e-8)
        clipped = np.stack([_flat(ups[i][1]) for i in range(len(ups))])
        np.testing.assert_allclose(clipped, f["clipped_%d" % rnd], rtol=1e-5, atol=1e-8)


def test_bucketing_two_rounds():
    f = fx("bucketing_n100")
    h = None
    for rnd in range(2):
        got, _, _, h = _run("bucketing_n100", rnd, helper=h)
        np.testing.assert_allclose(got, f["out_%d" % rnd], rtol=1e-5, atol=1e-8)


def test_sharding_too_few_clients():
    with pytest.raises(IndexError):
        _run("sharding_n25")


def test_geometric_median():
    f = fx("geomed_n24")
    got, res, _, _ = _run("geomed_n24")
    calls, upd, names, wv, dist = res
    np.testing.assert_allclose(got, f["out_0"], rtol=1e-5, atol=1e-8)
    assert calls == int(f["calls_0"]) and upd is True and names == list(range(24))
    np.testing.assert_allclose(wv, f["wv_0"], rtol=1e-5)
    np.testing.assert_allclose(dist, f["dist_0"], rtol=1e-5)


def test_dispatch_names():
    x, ns = case_rows("median_n24")
    p = dict(case_params("median_n24"), krum_f=5, trim_beta=0.2, fliter_l2_sigma=1e-5, geom_median_maxiter=4)
    h = dba.HelperAggregation(p)
    m = _Model()
    assert dba.aggregate(h, "median", m, _updates(x, ns)) is True
    np.testing.assert_array_equal(_flat(m.state_dict()).astype(np.float32), fx("median_n24")["out_0"])
    with pytest.raises(NameError):   # the reference's helper.py:1417 raises on every call
        dba.aggregate(h, "foolsgold", m, {i: (c, list(d.values())) for i, (c, d) in _updates(x, ns).items()})


@pytest.mark.parametrize("name", ["foolsgold_n24", "foolsgold_mem_n24"])
def test_foolsgold(name):
    f = fx(name)
    h = dba.HelperAggregation(case_params(name))
    for rnd in range(2):
        x, ns = case_rows(name, rnd)
        ups = {i: (c, [d[k] for k, _ in DBA_LAYERS]) for i, (c, d) in _updates(x, ns).items()}
        with pytest.raises(NameError):
            h.foolsgold_update(_Model(), ups)
        wv, alpha = h.fg.last
        np.testing.assert_allclose(h.fg.memory.cpu().numpy(), f["memory_%d" % rnd], rtol=1e-15)
        np.testing.assert_allclose(wv.cpu().numpy(), f["wv_%d" % rnd], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(alpha.cpu().numpy(), f["alpha_%d" % rnd], rtol=1e-9, atol=1e-12)


# ------------------------------------------------------------- k10 kernels
@pytest.mark.parametrize("n", [1, 2, 3, 16, 17, 24, 33, 64, 100, 127, 128, 129, 200, 256, 257, 400, 512])
def test_order_stat_all_k(n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal((n, 1000)).astype(np.float32)
    x[:, 7] = 0.5                   # ties
    X = torch.from_numpy(x).to(DEV)
    s = np.sort(x, axis=0)
    for k in sorted({0, (n - 1) // 2, n - 1, n // 3}):
        np.testing.assert_array_equal(engine.order_stat(X, k).cpu().numpy(), s[k])


def test_order_stat_nan_and_strided():
    rng = np.random.default_rng(5)
    x = rng.standard_normal((40, 3000)).astype(np.float32)
    x[3, 10] = np.nan
    x[39, 2999] = np.nan
    X = torch.from_numpy(x).to(DEV)
    got = engine.order_stat(X[:, 1:2501], 19).cpu().numpy()
    np.testing.assert_array_equal(got, od.median(x[:, 1:2501]))
    assert np.isnan(got[9])
    # N > 128: the LDS bitonic path, same semantics (NaN anywhere -> NaN)
    y = rng.standard_normal((300, 2000)).astype(np.float32)
    y[17, 5] = np.nan
    Y = torch.from_numpy(y).to(DEV)
    got = engine.order_stat(Y[:, 3:1990], 149).cpu().numpy()
    np.testing.assert_array_equal(got, od.median(y[:, 3:1990]))
    assert np.isnan(got[2])
    # N > 512 (no ceiling below the reference's, helper.py:561): 16 / 2 / 1
    # coordinates per 64 KiB tile
    for n in (513, 1000, 9000):
        z = rng.standard_normal((n, 37)).astype(np.float32)
        z[n // 2, 7] = np.nan
        got = engine.order_stat(torch.from_numpy(z).to(DEV), (n - 1) // 2).cpu().numpy()
        np.testing.assert_array_equal(got, od.median(z))
        assert np.isnan(got[7])
    with pytest.raises(NotImplementedError):
        engine.order_stat(torch.zeros((16385, 8), device=DEV), 3)


@pytest.mark.parametrize("d,off", [(4096, 0), (1001, 0), (4096, 1)])
def test_rows_sum_div_and_weighted_sum_bit_exact(d, off):
    rng = np.random.default_rng(d + off)
    x = rng.standard_normal((9, d + 8)).astype(np.float32)
    w = rng.random(9).astype(np.float32)
    X = torch.from_numpy(x).to(DEV)[:, off:off + d]
    acc = np.zeros(d, np.float32)
    wacc = np.zeros(d, np.float32)
    for i, r in enumerate(x[:, off:off + d]):
        acc = acc + r
        wacc = wacc + w[i] * r
    np.testing.assert_array_equal(engine.rows_sum_div(X, 7).cpu().numpy(), acc / np.float32(7))
    np.testing.assert_array_equal(engine.weighted_sum(X, torch.from_numpy(w).to(DEV)).cpu().numpy(), wacc)


def test_running_clip_scale():
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((12, int(SEG[-1]))) * np.linspace(0.1, 20, 12)[:, None]).astype(np.float32)
    prev = rng.standard_normal(int(SEG[-1])).astype(np.float32)
    X = torch.from_numpy(x).to(DEV)
    p64 = torch.from_numpy(prev.astype(np.float64)).to(DEV)
    scale, nrm = engine.clip_scales(X, p64, list(SEG), 10., norms=True, running=True)
    ref = od.running_norm(x, prev.astype(np.float64), SEG)
    np.testing.assert_allclose(nrm.cpu().numpy(), ref, rtol=1e-12)
    np.testing.assert_allclose(scale.cpu().numpy(), np.minimum(1.0, 10. / ref), rtol=1e-12)
