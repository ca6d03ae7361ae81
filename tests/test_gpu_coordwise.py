"""GPU parity of the coordinate-wise aggregators (k1) against the oracle and the
golden fixtures: bit-exact (assert_array_equal) for average, median and
trimmed_mean at every size, including the ragged / NaN / inf / tie cases."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import fixtures, gpu_available, GOLDEN
from oracle import robust_np as orc
from synth import make_rows, make_convnet_round

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from srfl_amd import engine, robust_estimator as gre

CW = fixtures(func="median") + fixtures(func="trimmed_mean")


@pytest.mark.parametrize("rec", CW, ids=[r["name"] for r in CW])
def test_golden_coordwise(rec):
    xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
    if rec["func"] == "median":
        got = gre.median(xs)
    else:
        got = gre.trimmed_mean(xs, rec["params"]["beta"])
    want = rec["out"]
    assert got.shape == want.shape and got.dtype == want.dtype
    if want.size == 1 and rec["func"] == "trimmed_mean" and rec["x"].shape[0] > 8:
        # numel == 1: numpy switches to a pairwise sum; fp32 tolerance
        np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-9)
    else:
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("n", [1, 2, 3, 7, 15, 16, 17, 31, 33, 64, 65, 99, 100, 101, 127, 128, 129, 200, 256, 512, 1000, 4097, 9000])   # > 4096: 1 coordinate per LDS tile
def test_every_register_and_lds_bucket(n):
    d = 1031  # not a multiple of 4 / 256: exercises tail lanes
    x = make_rows(n, d, seed=1000 + n)
    X = torch.from_numpy(x).cuda()
    np.testing.assert_array_equal(engine.median(X).cpu().numpy(), orc.median(list(x)))
    np.testing.assert_array_equal(engine.trimmed_mean(X, 0.1).cpu().numpy(), orc.trimmed_mean(list(x)))
    np.testing.assert_array_equal(engine.average(X).cpu().numpy(), orc.average(list(x)))


@pytest.mark.parametrize("beta", [0.0, 0.05, 0.25, 0.49, 0.5, 0.7])
def test_trim_fractions(beta):
    x = make_rows(100, 777, seed=7)
    got = engine.trimmed_mean(torch.from_numpy(x).cuda(), beta).cpu().numpy()
    with np.errstate(all="ignore"):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            want = orc.trimmed_mean(list(x), beta)
    np.testing.assert_array_equal(got, want)


def test_strided_rows_and_vec4_average():
    x = make_rows(64, 4096, seed=3)
    big = torch.from_numpy(x).cuda()
    sub = big[:, 5:5 + 3000]                      # ldx = 4096 != d, unaligned base
    np.testing.assert_array_equal(engine.trimmed_mean(sub).cpu().numpy(), orc.trimmed_mean(list(x[:, 5:3005])))
    np.testing.assert_array_equal(engine.average(big).cpu().numpy(), orc.average(list(x)))   # vec4 path
    np.testing.assert_array_equal(engine.average(sub).cpu().numpy(), orc.average(list(x[:, 5:3005])))


def test_expanded_and_overlapping_views_are_copied():
    """Row stride below d (an expanded 0-stride view, an overlapping
    as_strided view) must not make the kernels walk past the storage: the
    engine takes a contiguous copy (engine._unit_rows)."""
    v = torch.from_numpy(make_rows(1, 3000, seed=4)[0]).cuda()
    ex = v.expand(64, 3000)
    assert ex.stride(0) == 0
    np.testing.assert_array_equal(engine.trimmed_mean(ex).cpu().numpy(), engine.trimmed_mean(ex.contiguous()).cpu().numpy())
    np.testing.assert_array_equal(engine.median(ex).cpu().numpy(), v.cpu().numpy())
    base = torch.from_numpy(make_rows(1, 4000, seed=5)[0]).cuda()
    ov = base.as_strided((32, 3000), (31, 1))          # rows overlap (stride 31 < d)
    np.testing.assert_array_equal(engine.median(ov).cpu().numpy(), engine.median(ov.contiguous()).cpu().numpy())
    np.testing.assert_array_equal(engine.average(ov).cpu().numpy(), engine.average(ov.contiguous()).cpu().numpy())


def test_c1_convnet_round_bitexact():
    z = np.load(GOLDEN + "/c1_convnet_n100.npz")
    layers = make_convnet_round(int(z["n"]), int(z["seed"]))
    med = np.concatenate([gre.median(l).ravel() for l in layers])
    tm = np.concatenate([gre.trimmed_mean(l).ravel() for l in layers])
    np.testing.assert_array_equal(med, z["median"])
    np.testing.assert_array_equal(tm, z["trimmedmean"])


def test_full_size_properties():
    """C2 size (N=128, d=1e6): permutation invariance (bitwise) and the exact
    oracle on a 1e5-coordinate slice; device tensors in, device tensors out."""
    g = torch.Generator(device="cuda").manual_seed(0)
    X = 0.01 * torch.randn(128, 1_000_000, device="cuda", generator=g)
    tm = engine.trimmed_mean(X)
    perm = torch.randperm(128, device="cuda", generator=g)
    assert torch.equal(tm, engine.trimmed_mean(X[perm].contiguous()))
    md = engine.median(X)
    assert torch.equal(md, engine.median(X[perm].contiguous()))
    sl = X[:, :100_000].cpu().numpy()
    np.testing.assert_array_equal(tm[:100_000].cpu().numpy(), orc.trimmed_mean(list(sl)))
    np.testing.assert_array_equal(md[:100_000].cpu().numpy(), orc.median(list(sl)))
    out = gre.trimmed_mean(X)            # device in -> device out
    assert out.is_cuda and torch.equal(out, tm)


@pytest.mark.parametrize("n", [100, 128])
@pytest.mark.parametrize("d,ldx", [(64, 64), (65, 68), (1031, 1040), (300_000, 300_000), (299_999, 300_004)])
def test_exact_n_paths_ragged_bitexact(n, d, ldx):
    """The exact-N k-select paths (select_plain_kernel for the trimmed mean,
    select_reg_kernel for the median; N = 100 / 128) over ragged widths (a
    partial last 64-coordinate tile) and padded rows (ldx > d), with NaN / inf
    columns, against the oracle."""
    import warnings
    rng = np.random.default_rng(n + d)
    full = make_rows(n, ldx, seed=d + n)
    full[rng.integers(0, n, 40), rng.integers(0, d, 40)] = np.nan
    full[rng.integers(0, n, 40), rng.integers(0, d, 40)] = np.inf
    full[rng.integers(0, n, 40), rng.integers(0, d, 40)] = -np.inf
    col = int(rng.integers(0, d))
    full[: n // 5, col] = np.nan              # more NaNs than the trim count -> NaN
    X = torch.from_numpy(full).cuda()[:, :d]
    x = full[:, :d]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        np.testing.assert_array_equal(engine.trimmed_mean(X).cpu().numpy(), orc.trimmed_mean(list(x)))
        np.testing.assert_array_equal(engine.median(X).cpu().numpy(), orc.median(list(x)))


@pytest.mark.parametrize("n", [129, 200, 256, 257, 300, 384, 511, 512])
def test_multilane_path_bitexact(n):
    """N in (128, 512]: 2 or 4 lanes per coordinate with DPP bitonic merges
    (exact N = 512 specialisation and runtime-N padding), NaN / inf / ties."""
    import warnings
    rng = np.random.default_rng(n)
    d = 5000 + n
    x = make_rows(n, d, seed=3 * n)
    x[:, :40] = rng.integers(-2, 3, size=(n, 40)).astype(np.float32)     # ties
    x[rng.integers(0, n, 60), rng.integers(0, d, 60)] = np.inf
    x[rng.integers(0, n, 60), rng.integers(0, d, 60)] = -np.inf
    x[rng.integers(0, n, 60), rng.integers(0, d, 60)] = np.nan
    x[: int(0.1 * n) + 1, 77] = np.nan                                  # NaN survives the trim
    X = torch.from_numpy(x).cuda()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        np.testing.assert_array_equal(engine.trimmed_mean(X).cpu().numpy(), orc.trimmed_mean(list(x)))
        np.testing.assert_array_equal(engine.median(X).cpu().numpy(), orc.median(list(x)))
        for beta in (0.0, 0.3):
            np.testing.assert_array_equal(engine.trimmed_mean(X, beta).cpu().numpy(), orc.trimmed_mean(list(x), beta))


@pytest.mark.parametrize("n", [100, 128, 129, 256, 512])
def test_denormals_and_signed_zeros_bitwise(n):
    """The plain networks recover each compare-exchange's max as a ^ b ^ min
    (csrc/sra_common.hpp ce_pair_plain), which is exact only if v_min_f32
    returns one of its operands bit for bit: columns of fp32 denormals of
    both signs, ±0, ±FLT_MAX and ±inf must come out as the oracle's bit
    patterns (compared as uint32, so -0 != +0), for the exact-N kernel
    (N = 100 / 128) and the multi-lane one (N > 128)."""
    rng = np.random.default_rng(77 + n)
    d = 2048 + 17
    x = make_rows(n, d, seed=n)
    tiny = np.float32(1.4e-45)
    pool = np.array([0.0, -0.0, tiny, -tiny, 3 * tiny, -7 * tiny, np.float32(1.1754942e-38),
                     -np.float32(1.1754942e-38), np.finfo(np.float32).max, -np.finfo(np.float32).max,
                     np.inf, -np.inf], np.float32)
    # a third of the columns entirely from the special pool, the rest salted
    cols = rng.choice(d, d // 3, replace=False)
    x[:, cols] = rng.choice(pool, size=(n, cols.size))
    x[rng.integers(0, n, 4000), rng.integers(0, d, 4000)] = rng.choice(pool, 4000)
    # all-negative-zero window columns (the sum starts from the first kept row)
    x[:, :3] = np.float32(-0.0)
    X = torch.from_numpy(x).cuda()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want_tm = np.asarray(orc.trimmed_mean(list(x)), np.float32)
        want_md = np.asarray(orc.median(list(x)), np.float32)
    got_tm = engine.trimmed_mean(X).cpu().numpy()
    got_md = engine.median(X).cpu().numpy()
    np.testing.assert_array_equal(got_tm, want_tm)
    np.testing.assert_array_equal(got_md, want_md)
    # bit patterns, except where the sorted kept window mixes -0 and +0 (numpy's
    # tie order among equal zeros is its sort's, not a defined one)
    srt = np.sort(x, axis=0)
    b = int(n * 0.1)
    win = srt[b:n - b]
    mixed = (np.signbit(win) & (win == 0)).any(axis=0) & (~np.signbit(win) & (win == 0)).any(axis=0)
    ok = ~mixed
    assert ok[:3].all()
    np.testing.assert_array_equal(got_tm.view(np.uint32)[ok], want_tm.view(np.uint32)[ok])
