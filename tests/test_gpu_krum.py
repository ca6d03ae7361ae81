"""GPU parity of the pairwise-L2 family (k2 Gram on MFMA + k3 client-space
scoring + k5 bucket means) against the golden fixtures and the oracle.

Tolerance: the Gram route computes ||x_i - x_j||^2 = G_ii + G_jj - 2 G_ij from
a centred fp32-MFMA Gram with an fp64 reduction, the reference computes each
distance with an fp32 BLAS dot of the difference; both carry ~1e-6 relative
error, so Krum scores are compared at rtol 1e-4 and the chosen index must be
identical (the fixtures have no near-ties)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import fixtures, gpu_available
from oracle import robust_np as orc
from synth import make_rows, make_clients

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from srfl_amd import engine, robust_estimator as gre

SCORE_RTOL = 1e-4

KR = fixtures(func="krum")
KR_ = fixtures(func="krum_")
MK = fixtures(func="mom_krum")


@pytest.mark.parametrize("rec", KR, ids=[r["name"] for r in KR])
def test_golden_krum(rec):
    xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
    got, idx = gre.krum(xs, rec["params"]["f"])
    assert idx == int(rec["index"])
    assert got is xs[idx]                       # alias semantics of the reference
    np.testing.assert_array_equal(got, rec["out"])


@pytest.mark.parametrize("rec", KR_, ids=[r["name"] for r in KR_])
def test_golden_krum_scores(rec):
    xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
    got = np.array(gre.krum_(xs, rec["params"]["f"]), dtype=np.float32)
    np.testing.assert_allclose(got, rec["out"], rtol=SCORE_RTOL, atol=1e-7)


@pytest.mark.parametrize("rec", MK, ids=[r["name"] for r in MK])
def test_golden_mom_krum(rec):
    xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
    got = gre.mom_krum(xs, rec["params"]["f"])
    np.testing.assert_array_equal(got, rec["out"])


@pytest.mark.parametrize("n", [1, 2, 3, 31, 32, 33, 64, 100, 128, 129, 160, 200, 256, 257, 300, 384, 512])
def test_gram_matches_fp64(n):
    d = 3000
    x = make_rows(n, d, seed=200 + n, byz=min(3, n // 4))
    X = torch.from_numpy(x).cuda()
    G = engine.gram(X).cpu().numpy()
    x64 = x.astype(np.float64)
    d2 = ((x64[:, None, :] - x64[None, :, :]) ** 2).sum(-1)
    got = np.diag(G)[:, None] + np.diag(G)[None, :] - 2 * G
    np.testing.assert_allclose(got, d2, rtol=2e-5, atol=1e-9 * d2.max())


@pytest.mark.parametrize("k", [1, 5, 257, 600])
def test_gram_n128_whole_stages(k):
    """N = 128 with d a multiple of the 128-coordinate stage: the software-
    pipelined Gram (gram_glds_kernel) when selected; workgroups with 0, 1, 2 and
    3 stages; identical rows keep distance exactly 0."""
    n, d = 128, 128 * k
    x = make_rows(n, d, seed=900 + k, byz=8, identical_byz=True)
    G = engine.gram(torch.from_numpy(x).cuda()).cpu().numpy()
    xc = x.astype(np.float64)
    xc -= xc.mean(axis=0)
    gc = xc @ xc.T
    d2 = np.maximum(np.diag(gc)[:, None] + np.diag(gc)[None, :] - 2 * gc, 0.0)
    got = np.diag(G)[:, None] + np.diag(G)[None, :] - 2 * G
    np.testing.assert_allclose(got, d2, rtol=2e-5, atol=1e-9 * d2.max())
    for i in range(8):
        for j in range(8):
            assert got[i, j] == 0.0


def test_identical_rows_zero_distance_and_unaligned():
    x = make_rows(40, 2051, seed=5, byz=8, identical_byz=True)
    X = torch.from_numpy(x).cuda()
    G = engine.gram(X[:, 3:]).cpu().numpy()        # unaligned base -> scalar staging path
    for i in range(8):
        for j in range(8):
            assert G[i, i] + G[j, j] - 2 * G[i, j] == 0.0


@pytest.mark.parametrize("n,f", [(128, 20), (100, 20), (64, 10), (20, 25), (129, 20), (200, 20), (256, 40),
                                 (300, 20), (512, 50), (512, 10), (512, 3)])   # m = 500, 507: three split levels
def test_krum_index_against_oracle(n, f):
    d = 20_000 if n <= 256 else 4_000
    x = make_rows(n, d, seed=300 + n, byz=min(f, n // 3))
    xs = list(x)
    want_scores = orc.krum_(xs, f)
    want_idx = int(np.argmin(want_scores))
    order, scores = engine.krum_select(torch.from_numpy(x).cuda(), f, 1)
    assert int(order.cpu()[0]) == want_idx
    np.testing.assert_allclose(scores.cpu().numpy(), np.array(want_scores, np.float32), rtol=SCORE_RTOL)


def test_device_krum_row_and_full_size():
    """C3-size (N=128, d=1e7): device in, device out, chosen row gathered on
    device; the pick and the scores checked against an independent fp64
    evaluation (torch's float64 GEMM of the full matrix, distances in fp64,
    the oracle's scoring), not against the kernel's own Gram."""
    g = torch.Generator(device="cuda").manual_seed(3)
    X = 0.01 * torch.randn(128, 10_000_000, device="cuda", generator=g)
    X[:20] = 0.05                         # far-away identical Byzantine group
    row, order = engine.krum(X, 20)
    idx = int(order.cpu()[0])
    assert idx >= 20
    assert torch.equal(row, X[idx])
    X64 = X.double()
    sq = (X64 * X64).sum(1)
    G64 = X64 @ X64.T
    del X64
    d2 = (sq[:, None] + sq[None, :] - 2.0 * G64).clamp_min(0.0).cpu().numpy()
    dist = np.sqrt(d2).astype(np.float32)
    want = orc.krum_scores_from_dist(dist, 20)
    assert idx == int(np.argmin(want))
    _, scores = engine.krum_select(X, 20, 1)
    np.testing.assert_allclose(scores.cpu().numpy(), np.asarray(want, np.float32), rtol=SCORE_RTOL)


def test_bucket_means_and_empty_bucket():
    x = make_rows(50, 1001, seed=9)
    X = torch.from_numpy(x).cuda()
    B = engine.bucket_means(X, 3, 17).cpu().numpy()
    want = np.array(orc.bucket_means(list(x), 3, 17))
    np.testing.assert_array_equal(B, want)
    with pytest.raises(ValueError):
        engine.bucket_means(X, 4, 14)     # bucket 13 would start at row 52 > 50


def test_identical_rows_zero_distance_pairs():
    """N > 256 (the pair path: 128-row blocks, one launch per pair, a common
    shift): identical clients spread over different blocks still get exactly
    zero distance."""
    x = make_rows(400, 3000, seed=6, byz=0)
    for r in (5, 130, 260, 399):
        x[r] = x[77]
    G = engine.gram(torch.from_numpy(x).cuda()).cpu().numpy()
    same = [77, 5, 130, 260, 399]
    for i in same:
        for j in same:
            assert G[i, i] + G[j, j] - 2 * G[i, j] == 0.0, (i, j)


@pytest.mark.parametrize("n,f", [(300, 20), (512, 100)])
def test_bulyan_krum_many_clients(n, f):
    """Bulyan-Krum with N > 256: the pair Gram, the 512-wide Krum rounds and
    (theta > 128) the LDS per-coordinate stage, against the oracle's selection."""
    x = make_rows(n, 300, seed=n + f, byz=f // 2)
    _, removed = orc.bulyan_select(list(x), f, "krum")
    _, sel = engine.bulyan(torch.from_numpy(x).cuda(), f, "krum", selected=True)
    assert sel.cpu().tolist() == removed


@pytest.mark.parametrize("n,f,d", [(600, 20, 3000), (1024, 100, 2000), (1100, 3, 2000), (2100, 40, 64)])
def test_krum_beyond_512_clients(n, f, d):
    """No client ceiling the reference lacks (robust_estimator.py:234-249 has
    none): N > 512 takes the pair Gram over 128-client blocks, the dynamic-LDS
    row sorts and the global-scratch rounds (krum_rounds_huge_kernel).
    m = 1095 (N = 1100, f = 3) needs four split levels of numpy's pairwise sum;
    d = 64 is the exact per-pair route."""
    x = make_rows(n, d, seed=310 + n, byz=min(f, n // 3))
    want = orc.krum_(list(x), f)
    order, scores = engine.krum_select(torch.from_numpy(x).cuda(), f, 1)
    assert int(order.cpu()[0]) == int(np.argmin(want))
    np.testing.assert_allclose(scores.cpu().numpy(), np.array(want, np.float32), rtol=SCORE_RTOL)


@pytest.mark.parametrize("n,f,d,rounds", [(700, 30, 3000, 6), (1500, 50, 128, 4)])
def test_krum_rounds_beyond_512_clients(n, f, d, rounds):
    """Bulyan-Krum-style rounds (delete the pick, re-score the rest with f
    fixed, robust_estimator.py:289-296) at N > 512, from the data and from the
    Gram (krum_from_gram, the sharded route's entry)."""
    x = make_rows(n, d, seed=410 + n, byz=f // 2)
    dist = orc.pairwise_l2(list(x))
    alive = list(range(n))
    want = []
    for _ in range(rounds):
        sc = orc.krum_scores_from_dist(dist[np.ix_(alive, alive)], f)
        want.append(alive.pop(int(np.argmin(sc))))
    X = torch.from_numpy(x).cuda()
    order, _ = engine.krum_select(X, f, rounds, scores=False)
    assert order.cpu().tolist() == want
    if d > 1024:
        order_g, _ = engine.krum_from_gram(engine.gram(X), f, rounds, scores=False)
        assert order_g.cpu().tolist() == want


def test_gram_beyond_512_clients():
    """The pair Gram at N = 1000 (8 blocks, 28 pair launches) against fp64."""
    n, d = 1000, 2500
    x = make_rows(n, d, seed=77, byz=5)
    G = engine.gram(torch.from_numpy(x).cuda()).cpu().numpy()
    xc = x.astype(np.float64)
    xc -= xc.mean(axis=0)
    gc = xc @ xc.T
    d2 = np.maximum(np.diag(gc)[:, None] + np.diag(gc)[None, :] - 2 * gc, 0.0)
    got = np.diag(G)[:, None] + np.diag(G)[None, :] - 2 * G
    np.testing.assert_allclose(got, d2, rtol=2e-5, atol=1e-9 * d2.max())


def test_gram_buckets_beyond_fused_range():
    """More than 192 buckets (a sharded mom_krum at N = 900): the bucket Gram
    falls back to the Gram of the materialised means; its distances match an
    fp64 evaluation of the means' distances, and sharded-style Krum over it
    picks the oracle's bucket."""
    n, d, f = 900, 3000, 20
    x = make_rows(n, d, seed=515, byz=30)
    X = torch.from_numpy(x).cuda()
    G = engine.gram_buckets(X, 3).cpu().numpy()
    B = np.array(orc.bucket_means(list(x), 3, 300), dtype=np.float64)
    Bc = B - B.mean(axis=0)
    gc = Bc @ Bc.T
    d2 = np.maximum(np.diag(gc)[:, None] + np.diag(gc)[None, :] - 2 * gc, 0.0)
    got = np.diag(G)[:, None] + np.diag(G)[None, :] - 2 * G
    # the means' spread is a third of the rows' while the Byzantine offset is
    # not, so the nearest pairs cancel more of G_ii + G_jj - 2 G_ij: the score
    # tolerance (SCORE_RTOL), not the raw-row Gram test's 2e-5
    np.testing.assert_allclose(got, d2, rtol=SCORE_RTOL, atol=1e-9 * d2.max())
    order, _ = engine.krum_from_gram(torch.from_numpy(G).cuda(), f, 1, scores=False)
    want = int(np.argmin(orc.krum_(list(B.astype(np.float32)), f)))
    assert int(order.cpu()[0]) == want
