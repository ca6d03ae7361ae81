"""GPU parity of the fused mom_krum route (csrc/gram_bucket.hip + krum.hip's
sra_mom_krum_f32): the bucket means of src/robust_estimator.py:250-256 are
formed inside the Gram's loads and never written.

Checked against
  * the oracle's bucket means (np.mean order) and an fp64 distance matrix of
    them: the fused Gram's distances at the Gram tolerance of test_gpu_krum.py;
  * the unfused route (sra_bucket_mean_f32 + sra_krum_select_f32): the same
    bucket and the returned row bit for bit;
  * the oracle's mom_krum: the returned row bit for bit (the fixtures of
    test_gpu_krum.py::test_golden_mom_krum run through the fused route too);
  * at the C5 per-GPU size (N = 512, d = 1.25e7), an independent fp64 torch
    evaluation of the bucket distances and the oracle's scoring.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import gpu_available
from oracle import robust_np as orc
from synth import make_rows

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    from srfl_amd import engine


def _bucket_means64(x, bs):
    nb = -(-x.shape[0] // bs)
    return np.array(orc.bucket_means(list(x), bs, nb)).astype(np.float64)


def _dist2(b64):
    return ((b64[:, None, :] - b64[None, :, :]) ** 2).sum(-1)


@pytest.mark.parametrize("n,bs", [(1, 3), (2, 3), (7, 3), (96, 3), (128, 3), (200, 3), (384, 3), (385, 3), (400, 3),
                                  (512, 3), (576, 3), (150, 1), (192, 1), (300, 2), (512, 4), (766, 4)])
def test_gram_buckets_matches_fp64(n, bs):
    d = 3000
    x = make_rows(n, d, seed=700 + n + bs, byz=min(9, n // 4))
    G = engine.gram_buckets(torch.from_numpy(x).cuda(), bs).cpu().numpy()
    d2 = _dist2(_bucket_means64(x, bs))
    got = np.diag(G)[:, None] + np.diag(G)[None, :] - 2 * G
    np.testing.assert_allclose(got, d2, rtol=2e-5, atol=1e-9 * max(d2.max(), 1e-30))


@pytest.mark.parametrize("n,f,bs,d", [(512, 20, 3, 20_000), (400, 10, 3, 4099), (128, 5, 3, 64), (96, 3, 3, 1),
                                      (300, 20, 2, 3001), (700, 30, 4, 5000), (150, 20, 1, 2000), (512, 60, 3, 777)])
def test_fused_equals_unfused_and_oracle(n, f, bs, d):
    x = make_rows(n, d, seed=n + f + d, byz=min(3 * f, n // 3))
    X = torch.from_numpy(x).cuda()
    row, order = engine.mom_krum(X, f, bs)
    row_u, order_u = engine.mom_krum(X, f, bs, fused=False)
    assert int(order.cpu()[0]) == int(order_u.cpu()[0])
    assert torch.equal(row, row_u)
    want = orc.mom_krum(list(x), f, bs)
    np.testing.assert_array_equal(row.cpu().numpy(), want)


def test_unaligned_and_strided_views():
    """Rows that are not 16-byte aligned / a row stride that is not a multiple
    of 4 take the guarded scalar loads; same pick and row as the unfused route."""
    x = make_rows(260, 4101, seed=11, byz=30)
    X = torch.from_numpy(x).cuda()
    for V in (X[:, 3:], X[:, 1:4000], X[::2, :]):
        row, order = engine.mom_krum(V, 10)
        row_u, order_u = engine.mom_krum(V, 10, fused=False)
        assert int(order.cpu()[0]) == int(order_u.cpu()[0])
        assert torch.equal(row, row_u)
        np.testing.assert_array_equal(row.cpu().numpy(), orc.mom_krum(list(V.cpu().numpy()), 10))


def test_identical_buckets_zero_distance():
    x = make_rows(384, 2048, seed=12, byz=0)
    for b in (3, 40, 127):           # buckets 3, 40, 127 take bucket 0's three clients
        x[3 * b:3 * b + 3] = x[0:3]
    G = engine.gram_buckets(torch.from_numpy(x).cuda(), 3).cpu().numpy()
    same = [0, 3, 40, 127]
    for i in same:
        for j in same:
            assert G[i, i] + G[j, j] - 2 * G[i, j] == 0.0, (i, j)


@pytest.mark.parametrize("kind", ["nan", "inf"])
def test_nonfinite_client_exact_route(kind):
    """A non-finite client makes its bucket mean non-finite: the Gram flags it and
    the distances come from the exact per-pair route, which forms the bucket
    means on the fly (krum.hip row_value)."""
    x = make_rows(300, 1500, seed=13, byz=15)
    x[100, 7] = np.nan if kind == "nan" else np.inf
    X = torch.from_numpy(x).cuda()
    row, order = engine.mom_krum(X, 10)
    row_u, order_u = engine.mom_krum(X, 10, fused=False)
    assert int(order.cpu()[0]) == int(order_u.cpu()[0])
    assert torch.equal(row.nan_to_num(), row_u.nan_to_num())
    with np.errstate(all="ignore"):
        want = orc.mom_krum(list(x), 10)
    np.testing.assert_array_equal(row.cpu().numpy(), want)


def test_c5_size_against_fp64():
    """C5 per-GPU shape (N = 512 clients, d = 1.25e7, 171 buckets of 3), a far
    Byzantine group of 60 clients (20 buckets): the fused pick equals the
    unfused one and the argmin of the oracle's scoring over an independent fp64
    distance matrix of the bucket means; the row equals that bucket's mean."""
    n, d, f = 512, 12_500_000, 20
    g = torch.Generator(device="cuda").manual_seed(5)
    X = 0.01 * torch.randn(n, d, device="cuda", generator=g)
    X += 0.001 * torch.randn(1, d, device="cuda", generator=g)
    X[:60] = -0.02
    row, order = engine.mom_krum(X, f)
    idx = int(order.cpu()[0])
    B = engine.bucket_means(X, 3, 171)
    assert torch.equal(row, B[idx])
    _, order_u = engine.mom_krum(X, f, fused=False)
    assert idx == int(order_u.cpu()[0])
    del X
    B64 = B.double()
    del B
    sq = (B64 * B64).sum(1)
    G64 = B64 @ B64.T
    del B64
    d2 = (sq[:, None] + sq[None, :] - 2.0 * G64).clamp_min(0.0).cpu().numpy()
    want = orc.krum_scores_from_dist(np.sqrt(d2).astype(np.float32), f)
    assert idx == int(np.argmin(want))
    assert idx >= 20
