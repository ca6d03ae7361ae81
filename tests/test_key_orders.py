"""CPU checks of two arithmetic facts the round-6 kernels rely on.

1. ``x + (-0.0f) == x`` bit for bit for every float32 x (NaN stays NaN): the
   Bulyan trimmed-mean window sum (csrc/bulyan.hip, select_dist_rows_kernel)
   adds -0 for edge slots outside the window instead of branching, and must
   stay bit-identical with numpy's sequential sum (robust_estimator.py:223-232).
2. The Krum-round argmin key (csrc/krum.hip, krum_rounds_kernel): one uint64
   per row, (class 0 NaN / 1 number / 2 removed) << 48 | order-preserving
   value bits << 16 | index, whose minimum is np.argmin's pick over the alive
   rows -- the first NaN if any, else the first minimum, -0 equal to +0
   (robust_estimator.py:240-244, np.argmin semantics).
"""
import numpy as np


def _f32_bits(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def test_neg_zero_is_additive_identity():
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.17549435e-38,
                         -1.17549435e-38, 3.4028235e38, -3.4028235e38, 1.0, -1.0], dtype=np.float32)
    rng = np.random.default_rng(0)
    rand = rng.standard_normal(4096).astype(np.float32) * np.float32(1e3)
    bits = rng.integers(0, 2**32, size=4096, dtype=np.uint64).astype(np.uint32).view(np.float32)
    for xs in (specials, rand, bits):
        with np.errstate(invalid="ignore"):   # signalling-NaN bit patterns
            y = xs + np.float32(-0.0)
        nan = np.isnan(xs)
        assert np.array_equal(np.isnan(y), nan)
        assert np.array_equal(_f32_bits(y[~nan]), _f32_bits(xs[~nan]))
    # and a sequential sum with -0 terms interleaved is the same sum
    v = rng.standard_normal(200).astype(np.float32)
    acc_a = np.float32(0.0)
    acc_b = np.float32(0.0)
    for x in v:
        acc_a = np.float32(acc_a + x)
        acc_b = np.float32(np.float32(acc_b + x) + np.float32(-0.0))
    assert _f32_bits(acc_a) == _f32_bits(acc_b)


def _key(score, alive, i):
    v = np.float32(score)
    if not alive:
        cls = 2
        ob = 0
    elif np.isnan(v):
        cls = 0
        ob = 0
    else:
        cls = 1
        b = int(_f32_bits(np.float32(v + np.float32(0.0))))   # -0 -> +0
        ob = (~b) & 0xFFFFFFFF if b & 0x80000000 else b | 0x80000000
    return (cls << 48) | (ob << 16) | i


def _reference_pick(scores, alive):
    idx = [i for i in range(len(scores)) if alive[i]]
    if not idx:
        return -1
    sub = np.asarray([scores[i] for i in idx], dtype=np.float32)
    return idx[int(np.argmin(sub))]   # np.argmin: first NaN, else first minimum


def test_krum_argmin_key_matches_numpy():
    rng = np.random.default_rng(1)
    pool = np.array([0.0, -0.0, 1.0, 2.0, np.inf, np.nan, 1e-45, 3.0e38], dtype=np.float32)
    for trial in range(3000):
        n = int(rng.integers(1, 130))
        if trial % 3 == 0:
            scores = rng.choice(pool, size=n)                       # ties, signed zeros, NaN, inf
        else:
            scores = rng.standard_normal(n).astype(np.float32) ** 2
            if trial % 5 == 0:
                scores[rng.integers(0, n)] = np.nan
        alive = rng.random(n) < 0.8
        keys = [_key(scores[i], bool(alive[i]), i) for i in range(n)]
        best = min(keys)
        cls, bi = best >> 48, best & 0xFFFF
        pick = bi if cls < 2 else -1
        assert pick == _reference_pick(scores, alive), (trial, scores, alive)
