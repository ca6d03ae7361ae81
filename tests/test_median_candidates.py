"""The one-read Bulyan median round (csrc/bulyan.hip median_pass_kernel /
median_finish_kernel) rests on a rule: after sorting the column of the n
remaining clients (NaN as +inf, padded to P = 16*ceil(n/16) slots with
(P - n) // 2 copies of -inf below and +inf above), the padded slots P/2 - 2,
P/2 - 1, P/2 (c0, c1, c2) and the NaN count determine the median of the column
with any one client k removed:
  n odd:  (c1 + c2), (c0 + c2) or (c0 + c1) times 0.5 as x_k <= c0, <= c1, above
  n even: c2 if x_k <= c1 else c1
  NaN if a NaN remains.
This checks the rule bit for bit against numpy's median of the reduced column
(robust_estimator.py:297-322 via oracle.robust_np.median semantics), with ties,
NaN and infinities.  CPU only: it restates the kernel's arithmetic in numpy."""
import numpy as np
import pytest


def candidates(col):
    n = col.shape[0]
    P = 16 * (-(-n // 16))
    kb = (P - n) // 2
    v = np.where(np.isnan(col), np.float32(np.inf), col).astype(np.float32)
    pad = np.concatenate([np.full(kb, -np.inf, np.float32), np.sort(v),
                          np.full(P - n - kb, np.inf, np.float32)])
    return pad[P // 2 - 2], pad[P // 2 - 1], pad[P // 2], int(np.isnan(col).sum())


def finish(c0, c1, c2, nan_cnt, n, x):
    half = np.float32(0.5)
    if n & 1:
        if x <= c0:
            res = (c1 + c2) * half
        elif x <= c1:
            res = (c0 + c2) * half
        else:
            res = (c0 + c1) * half
    else:
        res = c2 if x <= c1 else c1
    if nan_cnt - (1 if np.isnan(x) else 0) > 0:
        res = np.float32(np.nan)
    return np.float32(res)


def numpy_median(col):
    """np.median of a float32 column: NaN if any NaN, else the middle value or
    the fp32 mean of the two middle values (what select_dist_rows_kernel does)."""
    if np.isnan(col).any():
        return np.float32(np.nan)
    s = np.sort(col)
    m = len(s)
    if m & 1:
        return s[m // 2]
    return np.float32((s[m // 2 - 1] + s[m // 2]) * np.float32(0.5))


@pytest.mark.parametrize("n", [2, 3, 4, 5, 16, 17, 31, 32, 33, 47, 64, 87, 88, 100, 127, 128])
def test_rule_matches_median_of_reduced_column(n):
    rng = np.random.default_rng(1000 + n)
    for trial in range(60):
        kind = trial % 6
        if kind == 0:
            col = rng.standard_normal(n).astype(np.float32)
        elif kind == 1:      # heavy ties
            col = rng.integers(0, 3, n).astype(np.float32)
        elif kind == 2:      # one NaN
            col = rng.standard_normal(n).astype(np.float32)
            col[rng.integers(n)] = np.nan
        elif kind == 3:      # two NaNs and infinities
            col = rng.standard_normal(n).astype(np.float32)
            col[rng.integers(n)] = np.inf
            col[rng.integers(n)] = -np.inf
            if n >= 4:
                col[rng.choice(n, 2, replace=False)] = np.nan
        elif kind == 4:      # all equal
            col = np.full(n, np.float32(rng.standard_normal()))
        else:                # wide magnitudes
            col = (rng.standard_normal(n) * 10.0 ** rng.integers(-20, 20, n)).astype(np.float32)
        c0, c1, c2, nan_cnt = candidates(col)
        for k in range(n):
            want = numpy_median(np.delete(col, k))
            got = finish(c0, c1, c2, nan_cnt, n, col[k])
            assert (np.isnan(want) and np.isnan(got)) or want.tobytes() == got.tobytes(), (n, trial, k, want, got)
