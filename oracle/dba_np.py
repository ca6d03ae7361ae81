"""CPU oracle for the DBA harness's aggregators (src/DBA/helper.py).

TEST INFRASTRUCTURE ONLY -- like ``robust_np``, nothing in the product path
imports this module; only ``tests/`` use it, as the checker.

The DBA ``Helper`` re-implements the robust aggregators in torch with its own
semantics.  Each function below restates one of them over a client-major
``(N, D)`` float32 matrix ``X`` (the update dicts flattened in layer order) and
a layer table ``seg`` (column offsets, seg[0] = 0, seg[-1] = D), citing the
``helper.py`` lines it follows.  Parity pin: ``tests/test_dba_oracle.py``
checks every function against ``tests/golden/dba_*.npz``, produced by the LIVE
reference methods (``tests/golden/gen_dba_fixtures.py``).
"""
from __future__ import annotations

import math

import numpy as np

from . import robust_np as rn

HISTORY_TAU = 10.       # helper.py:58
SHARD_BUCKETS = 50      # helper.py:1151


def layers(seg):
    return [(int(seg[i]), int(seg[i + 1])) for i in range(len(seg) - 1)]


def _seq_sum(rows):
    acc = np.zeros(rows.shape[1], dtype=np.float32)
    for r in rows:
        acc = acc + r
    return acc


def fed_avg(X):
    """helper.py:251-289: torch.mean over the clients of every layer (fp32)."""
    return (_seq_sum(X) / np.float32(X.shape[0])).astype(np.float32)


def median(X):
    """helper.py:529-569: torch.median(dim=0).values -- the LOWER median
    s[(N-1)//2]; a NaN anywhere in a column gives NaN."""
    s = np.sort(X, axis=0)
    out = s[(X.shape[0] - 1) // 2].copy()
    out[np.isnan(X).any(axis=0)] = np.nan
    return out


def trimmed_mean(X, beta=0.1):
    """helper.py:892-930: torch.sort then torch.mean of s[b : N-b], b = int(N*beta)."""
    n = X.shape[0]
    b = int(n * beta)
    s = np.sort(X, axis=0)[b:n - b]
    return (_seq_sum(s) / np.float32(s.shape[0])).astype(np.float32)


def krum(X, seg, f=0):
    """helper.py:676-720: Krum PER LAYER (self excluded, N-f-2 nearest,
    non-squared L2); each layer takes its own argmin client's values."""
    out = np.empty(X.shape[1], dtype=np.float32)
    picks = []
    for lo, hi in layers(seg):
        i = int(np.argmin(rn.krum_(list(X[:, lo:hi]), f)))
        picks.append(i)
        out[lo:hi] = X[i, lo:hi]
    return out, picks


def mom_krum(X, bucket_size=3):
    """helper.py:833-890.  ``[copy.deepcopy(samples[0])] * bucket_num`` makes
    every bucket ONE dict (:859), so each layer ends as the LAST bucket's sum
    divided by (its size + 1) (:863), all buckets are identical, every Krum
    score is 0 and argmin picks bucket 0 -- that same tensor."""
    n = X.shape[0]
    nb = int(np.ceil(n * 1. / bucket_size))
    lo = (nb - 1) * bucket_size
    hi = min(nb * bucket_size, n)
    return (_seq_sum(X[lo:hi]) / np.float32(hi - lo + 1)).astype(np.float32)


def _krum_scores_self(dist, f):
    """helper.py:976-981: distances to ALL remaining clients including the
    zero self-distance, sum of the first size - i - f - 2 after argsort."""
    m = dist.shape[0]
    k = m - f - 2
    return np.array([np.sort(dist[j])[:k].sum() for j in range(m)])


def bulyan_select(X, f, aggsubfunc):
    """Selection rounds of Helper.bulyan_krum (:968-984), bulyan_median
    (:1018-1034) and bulyan_trimmed_mean (:1082-1103)."""
    n = X.shape[0]
    theta = n - 2 * f
    rows = [X[i].astype(np.float32) for i in range(n)]
    remaining = list(range(n))
    selected = []
    if aggsubfunc == "krum":
        dist = rn.pairwise_l2(rows)
        for _ in range(theta):
            sub = dist[np.ix_(remaining, remaining)]
            pick = int(np.argmin(_krum_scores_self(sub, f)))
            selected.append(rows[remaining.pop(pick)])
        return selected
    for i in range(theta):
        live = np.array([rows[j] for j in remaining])
        if aggsubfunc == "median":   # torch.median: the lower median, NaN propagates (:1038)
            agg = median(live)
        else:
            b = int((n - i) * 0.1)
            agg = trimmed_mean(live, 0.1) if b > 0 else fed_avg(live)
        selected.append(agg)
        best, best_d = None, np.inf
        for pos, r in enumerate(live):
            dd = float(np.sqrt(np.sum((agg.astype(np.float64) - r) ** 2)))
            if dd < best_d:
                best, best_d = pos, dd
        assert best is not None
        remaining.pop(best)
    return selected


def bulyan(X, seg, f, aggsubfunc):
    """Helper.bulyan_* per layer: selection, then the per-coordinate stage
    (:934-940) -- computed here with robust_np's fp64 rule, the one the device
    shares.  DBA evaluates that stage in fp32, where an even theta's exact tie
    between the two middle values is decided by rounding; ``bulyan_candidates``
    gives both outcomes for the tests."""
    theta = X.shape[0] - 2 * f
    if theta <= 0:
        raise RuntimeError("bulyan needs N > 2f")
    out = np.empty(X.shape[1], dtype=np.float64)
    for lo, hi in layers(seg):
        sel = np.array(bulyan_select(X[:, lo:hi], f, aggsubfunc), dtype=np.float64)
        out[lo:hi] = rn.bulyan_coordinates(sel, theta - 2 * f)
    return out


def bulyan_candidates(X, seg, f, aggsubfunc):
    """(2, D): the mean of the beta values nearest s[(theta-1)//2] and nearest
    s[theta//2] of each coordinate's theta selected values -- the two answers
    helper.py:934-940 can give (equal for odd theta)."""
    theta = X.shape[0] - 2 * f
    beta = theta - 2 * f
    out = np.empty((2, X.shape[1]), dtype=np.float64)
    for lo, hi in layers(seg):
        sel = np.array(bulyan_select(X[:, lo:hi], f, aggsubfunc), dtype=np.float64)
        s = np.sort(sel, axis=0)
        for w, k in enumerate(((theta - 1) // 2, theta // 2)):
            dist = np.abs(s - s[k][None, :])
            idx = np.argsort(dist, axis=0, kind="stable")[:beta]
            out[w, lo:hi] = np.take_along_axis(s, idx, axis=0).mean(axis=0)
    return out


def filterl2(X, seg, sigma=1, expansion=1, eps=0.2):
    """helper.py:607-674: per layer, itv = ITV = 1000 whatever the caller passes
    (:650), then filterl2_ (:571-605, the same iteration as robust_estimator's)."""
    out = np.empty(X.shape[1], dtype=np.float64)
    for lo, hi in layers(seg):
        out[lo:hi] = rn.filterL2(X[:, lo:hi].astype(np.float32), eps, sigma, expansion, 1000)
    return out


def ex_noregret(X, seg, eps=1. / 12, sigma=1, expansion=20, itv=1000):
    """helper.py:466-527: per layer; ``itv=None`` becomes int(sqrt(numel)) of
    the FIRST layer and is kept for the later ones (:507-508)."""
    out = np.empty(X.shape[1], dtype=np.float64)
    for lo, hi in layers(seg):
        if itv is None:
            itv = int(np.sqrt(hi - lo))
        out[lo:hi] = rn.ex_noregret(X[:, lo:hi].astype(np.float32), eps, sigma, expansion, itv)
    return out


def running_norm(X, prev, seg):
    """helper.py:753-757: norm = sqrt(norm + ||layer - prev||^2) after every layer."""
    nrm = np.zeros(X.shape[0])
    for lo, hi in layers(seg):
        sq = np.linalg.norm(X[:, lo:hi].astype(np.float64) - prev[lo:hi], axis=1) ** 2
        nrm = np.sqrt(nrm + sq)
    return nrm


def history(X, prev, seg, tau=HISTORY_TAU):
    """helper.py:722-777: clip every client against prev with the running norm
    (written back into the caller's dicts, :759), mean, prev <- mean.
    Returns (clipped rows, aggregate)."""
    if prev is None:
        prev = np.zeros(X.shape[1], dtype=np.float32)
    nrm = running_norm(X, prev, seg)
    with np.errstate(divide="ignore", invalid="ignore"):
        t = tau / nrm
    scale = np.where(t < 1, t, 1.0)
    clipped = (X.astype(np.float64) - prev) * scale[:, None]
    return clipped, clipped.mean(axis=0)


def shard_permutation(n, rnd):
    """random.shuffle(samples) of helper.py:1152 as a permutation of 0..n-1."""
    order = list(range(n))
    rnd.shuffle(order)
    return order


def sharding(X, rnd):
    """helper.py:1139-1166: shuffle, then 50 shards of ceil(N/50) consecutive
    clients, each averaged (copy + sequential += then /= count).  A shard that
    starts past the end raises IndexError like samples[begin_index]."""
    n = X.shape[0]
    order = shard_permutation(n, rnd)
    bs = int(np.ceil(n * 1. / SHARD_BUCKETS))
    out = []
    for i in range(SHARD_BUCKETS):
        b, e = i * bs, min((i + 1) * bs, n)
        if b >= n:
            raise IndexError("list index out of range")
        rows = X[order[b:e]]
        out.append(rows[0].copy() if e - b == 1 else (_seq_sum(rows) / np.float32(e - b)).astype(np.float32))
    return np.array(out)


def bucketing(X, prev, seg, rnd, tau=HISTORY_TAU):
    """helper.py:779-831: sharding (always), then history's clipping and mean."""
    return history(sharding(X, rnd), prev, seg, tau)


def geometric_median(X, ns, seg, maxiter=4, eps=1e-5, ftol=1e-6):
    """helper.py:327-410 (RFA, Weiszfeld).  Returns (median, calls, wv, dists)."""
    alphas = (np.asarray(ns, dtype=np.float64) / np.sum(ns)).astype(np.float32)

    def wavg(w):
        c = (w / np.float32(np.sum(w, dtype=np.float32))).astype(np.float32)
        acc = np.zeros(X.shape[1], dtype=np.float32)
        for ci, r in zip(c, X):
            acc = acc + np.float32(ci) * r
        return acc

    def dist(m):
        return np.sqrt(((X.astype(np.float64) - m) ** 2).sum(axis=1))

    def obj(m):
        return float(np.sum(alphas.astype(np.float64) * dist(m)))

    med = wavg(alphas)
    calls, ov, wv = 1, obj(med), None
    for _ in range(maxiter):
        prev_ov = ov
        w = (alphas / np.maximum(eps, dist(med))).astype(np.float32)
        w = (w / np.sum(w, dtype=np.float32)).astype(np.float32)
        med = wavg(w)
        calls += 1
        ov = obj(med)
        if abs(prev_ov - ov) < ftol * ov:
            break
        wv = w.copy()
    if wv is None:
        raise AttributeError("'NoneType' object has no attribute 'cpu'")   # helper.py:408 on an early break
    return med, calls, wv, dist(med)


def update_norm(v):
    return math.sqrt(float(np.sum(np.asarray(v, dtype=np.float64) ** 2)))


def foolsgold_weights(grads):
    """FoolsGold.foolsgold (helper.py:1388-1417): cosine similarity of the client
    features (sklearn: rows scaled to unit L2 norm, zero rows left as they are),
    pardoning, clip, rescale, logit.  Returns (wv, alpha) -- the values the
    reference holds when its ``return wv,alpha(base)`` raises NameError."""
    g = np.asarray(grads, dtype=np.float64)
    n = g.shape[0]
    nrm = np.sqrt(np.einsum("ij,ij->i", g, g))
    nrm[nrm == 0.0] = 1.0
    u = g / nrm[:, None]
    cs = u @ u.T - np.eye(n)
    maxcs = np.max(cs, axis=1)
    for i in range(n):
        for j in range(n):
            if i != j and maxcs[i] < maxcs[j]:
                cs[i][j] = cs[i][j] * maxcs[i] / maxcs[j]
    wv = 1 - np.max(cs, axis=1)
    wv[wv > 1] = 1
    wv[wv < 0] = 0
    alpha = np.max(cs, axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        wv = wv / np.max(wv)
        wv[(wv == 1)] = .99
        wv = np.log(wv / (1 - wv)) + 0.5
    wv[(np.isinf(wv) + wv > 1)] = 1
    wv[(wv < 0)] = 0
    return wv, alpha


def foolsgold_features(X, seg, memory, names, use_memory):
    """FoolsGold.aggregate_gradients (helper.py:1328-1345): the second-to-last
    layer of every client in fp64, accumulated per client name into ``memory``
    (a dict, updated in place); returns the matrix FoolsGold weighs."""
    lo, hi = int(seg[-3]), int(seg[-2])
    grads = X[:, lo:hi].astype(np.float64)
    mem = np.zeros_like(grads)
    for i, nm in enumerate(names):
        memory[nm] = memory[nm] + grads[i] if nm in memory else grads[i].copy()
        mem[i] = memory[nm]
    return mem if use_memory else grads
