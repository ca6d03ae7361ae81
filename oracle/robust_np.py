"""CPU oracle: a numpy restatement of the reference's robust aggregators.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path imports this module:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use it, and there only as the checker / the timed CPU port.  The
product path (``secure-robust-federated-learning_amd``) fails loudly when its
HIP library is missing; it never falls back to this file.

Each function restates the algorithm of the reference
(wanglun1996/secure-robust-federated-learning @ v1, ``src/robust_estimator.py``
and the inline aggregators of ``src/simulate.py``) from its observable
behaviour, citing the reference ``file:line`` it follows.  The numpy operations
are chosen so that the floating-point evaluation order matches the reference
where that is cheap (sequential axis-0 sums, numpy pairwise sums, BLAS dots),
which is what makes ``median``/``trimmed_mean``/``bulyan`` bit-exact against the
golden fixtures in ``tests/golden`` (generated from the live reference by
``tests/golden/gen_fixtures.py``).

Parity pin: ``tests/test_oracle_golden.py`` checks every function here against
those fixtures.  The reference ships no golden vectors of its own (SURVEY.md
§4, §8c), so the fixtures are the only pin.
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import eigh
from scipy.special import rel_entr

ITV = 1000        # robust_estimator.py:40
MAX_ITER = 100    # robust_estimator.py:39 (unused by the reference too)


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------
def _as_rows(samples):
    """Stack a list of same-shape arrays into (N, D) plus the layer shape."""
    arr = np.array(samples)
    return arr.reshape(arr.shape[0], -1), arr.shape[1:]


def _l2(v):
    """np.linalg.norm(v) for ord=None: sqrt(dot(ravel, ravel)) in v's dtype."""
    flat = v.ravel(order="K")
    return np.sqrt(flat.dot(flat))


def pairwise_l2(rows):
    """Symmetric matrix of ||x_i - x_j|| (robust_estimator.py:242 evaluates the
    same BLAS dot per ordered pair; (a-b) and (b-a) give bitwise-equal dots, so
    only i<j is evaluated here)."""
    n = len(rows)
    out = np.zeros((n, n), dtype=np.result_type(rows[0].dtype, np.float32))
    for i in range(n):
        for j in range(i + 1, n):
            out[i, j] = out[j, i] = _l2(rows[i] - rows[j])
    return out


def krum_scores_from_dist(dist, f):
    """Krum metric from a distance matrix (robust_estimator.py:234-244).

    score_i = numpy pairwise sum of the (n-f-2) smallest distances from i to
    the other clients, with Python slice semantics for a non-positive count.
    """
    n = dist.shape[0]
    keep = n - f - 2
    scores = []
    for i in range(n):
        others = np.delete(dist[i], i)
        scores.append(np.sort(others)[:keep].sum())
    return scores


def bucket_count(n, eps, delta):
    """Bucket count/size of the MoM wrappers (robust_estimator.py:136-137, 211-212),
    evaluated in float64 exactly as the reference does."""
    num = int(np.floor(eps * n) + np.log(1.0 / delta))
    size = int(np.ceil(n * 1.0 / num))
    return num, size


def bucket_means(samples, bucket_size, bucket_num):
    """Means of consecutive buckets in list order (robust_estimator.py:138-140,
    213-216, 254-256).  An empty trailing bucket yields a NaN scalar, which the
    reference's later ``np.array`` rejects with ValueError; reproduce that."""
    n = len(samples)
    means = []
    for b in range(bucket_num):
        lo, hi = b * bucket_size, min((b + 1) * bucket_size, n)
        if hi <= lo:
            raise ValueError("empty bucket %d (N=%d, bucket_size=%d, buckets=%d)"
                             % (b, n, bucket_size, bucket_num))
        means.append(np.mean(samples[lo:hi], axis=0))
    return means


def chunk_sizes(feature_size, itv):
    """itv-wide chunks of a flattened layer, last one partial
    (robust_estimator.py:116-124, 192-200)."""
    if itv is None:
        itv = int(np.floor(np.sqrt(feature_size)))
    full = int(feature_size // itv)
    sizes = [itv] * full
    if feature_size % itv:
        sizes.append(feature_size - full * itv)
    return sizes


# ----------------------------------------------------------------------------
# coordinate-wise
# ----------------------------------------------------------------------------
def average(samples):
    """Inline ``--agg average`` (simulate.py:235-244): np.average(axis=0)."""
    return np.array(samples).mean(axis=0)


def median(samples):
    """robust_estimator.py:220-221: coordinate-wise np.median over clients."""
    return np.median(np.asarray(samples), axis=0)


def trimmed_mean(samples, beta=0.1):
    """robust_estimator.py:223-232: sort along clients, drop int(N*beta) from
    each end, mean of the rest (sequential fp32 sum in ascending order)."""
    stacked = np.array(samples)
    n = stacked.shape[0]
    cut = int(n * beta)
    ordered = np.sort(stacked, axis=0)
    return ordered[cut:n - cut].mean(axis=0)


# ----------------------------------------------------------------------------
# Krum family
# ----------------------------------------------------------------------------
def krum_(samples, f):
    """robust_estimator.py:234-244 (list of per-client Krum scores)."""
    rows = [np.asarray(s) for s in samples]
    return krum_scores_from_dist(pairwise_l2(rows), f)


def krum(samples, f):
    """robust_estimator.py:246-249: the client with the smallest score (first on
    ties); returns the caller's own object and its index."""
    scores = krum_(samples, f)
    idx = int(np.argmin(scores))
    return samples[idx], idx


def mom_krum(samples, f, bucket_size=3):
    """robust_estimator.py:251-257 (``--agg clustering``, simulate.py:389-397)."""
    num = int(np.ceil(len(samples) * 1.0 / bucket_size))
    return krum(bucket_means(samples, bucket_size, num), f=f)[0]


# ----------------------------------------------------------------------------
# Bulyan
# ----------------------------------------------------------------------------
def bulyan_median(arr):
    """robust_estimator.py:259-270 for one coordinate: index minimising the
    total |a_i - a_j| (numpy pairwise fp64 row sum, first index) and its row."""
    a = np.asarray(arr, dtype=np.float64)
    dist = np.abs(a[:, None] - a[None, :])
    np.fill_diagonal(dist, 0.0)   # the reference never writes the diagonal (np.zeros): |inf - inf| is not NaN there
    total = dist.sum(axis=-1)
    m = int(np.argmin(total))
    return m, dist[m]


def bulyan_one_coordinate(arr, beta):
    """robust_estimator.py:272-275: mean of the beta values nearest the
    Bulyan median (argsort order, numpy pairwise mean)."""
    _, row = bulyan_median(arr)
    return np.mean(np.asarray(arr)[np.argsort(row)[:beta]])


def bulyan_coordinates(selected, beta, block=2048):
    """Vectorised robust_estimator.py:324-330: bulyan_one_coordinate for every
    coordinate of the (theta, D) float64 matrix ``selected``.

    The (block, theta, theta) distance cube is reduced over its contiguous last
    axis, which makes numpy use the same pairwise row sum as the reference's
    per-coordinate theta x theta matrix; argsort/mean run per row with the same
    kernels as the reference's 1-D calls."""
    sel = np.ascontiguousarray(np.asarray(selected, dtype=np.float64).T)  # (D, theta)
    d = sel.shape[0]
    out = np.empty(d, dtype=np.float64)
    for lo in range(0, d, block):
        a = sel[lo:lo + block]
        cube = np.abs(a[:, :, None] - a[:, None, :])
        idx = np.arange(a.shape[1])
        cube[:, idx, idx] = 0.0   # diagonal stays 0 in the reference (np.zeros), even for inf / NaN values
        med = cube.sum(axis=-1).argmin(axis=-1)
        row = cube[np.arange(a.shape[0]), med]
        order = np.argsort(row, axis=-1)[:, :beta]
        out[lo:lo + block] = np.take_along_axis(a, order, axis=-1).mean(axis=-1)
    return out


def _pw64(a):
    """numpy's pairwise float64 summation order, restated (loops_utils.h.src)."""
    n = len(a)
    if n < 8:
        r = 0.0
        for v in a:
            r += v
        return r
    if n <= 128:
        acc = [a[k] for k in range(8)]
        i = 8
        while i < n - (n % 8):
            for k in range(8):
                acc[k] += a[i + k]
            i += 8
        res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]))
        while i < n:
            res += a[i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pw64(a[:n2]) + _pw64(a[n2:])


def bulyan_keep(theta, beta):
    """How many values ``arr[np.argsort(row)[:beta]]`` keeps (Python slice
    semantics, robust_estimator.py:274): a negative beta (2f < N < 4f, e.g.
    N=100 with malnum 30) drops -beta from the far end."""
    return min(beta, theta) if beta >= 0 else max(theta + beta, 0)


def bulyan_one_coordinate_leftfirst(arr, beta):
    """bulyan_one_coordinate with a DEFINED tie rule for the beta-nearest set.

    The reference takes np.argsort(distances)[:beta]; numpy's quicksort is
    unstable, so when a value left of the Bulyan median and one right of it are
    at exactly the same distance, which one enters the set depends on the numpy
    build (introsort in 1.21, x86-simd-sort AVX-512 in 2.x).  This restatement
    (and the GPU kernel) grows the window left-first on such ties; everywhere
    else it equals the reference bit for bit.  A NaN among the values makes
    every total distance NaN, so np.argmin picks index 0 and NaN distances sort
    last; infinities change the centre too (robust_estimator.py:261-275)."""
    a = np.asarray(arr, dtype=np.float64)
    theta = len(a)
    keep = bulyan_keep(theta, beta)
    if not np.isfinite(a).all():
        # NaN makes every total NaN (argmin -> 0); one infinity makes every total
        # infinite (-> 0); two equal infinities sit at NaN distance (-> the first
        # of them).  Restated by definition: argsort of the distance row with NaN
        # last, equal distances smaller value first, then index.
        m, row = bulyan_median(a)
        row = np.where(np.arange(theta) == m, 0.0, row)
        key_nan = np.isnan(row)
        order = np.lexsort((np.arange(theta), np.where(key_nan, 0.0, a), np.where(key_nan, 0.0, row), key_nan))
        if keep == 0:
            return np.nan
        return _pw64([a[k] for k in order[:keep]]) / keep
    m, _ = bulyan_median(a)
    am = a[m]
    v = np.sort(a)
    live = len(v)
    if keep == 0:
        return np.nan
    pl = int(np.searchsorted(v, am, side="left"))
    pr = int(np.searchsorted(v, am, side="right")) - 1
    seq = [am] * min(pr - pl + 1, keep)
    l, r = pl, pr
    while len(seq) < keep:
        dl = am - v[l - 1] if l > 0 else np.inf
        dr = v[r + 1] - am if r < live - 1 else np.inf
        if dl <= dr:
            l -= 1
            seq.append(v[l])
        else:
            r += 1
            seq.append(v[r])
    return _pw64(seq) / keep


def bulyan_boundary_tie(arr, beta):
    """True when the beta-nearest set of a coordinate is ambiguous: values on
    both sides of the Bulyan median at exactly the boundary distance."""
    a = np.asarray(arr, dtype=np.float64)
    m, row = bulyan_median(a)
    keep = bulyan_keep(len(a), beta)
    if keep <= 0 or keep >= len(a) or np.isnan(a).any():
        return False
    dist = np.sort(row)
    cut = dist[keep - 1]
    if dist[keep] != cut:
        return False
    at = a[row == cut]
    return bool((at < a[m]).any() and (at > a[m]).any())


def bulyan_select(rows, f, aggsubfunc):
    """The theta selection rounds of robust_estimator.py:286-322.

    Returns (selected vectors, trace of removed client indices into ``rows``).
    ``krum`` appends the Krum-chosen client itself; ``median`` and
    ``trimmedmean`` append the aggregate vector and then drop the client
    nearest to it (first strict minimum)."""
    n = len(rows)
    theta = n - 2 * f
    remaining = list(range(n))
    selected, removed = [], []
    if aggsubfunc == "krum":
        dist = pairwise_l2(rows)
        for _ in range(theta):
            sub = dist[np.ix_(remaining, remaining)]
            pick = int(np.argmin(krum_scores_from_dist(sub, f)))
            client = remaining.pop(pick)
            selected.append(rows[client])
            removed.append(client)
    elif aggsubfunc in ("median", "trimmedmean"):
        for _ in range(theta):
            live = [rows[i] for i in remaining]
            agg = median(live) if aggsubfunc == "median" else trimmed_mean(live)
            selected.append(agg)
            best, best_d = None, np.inf
            for pos, r in enumerate(live):
                dd = _l2(agg - r)
                if dd < best_d:
                    best, best_d = pos, dd
            if best is None:
                # every distance NaN / inf: `assert min_index != None`
                # (robust_estimator.py:308, 321)
                raise AssertionError("bulyan %s round: no finite distance" % aggsubfunc)
            removed.append(remaining.pop(best))
    return selected, removed


def bulyan(grads, f, aggsubfunc="trimmedmean"):
    """robust_estimator.py:277-332."""
    rows, shape = _as_rows(grads)
    rows = [r for r in rows]
    n = len(rows)
    theta = n - 2 * f
    if theta <= 0:
        # the reference indexes an empty selection (robust_estimator.py:327)
        raise IndexError("bulyan needs N > 2f (theta=%d)" % theta)
    selected, _ = bulyan_select(rows, f, aggsubfunc)
    if not selected:
        raise IndexError("bulyan selected no gradients")
    sel = np.array([np.asarray(g, dtype=np.float64).ravel() for g in selected])
    beta = theta - 2 * f
    return bulyan_coordinates(sel, beta).reshape(shape)


# ----------------------------------------------------------------------------
# spectral filters
# ----------------------------------------------------------------------------
def _weighted_cov(centered, c, order="gemm"):
    """The weighted covariance of robust_estimator.py:158; ``order="reverse"``
    sums the clients' outer products in reverse client order instead (the same
    mathematics in another fp64 evaluation order, used to measure how far the
    reference's own result moves under rounding: tests/test_gpu_filters.py)."""
    if order == "reverse":
        z, w = centered[::-1], c[::-1]
        return (z.T * w) @ z / w.sum()
    return (centered.T * c) @ centered / c.sum()


def _top_eig(z, c, order):
    """Top eigenpair (lambda, unit v) of the weighted covariance of the centred
    chunk z (robust_estimator.py:158-161).  order "gemm" / "reverse": LAPACK on
    the k x k covariance (the reference's primal form, two fp64 client orders);
    "dual": LAPACK on the n x n matrix M = W^1/2 Z Z^T W^1/2 (w = c / sum c),
    whose nonzero spectrum is the covariance's, v = Z^T W^1/2 u / |.| -- the
    same mathematics ~100x faster at n = 128, k = 1000, used as the checker of
    the full-size device traces (tests/test_gpu_filter_trace.py)."""
    k = z.shape[1]
    if order in ("dual", "dual_reverse"):
        # dual_reverse: the same with the clients in reverse order (another
        # rounding of the same mathematics)
        n = z.shape[0]
        p = np.arange(n)[::-1] if order == "dual_reverse" else np.arange(n)
        sw = np.sqrt(c[p] / c[p].sum())
        zs = z[p] * sw[:, None]
        lam, u = eigh(zs @ zs.T, subset_by_index=[n - 1, n - 1])
        v = z[p].T @ (sw * u[:, 0])
        return lam[0], v / np.linalg.norm(v)
    lam, vec = eigh(_weighted_cov(z, c, order), subset_by_index=[k - 1, k - 1])
    return lam[0], vec[:, 0]


def _perturbed(c, perturb, it):
    """Test helper: c * (1 + scale * N(0,1)) with a per-(seed, iteration)
    stream -- a rounding-sized nudge of the weights, used to find which
    decisions of a chunk are robust to the rounding of an implementation."""
    if perturb is None:
        return c
    seed, scale = perturb
    return c * (1.0 + scale * np.random.default_rng((seed, it)).standard_normal(c.shape))


def filterL2_(samples, eps=0.2, sigma=1, expansion=20, order="gemm", trace=None, perturb=None):
    """robust_estimator.py:144-177 on one (n, k) chunk (primal k x k form).

    ``trace``: a list; one record per call is appended -- the decisions the
    reference makes (:163-174): ``removed`` = the ORIGINAL index of the
    argmax-tau client dropped at each iteration (first index on ties),
    ``iters`` = the iterations completed (< T when the early exit of :163-164
    fired), ``margin`` = (tau_max - tau_2nd) / tau_max per iteration (how
    close each removal was to a tie)."""
    x = np.asarray(samples)
    n0, k = x.shape
    c = np.ones(n0)
    alive = list(range(n0))
    rec = {"removed": [], "margin": [], "iters": 0} if trace is not None else None
    if rec is not None:
        trace.append(rec)
    for it in range(2 * int(eps * n0)):
        c = _perturbed(c, perturb, it)
        mu = np.average(x, axis=0, weights=c)
        z = x - mu
        lam, vec = _top_eig(z, c, order)
        if lam * lam <= expansion * sigma * sigma:
            return mu
        tau = (z @ vec) ** 2
        top = int(np.argmax(tau))
        if rec is not None:
            srt = np.sort(tau)
            rec["removed"].append(alive.pop(top))
            rec["margin"].append(float((srt[-1] - srt[-2]) / srt[-1]) if len(srt) > 1 else 1.0)
            rec["iters"] = it + 1
        c = c * (1 - tau / tau[top])
        x = np.delete(x, top, axis=0)
        c = np.delete(c, top)
        c = c / np.abs(c).sum()
    return np.average(x, axis=0, weights=c)


def _chunked(samples, itv, fn):
    rows, shape = _as_rows(samples)
    out, lo = [], 0
    for size in chunk_sizes(rows.shape[1], itv):
        out.append(fn(rows[:, lo:lo + size]))
        lo += size
    return np.concatenate(out, axis=0).reshape(shape)


def filterL2(samples, eps=0.2, sigma=1, expansion=20, itv=ITV, order="gemm", trace=None, perturb=None):
    """robust_estimator.py:180-208: filterL2_ over itv-wide chunks (``trace``:
    one filterL2_ record per chunk, in chunk order)."""
    return _chunked(samples, itv, lambda ch: filterL2_(ch, eps, sigma, expansion, order, trace, perturb))


def mom_filterL2(samples, eps=0.2, sigma=1, expansion=20, itv=ITV, delta=np.exp(-30), order="gemm",
                 trace=None, perturb=None):
    """robust_estimator.py:210-218 (trace: bucket indices, see filterL2_)."""
    num, size = bucket_count(len(samples), eps, delta)
    return filterL2(bucket_means(samples, size, num), eps, sigma, expansion, itv, order, trace, perturb)


def kl_capped_projection(c, eps, info=None):
    """The projection step of robust_estimator.py:77-99: among the candidates
    that cap the i+1 largest weights at 1/((1-eps)n) and rescale the rest to sum
    to one, keep the feasible one with the smallest KL(c || c_) (first on ties).
    Returns None when no candidate is feasible (the reference then fails on the
    next iteration).  ``info`` (a dict): ``capped`` = i+1 of the kept candidate,
    ``margin`` = relative KL gap to the runner-up (1.0 with a single feasible
    candidate)."""
    n = len(c)
    cap = 1.0 / (1 - eps) / n
    desc = np.argsort(c)[::-1]
    best, best_kl, best_i, kls = None, None, -1, []
    for i in range(n):
        head, tail = desc[:i + 1], desc[i + 1:]
        cand = c.copy()
        cand[head] = cap
        clip = 1 - cand[head].sum()
        if clip <= 0:
            break
        scale = clip / cand[tail].sum()
        cand[tail] = cand[tail] * scale
        if cand[tail[0]] > cap:
            continue
        kl = rel_entr(c, cand).sum()
        kls.append(kl)
        if best_kl is None or kl < best_kl:
            best, best_kl, best_i = cand, kl, i
    if info is not None:
        info["capped"] = best_i + 1
        srt = np.sort(kls)
        info["margin"] = float((srt[1] - srt[0]) / max(abs(srt[0]), 1e-300)) if len(srt) > 1 else 1.0
    return best


def ex_noregret_(samples, eps=1. / 12, sigma=1, expansion=20, dis_threshold=0.7, trace=None, order="gemm",
                 perturb=None):
    """robust_estimator.py:42-102 on one (n, k) chunk.  ``trace``: a list; one
    record per call is appended -- ``kept`` = the clients the Krum pre-filter
    keeps (:49-51, ascending original indices), ``capped`` = how many weights
    the chosen KL projection candidate caps at each iteration (:78-99),
    ``iters`` = the iterations completed (< T on the early exit :71-72),
    ``margin`` = the candidate's relative KL gap to the runner-up."""
    x = np.asarray(samples)
    n = len(x)
    f = int(np.ceil(eps * n))
    scores = krum_(list(x), f)
    keep = np.argpartition(scores, -f)[:-f]
    rec = None
    if trace is not None:
        rec = {"kept": sorted(int(i) for i in keep), "capped": [], "margin": [], "iters": 0}
        trace.append(rec)
    x = x[keep]
    m, k = x.shape
    if m < 2:
        # np.amax of the empty pairwise-distance list (f = 0 keeps nothing; one
        # client has no pair) raises ValueError in the reference
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    far = pairwise_l2(list(x))
    step = 0.5 / (np.amax(far[np.triu_indices(m, 1)]) ** 2)
    c = np.ones(m)
    for it in range(int(2 * eps * m)):
        if c is None:
            # the previous projection was infeasible (projected_c = None, :99):
            # np.average(weights=None) is the plain fp32 mean, the covariance
            # the fp32 mean of fp32 outer products, eigh in fp32 (:65-69); the
            # early exit returns that mean (:71-72), otherwise the update
            # c * (1 - step * tau) raises TypeError (:75)
            mu32 = np.average(x, axis=0)
            z32 = x - mu32
            cov32 = np.average(np.array([np.outer(r, r) for r in z32]), axis=0)
            lam32 = eigh(cov32, subset_by_index=[k - 1, k - 1], eigvals_only=True)[0]
            if lam32 * lam32 <= expansion * sigma * sigma:
                return mu32
            raise TypeError("unsupported operand type(s) for *: 'NoneType' and 'float' (ex_noregret, :75)")
        c = _perturbed(c, perturb, it)
        mu = np.average(x, axis=0, weights=c)
        z = x - mu
        lam, vec = _top_eig(z, c, order)
        if lam * lam <= expansion * sigma * sigma:
            return mu
        tau = (z @ vec) ** 2
        c = c * (1 - step * tau)
        info = {}
        c = kl_capped_projection(c, eps, info)
        if rec is not None:
            rec["capped"].append(info["capped"])
            rec["margin"].append(info["margin"])
            rec["iters"] = it + 1
    if c is None:
        # infeasible at the last iteration: the final np.average(weights=None) (:101)
        return np.average(x, axis=0)
    return np.average(x, axis=0, weights=c)


def ex_noregret(samples, eps=1. / 12, sigma=1, expansion=20, itv=ITV, trace=None, order="gemm"):
    """robust_estimator.py:104-133: ex_noregret_ over itv-wide chunks."""
    return _chunked(samples, itv, lambda ch: ex_noregret_(ch, eps, sigma, expansion, trace=trace, order=order))


def mom_ex_noregret(samples, eps=0.2, sigma=1, expansion=20, itv=ITV, delta=np.exp(-30), trace=None,
                    order="gemm"):
    """robust_estimator.py:135-142."""
    num, size = bucket_count(len(samples), eps, delta)
    return ex_noregret(bucket_means(samples, size, num), eps, sigma, expansion, itv, trace, order)


PERTURB_TRIALS = 4
PERTURB_SCALE = 1e-13


def trace_pair(args):
    """Test helper (picklable for a process pool): decision traces of one
    (n, k) chunk from the client-space oracle in two client orders ("dual",
    "dual_reverse") and PERTURB_TRIALS runs whose weights are nudged by
    PERTURB_SCALE relative noise every iteration.  args = (x, mode, eps,
    sigma, expansion).  Returns (row, agree, margin): row = the "dual" run's
    [iters, decision(n), active flag(n)] (trace_array layout + flags), agree =
    the leading iterations on which every run makes the same decision (a
    decision that a 1e-13 nudge flips is a near-tie decided by rounding), and
    the "dual" run's per-iteration margins."""
    x, mode, eps, sigma, expansion = args
    import warnings
    n = x.shape[0]
    runs = [("dual", None), ("dual_reverse", None)] + [("dual", (s, PERTURB_SCALE)) for s in range(PERTURB_TRIALS)]
    rows, margin = [], None
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for order, pt in runs:
            tr = []
            if mode == 0:
                filterL2_(x, eps, sigma, expansion, order=order, trace=tr, perturb=pt)
            else:
                ex_noregret_(x, eps, sigma, expansion, trace=tr, order=order, perturb=pt)
            flags = np.zeros(n, np.int32)
            if mode == 0:
                flags[:] = 1
                flags[tr[0]["removed"]] = 0
            else:
                flags[tr[0]["kept"]] = 1
            rows.append(np.concatenate([trace_array(tr, mode, n)[0], flags]))
            if margin is None:
                margin = np.array(tr[0]["margin"])
    a = rows[0]
    agree = int(a[0])
    for b in rows[1:]:
        diff = np.nonzero(a[1:1 + a[0]] != b[1:1 + a[0]])[0]
        if diff.size:
            agree = min(agree, int(diff[0]))
        elif a[0] != b[0]:
            agree = min(agree, int(min(a[0], b[0])))
    return a, agree, margin


def trace_array(records, mode, n):
    """Pack per-chunk filter traces into the engine's int32 layout
    (sra_filter_trace_f32): row = [iters, decision_0 .. decision_{T-1}, -1 pad]
    with decision = the removed client (filterL2) or the capped count
    (ex_noregret), T = 2 * int(eps * n) resp. int(2 * eps * n_kept) <= n."""
    out = np.full((len(records), 1 + n), -1, dtype=np.int32)
    for i, r in enumerate(records):
        dec = r["removed"] if mode == 0 else r["capped"]
        out[i, 0] = r["iters"]
        out[i, 1:1 + len(dec)] = dec
    return out


# ----------------------------------------------------------------------------
# stateful inline aggregators of simulate.py
# ----------------------------------------------------------------------------
def bucketing_round(layers_by_client, prev, buckets, perround, tau):
    """simulate.py:335-366 after the (first-round) shuffle of ``choices``:
    overlapping windows ``choices[b : b + perround//buckets]``, per-bucket mean,
    cross-layer-norm clipping against ``prev``, then the mean over buckets.
    ``layers_by_client[c][l]`` is client c's layer l, already in choices order."""
    width = perround // buckets
    nlayer = len(prev)
    bucket_avg = []
    for b in range(buckets):
        members = layers_by_client[b:b + width]
        bucket_avg.append([np.array([m[l] for m in members]).mean(axis=0) for l in range(nlayer)])
    for b in range(buckets):
        sq = 0.
        for l in range(nlayer):
            sq += _l2(bucket_avg[b][l] - prev[l]) ** 2
        nrm = np.sqrt(sq)
        for l in range(nlayer):
            bucket_avg[b][l] = (bucket_avg[b][l] - prev[l]) * min(1, tau / nrm)
    return [np.array([bucket_avg[b][l] for b in range(buckets)]).mean(axis=0) for l in range(nlayer)]


def history_round(layers_by_client, prev, tau):
    """simulate.py:367-388: clip every client's update against ``prev`` by the
    cross-layer norm (in place, as the reference mutates local_grads), then the
    mean over clients."""
    nlayer = len(prev)
    for grads in layers_by_client:
        sq = 0.
        for l in range(nlayer):
            sq += _l2(grads[l] - prev[l]) ** 2
        nrm = np.sqrt(sq)
        for l in range(nlayer):
            grads[l] = (grads[l] - prev[l]) * min(1, tau / nrm)
    return [np.array([g[l] for g in layers_by_client]).mean(axis=0) for l in range(nlayer)]


def dispatch_round(agg, local_grads, choices, args, prev):
    """One round of the reference's per-layer dispatch, simulate.py:231-398
    (the 14 ``--agg`` branches of simulate.py:76).  ``local_grads[c][l]`` is
    client c's layer l; ``choices`` the round's client array (shuffled in place
    on the first iclr2022_bucketing round, simulate.py:338-342).  Returns
    ``(average_grad, prev_average_grad)``; icml2021_history mutates
    ``local_grads`` like the reference (simulate.py:380)."""
    nlayer = len(local_grads[int(choices[0])])

    def layer(l):
        return [local_grads[c][l] for c in choices]

    eps = args.malnum * 1. / args.nworker
    if agg == "average":                                            # :235-244
        return [np.average(np.array(layer(l)), axis=0) for l in range(nlayer)], prev
    if agg == "krum":                                               # :245-253
        return [krum(layer(l), f=args.malnum)[0] for l in range(nlayer)], prev
    if agg == "filterl2":                                           # :254-262
        return [filterL2(layer(l), eps=eps, sigma=args.sigma) for l in range(nlayer)], prev
    if agg == "mom_filterl2":                                       # :263-271
        return [mom_filterL2(layer(l), eps=eps, sigma=args.sigma, delta=np.exp(-50 + args.malnum))
                for l in range(nlayer)], prev
    if agg == "median":                                             # :272-280
        return [median(layer(l)) for l in range(nlayer)], prev
    if agg == "trimmedmean":                                        # :281-289
        return [trimmed_mean(layer(l)) for l in range(nlayer)], prev
    if agg in ("bulyankrum", "bulyanmedian", "bulyantrimmedmean"):  # :290-316
        sub = agg[len("bulyan"):]
        return [bulyan(layer(l), args.malnum, aggsubfunc=sub) for l in range(nlayer)], prev
    if agg == "ex_noregret":                                        # :317-325
        return [ex_noregret(layer(l), eps=eps, sigma=args.sigma) for l in range(nlayer)], prev
    if agg == "mom_ex_noregret":                                    # :326-334
        return [mom_ex_noregret(layer(l), eps=eps, sigma=args.sigma, delta=np.exp(-50 + args.malnum))
                for l in range(nlayer)], prev
    if agg == "iclr2022_bucketing":                                 # :335-366
        if prev is None:
            prev = [np.zeros(np.shape(local_grads[int(choices[0])][l])) for l in range(nlayer)]
            for _ in range(nlayer):
                np.random.shuffle(choices)
        out = bucketing_round([local_grads[c] for c in choices], prev, args.buckets, args.perround, args.tau)
        return out, [a.copy() for a in out]
    if agg == "icml2021_history":                                   # :367-388
        if prev is None:
            prev = [np.zeros(np.shape(local_grads[int(choices[0])][l])) for l in range(nlayer)]
        out = history_round([local_grads[c] for c in choices], prev, args.tau)
        return out, [a.copy() for a in out]
    if agg == "clustering":                                         # :389-397
        return [mom_krum(layer(l), f=args.malnum) for l in range(nlayer)], prev
    raise ValueError("unknown aggregator %r" % agg)


def as_float32_rows(samples):
    """Convenience for tests/bench: (N, D) float32 C-contiguous copy."""
    rows, _ = _as_rows(samples)
    return np.ascontiguousarray(rows, dtype=np.float32)


__all__ = [
    "ITV", "MAX_ITER", "average", "median", "trimmed_mean", "krum_", "krum",
    "mom_krum", "bulyan_median", "bulyan_one_coordinate", "bulyan", "filterL2_",
    "filterL2", "mom_filterL2", "ex_noregret_", "ex_noregret", "mom_ex_noregret",
    "pairwise_l2", "krum_scores_from_dist", "bucket_count", "bucket_means",
    "chunk_sizes", "bulyan_coordinates", "bulyan_select", "kl_capped_projection",
    "bucketing_round", "history_round", "dispatch_round",
]
