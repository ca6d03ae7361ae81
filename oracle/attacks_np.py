"""CPU oracle for the attack-side callers of the aggregation path
(src/attack.py).

TEST INFRASTRUCTURE ONLY, like ``robust_np.py``: only ``tests/`` may use it,
as the checker.  Each function restates the reference's behaviour from its
observable semantics and cites the lines it follows; it is pinned against
``tests/golden/attack_*.npz``, which ``tests/golden/gen_attack_fixtures.py``
wrote by calling the live reference functions.

The per-element draws of ``attack_trimmedmean`` come from Python's own
``random`` module here (that IS the reference's generator); the device path
reproduces its Mersenne Twister stream.  ``mt19937_phased`` restates the
three-phase parallel twist that the device kernel uses, so the CPU tests can
check that decomposition against ``random.getrandbits(32)``.
"""
from __future__ import annotations

import random

import numpy as np


def _benign(m, mal_index):
    mal = set(int(i) for i in mal_index)
    return [c for c in range(m) if c not in mal]


def sign_of_benign_sum(rows):
    """np.sign of 0.0 + rows[0] + rows[1] + ... in float64 (attack.py:211-216, :170-173)."""
    acc = np.zeros(np.shape(rows[0]))
    for r in rows:
        acc += r
    return np.sign(acc)


def krum_pick_mixed(samples, f=1):
    """robust_estimator.krum (:234-249) on a list mixing float32 (benign) and
    float64 (malicious) arrays: per client, the norms to every other client
    (float32 BLAS norm for two float32 rows, float64 otherwise) collected in a
    float64 array, the smallest len-f-2 summed with numpy's pairwise sum,
    first argmin."""
    n = len(samples)
    keep = n - f - 2
    scores = []
    for i in range(n):
        dist = np.array([np.linalg.norm(samples[i] - samples[j]) for j in range(n) if j != i])
        scores.append(np.sum(dist[np.argsort(dist)[:keep]]))
    return int(np.argmin(scores))


def attack_krum(local_grads, mal_index, param_index, lower_bound=1e-8):
    """attack.py:202-262: returns (lambda, malicious layer value) and writes the
    malicious rows of layer ``param_index`` in place."""
    m = len(local_grads)
    benign = _benign(m, mal_index)
    s = sign_of_benign_sum([local_grads[c][param_index] for c in benign])
    mal = set(int(i) for i in mal_index)
    lam = 1.0                       # :237-238 (upper_bound is overwritten)
    while True:
        cand = [(-lam * s) if c in mal else local_grads[c][param_index] for c in range(m)]
        pick = krum_pick_mixed(cand, 1)
        if pick in mal or lam < lower_bound:
            break
        lam /= 2.0
    for kk in mal_index:
        local_grads[kk][param_index] = -lam * s
    return lam, -lam * s


def bulyan_attack_krum(shapes, local_grads, mal_index, param_index, lower_bound=1e-8, target_layer=0,
                       target_idx=0):
    """attack.py:264-308: attack_vec[idx] (np.zeros of the network's layer
    shapes) gets + 1 once for idx == target_idx when some c in
    range(#benign) equals target_layer (:278-282); lambda runs 1, 1/2, ...
    (upper_bound overwritten at :286) until krum(f=1) picks a malicious row or
    lambda < lower_bound; the malicious rows become -lambda * attack_vec.
    ``shapes`` = the network's parameter shapes.  Returns (lambda, row)."""
    m = len(local_grads)
    nben = len(_benign(m, mal_index))
    vec = np.zeros(shapes[param_index])
    if param_index == target_idx and 0 <= target_layer < nben:
        vec = vec + 1
    mal = set(int(i) for i in mal_index)
    lam = 1.0
    while True:
        cand = [(-lam * vec) if c in mal else local_grads[c][param_index] for c in range(m)]
        pick = krum_pick_mixed(cand, 1)
        if pick in mal or lam < lower_bound:
            break
        lam /= 2.0
    for kk in mal_index:
        local_grads[kk][param_index] = -lam * vec
    return lam, -lam * vec


def attack_trimmedmean(params, local_grads, mal_index, b=2, rng=random):
    """attack.py:157-198 with NumPy >= 2 scalar promotion: the per-element draw
    is a + (b - a) * r in float32 (a, b float32; the Python floats b and r are
    cast to float32).  ``params`` = the network's parameters as float32 arrays.
    Draws from ``rng`` (the ``random`` module by default) in the reference's
    nditer order, one ``random()`` per element."""
    m = len(local_grads)
    benign = _benign(m, mal_index)
    bf = np.float32(b)
    out = []
    for idx, p in enumerate(params):
        p = np.asarray(p, dtype=np.float32)
        sgn = sign_of_benign_sum([local_grads[c][idx] for c in benign]).ravel()
        t = np.stack([(p - local_grads[c][idx]).ravel() for c in benign])
        bmax, bmin = np.amax(t, axis=0), np.amin(t, axis=0)
        r = np.array([rng.random() for _ in range(p.size)], dtype=np.float64).astype(np.float32)
        neg = sgn < 0
        a = np.where(neg, np.where(bmin > 0, bmin / bf, bmin * bf), bmax).astype(np.float32)
        hi = np.where(neg, bmin, np.where(bmax > 0, bmax * bf, bmax / bf)).astype(np.float32)
        v = (a + (hi - a) * r).astype(np.float32)
        out.append((-v.astype(np.float64) + p.ravel().astype(np.float64)).reshape(p.shape))
    for c in mal_index:
        for idx in range(len(params)):
            local_grads[c][idx] = out[idx].copy()
    return out


def attack_xie(local_grads, weight, choices, mal_index):
    """attack.py:362-372."""
    mal = set(int(i) for i in mal_index)
    vec = []
    for i, pp in enumerate(local_grads[0]):
        tmp = np.zeros_like(pp)
        for j in choices:
            if int(j) not in mal:
                tmp += local_grads[j][i]
        vec.append((-weight) * tmp / len(choices))
    for i in mal_index:
        local_grads[i] = vec
    return vec


# ---------------------------------------------------------------------------
# the device kernel's MT19937 decomposition, restated for CPU checking
# ---------------------------------------------------------------------------
_N, _M = 624, 397
_H = _N - _M


def _temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def _mix(cur, nxt, far):
    y = (cur & np.uint32(0x80000000)) | (nxt & np.uint32(0x7FFFFFFF))
    return far ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908B0DF), np.uint32(0))


def mt19937_phased(state, nwords):
    """Words and advanced state, twisting in the kernel's three phases
    ([0,227) from old words; [227,454) and [454,624) from the previous phase's
    new words), each phase reading all operands before writing."""
    mt = np.array(state[:_N], dtype=np.uint32)
    pos = int(state[_N])
    out = []
    take = min(_N - pos, nwords) if pos < _N else 0
    out.append(_temper(mt[pos:pos + take]))
    done, pos = take, pos + take
    while done < nwords:
        for ph in range(3):
            kk = np.arange(ph * _H, min(ph * _H + _H, _N))
            nxt = np.where(kk + 1 < _N, kk + 1, 0)
            far = kk + _M if ph == 0 else kk - _H
            mt[kk] = _mix(mt[kk], mt[nxt], mt[far])
        take = min(nwords - done, _N)
        out.append(_temper(mt[:take]))
        done += take
        pos = take
    words = np.concatenate(out) if out else np.zeros(0, np.uint32)
    return words, tuple(int(v) for v in mt) + (pos,)
