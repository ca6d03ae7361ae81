"""The sorting-network building blocks of the k-select (csrc/sra_common.hpp),
checked on the CPU with the 0-1 principle (a comparator network sorts every
input iff it sorts every 0-1 input):

* Green's 60-comparator 16-input network (kGreen16) -- exhaustively, 2^16 inputs;
* the odd-even merge of two sorted halves (merge_stages) -- every pair of
  sorted 0-1 halves for 8, 16 and 32 inputs;
* the 3-input "sort4" block (min3 / med3 / max3 + insertion of the fourth
  value, sort4_blocks) -- every real-valued ordering, via all permutations of
  4 distinct values and all 0-1 inputs.
"""
from __future__ import annotations

import itertools
import os
import re

import numpy as np

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "secure-robust-federated-learning_amd", "csrc", "sra_common.hpp")


def green16():
    text = open(HDR).read()
    block = text[text.index("kGreen16[60][2] = {"):]
    block = block[:block.index("};")]
    pairs = [(int(a), int(b)) for a, b in re.findall(r"\{(\d+), (\d+)\}", block)]
    assert len(pairs) == 60
    return pairs


def apply(ces, x):
    x = x.copy()
    for a, b in ces:
        lo = np.minimum(x[:, a], x[:, b])
        hi = np.maximum(x[:, a], x[:, b])
        x[:, a], x[:, b] = lo, hi
    return x


def merge_stages(lo, n):
    """Restates BaseNet::merge_stages (odd-even merge of two sorted halves)."""
    ces = []
    p = n // 2
    k = p
    while k >= 1:
        j = k % p
        while j + k < n:
            for i in range(k):
                if i + j + k >= n:
                    break
                ces.append((lo + i + j, lo + i + j + k))
            j += 2 * k
        k >>= 1
    return ces


def is_sorted(x):
    return bool((np.diff(x.astype(np.int64), axis=1) >= 0).all())


def test_green16_sorts_all_01_inputs():
    ces = green16()
    m = np.arange(1 << 16, dtype=np.uint32)
    x = ((m[:, None] >> np.arange(16)) & 1).astype(np.uint8)
    assert is_sorted(apply(ces, x))


def test_merge_stages_merge_sorted_halves():
    for n in (8, 16, 32):
        h = n // 2
        rows = []
        for z1 in range(h + 1):
            for z2 in range(h + 1):
                a = [0] * z1 + [1] * (h - z1)
                b = [0] * z2 + [1] * (h - z2)
                rows.append(a + b)
        x = np.array(rows, dtype=np.uint8)
        assert is_sorted(apply(merge_stages(0, n), x))


def sort4(a0, a1, a2, d):
    med3 = lambda p, q, r: max(min(p, q), min(max(p, q), r))
    s0, s1, s2 = min(a0, a1, a2), med3(a0, a1, a2), max(a0, a1, a2)
    return [min(s0, d), med3(s0, s1, d), med3(s1, s2, d), max(s2, d)]


def test_sort4_block():
    for perm in itertools.permutations([1.5, -2.0, 7.25, 0.0]):
        assert sort4(*perm) == sorted(perm)
    for bits in itertools.product([0, 1, 2], repeat=4):   # ties included
        assert sort4(*bits) == sorted(bits)


# ---------------------------------------------------------------------------
# the fused three-input programs (csrc/net_fused.inc, tools/fuse_net.py)
# ---------------------------------------------------------------------------
INC = os.path.join(os.path.dirname(HDR), "net_fused.inc")


def fused_programs():
    """Parse the generated header: {name: (kind, dst, a, b, c, out, slots)}."""
    text = open(INC).read()
    progs = {}
    for m in re.finditer(r"struct (\w+) \{(.*?)\n\};", text, flags=re.S):
        body = m.group(2)

        def arr(nm):
            blk = re.search(r"%s\[\d+\] = \{([^}]*)\}" % nm, body).group(1)
            return [int(t) for t in blk.replace("\n", " ").split(",") if t.strip()]
        slots = int(re.search(r"kSlots = (\d+)", body).group(1))
        progs[m.group(1)] = (arr("kKind"), arr("kDst"), arr("kA"), arr("kB"), arr("kC"), arr("kOut"), slots)
    return progs


def run_fused(prog, X):
    kind, dst, A, B, C, out, slots = prog
    v = [None] * slots
    for i in range(X.shape[0]):
        v[i] = X[i]
    for k, d, a, b, c in zip(kind, dst, A, B, C):
        if k == 1:
            r = np.minimum(v[a], v[b])
        elif k == 2:
            r = np.maximum(v[a], v[b])
        elif k == 3:
            r = np.minimum(np.minimum(v[a], v[b]), v[c])
        elif k == 4:
            r = np.maximum(np.maximum(v[a], v[b]), v[c])
        else:
            assert k == 5
            r = np.maximum(np.minimum(v[a], v[b]), np.minimum(np.maximum(v[a], v[b]), v[c]))
        v[d] = r
    return np.array([v[o] for o in out])


def test_fused_programs_sort():
    """Every generated program, as the kernels run it, returns np.sort's kept
    ranks on columns with heavy ties (integers in [-3, 3]) and on Gaussian
    columns, in its input form (sorted 4-blocks + +inf pads, or bitonic)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HDR)), "..", "tools"))
    import fuse_net as fn
    progs = fused_programs()
    assert set(progs) == {p[0] for p in fn.PROGRAMS}
    for name, p2, pr, olo, ohi, net in fn.PROGRAMS:
        for seed in (3, 4):
            X, want = fn.random_inputs(p2, pr, net, 4000, seed)
            got = run_fused(progs[name], X)
            np.testing.assert_array_equal(got, want[olo:ohi], err_msg=name)
        rng = np.random.default_rng(5)
        T = rng.integers(-3, 4, size=(pr, 4000)).astype(np.float64)
        want = np.sort(T, axis=0)
        if net == "from4":
            for b in range(0, pr, 4):
                T[b:b + 4] = np.sort(T[b:b + 4], axis=0)
        else:
            T = np.vstack([np.sort(T[:pr // 2], axis=0), np.sort(T[pr // 2:], axis=0)[::-1]])
        T = np.vstack([T, np.full((p2 - pr, 4000), np.inf)])
        np.testing.assert_array_equal(run_fused(progs[name], T), want[olo:ohi], err_msg=name)


def test_fused_header_is_generated():
    """net_fused.inc is exactly what tools/fuse_net.py emits today."""
    import subprocess
    import sys
    import tempfile
    tool = os.path.join(os.path.dirname(os.path.dirname(HDR)), "..", "tools", "fuse_net.py")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "net_fused.inc")
        subprocess.run([sys.executable, tool, "--emit-all", out], check=True, capture_output=True)
        assert open(out).read() == open(INC).read()
