"""CPU: the oracle's spectral filters make the live reference's decisions.

The trace fixtures (tests/golden/trace_*.npz) hold, per itv-chunk, the
reference's per-iteration decisions recorded by gen_filter_traces.py (the
argmax-tau client removed by filterL2_, robust_estimator.py:166-172; the kept
KL-projection candidate and the Krum pre-filter's kept set of ex_noregret_,
:49-51, :78-99), the prefix of iterations on which three independent fp64
oracle evaluations agree with it, and a per-chunk output bound
(add_trace_bounds.py).  The GPU side is tests/test_gpu_filter_trace.py.
"""
from __future__ import annotations

import warnings

import numpy as np
import pytest

from conftest import trace_fixtures
from oracle import robust_np as orc

TRACES = trace_fixtures()


def _run(rec, order):
    p, func = rec["params"], rec["func"]
    args = (list(rec["x"]), p["eps"], p["sigma"], p["expansion"], p["itv"])
    tr = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if func == "ex_noregret":
            out = orc.ex_noregret(*args, trace=tr, order=order)
        elif func == "mom_filterL2":
            out = orc.mom_filterL2(*args, p["delta"], order=order, trace=tr)
        else:
            out = orc.filterL2(*args, order=order, trace=tr)
    return out, tr


def test_trace_fixtures_present():
    names = {r["name"] for r in TRACES}
    for f in ("filterL2", "ex_noregret", "mom_filterL2"):
        assert {"trace_%s_%s" % (f, s) for s in ("bench", "c5" if f.startswith("mom") else "c4")} <= names
    for r in TRACES:
        assert r["trace"].shape[0] == r["bound"].shape[0] == r["agree"].shape[0]
        assert (r["agree"] <= r["trace"][:, 0]).all()


@pytest.mark.parametrize("rec", TRACES, ids=[r["name"] for r in TRACES])
def test_dual_oracle_trace_and_bound(rec):
    """The client-space oracle (the checker of the full-size device traces)
    makes the reference's decisions on the agreed prefix and lands in bound."""
    out, tr = _run(rec, "dual")
    mode = 1 if rec["func"] == "ex_noregret" else 0
    n = rec["trace"].shape[1] // 2
    got = orc.trace_array(tr, mode, n)
    for c, a in enumerate(rec["agree"]):
        np.testing.assert_array_equal(got[c, 1:1 + a], rec["trace"][c, 1:1 + a])
        if mode == 1:
            kept = np.zeros(n, np.int32)
            kept[tr[c]["kept"]] = 1
            np.testing.assert_array_equal(kept, rec["trace"][c, 1 + n:])
        sl = slice(c * rec["params"]["itv"], (c + 1) * rec["params"]["itv"])
        err = np.abs(out[sl] - rec["out"][sl]).max() / np.abs(rec["out"][sl]).max()
        assert err <= rec["bound"][c]


@pytest.mark.parametrize("name", [pytest.param("trace_filterL2_c4", marks=pytest.mark.slow), "trace_ex_noregret_c4"])
def test_primal_oracle_full_trace(name):
    """The primal (k x k LAPACK) oracle reproduces every decision of the C4
    chunks exactly, iteration count included."""
    rec = next(r for r in TRACES if r["name"] == name)
    _, tr = _run(rec, "gemm")
    mode = 1 if rec["func"] == "ex_noregret" else 0
    n = rec["trace"].shape[1] // 2
    np.testing.assert_array_equal(orc.trace_array(tr, mode, n), rec["trace"][:, :1 + n])
