"""Record the LIVE reference's per-iteration filter decisions (build container only).

filterL2_ (robust_estimator.py:144-177) removes the argmax-tau client every
iteration and exits early on lambda^2 <= expansion * sigma^2; ex_noregret_
(:42-102) keeps the Krum pre-filter's clients (:49-51) and, every iteration,
keeps the capped-simplex candidate with the smallest KL (:78-99).  The C4/C5
fixtures of gen_fixtures.py store only final outputs; this script re-runs the
reference on the same inputs (and on bench-shaped chunks: i.i.d. 0.01 N(0,1)
fp32, as bench.py's synthetic data) and records, per chunk:

  filterL2 / mom_filterL2: the ORIGINAL index of the client (bucket) removed at
      each iteration, the iteration count (< T on an early exit) and
      (tau_max - tau_2nd) / tau_max per iteration (how close to a tie);
  ex_noregret: the pre-filter's kept set, the capped count of the chosen
      projection candidate per iteration and its relative KL margin.

How the decisions are observed (no reference code is copied): ``np.argmax``,
``np.argpartition``, ``eigh`` and ``rel_entr`` are looked up in the
reference module's globals at call time, so the module attributes are replaced
by recording wrappers for the duration of one call (``np`` by a proxy module
that forwards every other attribute to numpy).  The eigh shim of
gen_fixtures.load_reference stays underneath.

Writes tests/golden/trace_*.npz: x (inputs), out (reference output), trace
(int32 [chunks, 1 + 2n]: iters, decisions (-1 padded to n), kept flags
(ex_noregret) / ones), margin (float64 [chunks, n], nan padded), params.
Usage: python tests/golden/gen_filter_traces.py [name-substring ...]
"""
from __future__ import annotations

import json
import os
import sys
import types
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_fixtures import load_reference  # noqa: E402

PC = {"eps": 0.2, "sigma": 1e-5, "expansion": 20, "itv": 1000}


class _Recorder:
    def __init__(self, ref):
        self.ref = ref
        self.chunks = []

    def install(self):
        ref, rec = self.ref, self
        real_np, real_eigh, real_rel = ref.np, ref.eigh, ref.rel_entr
        proxy = types.ModuleType("np_proxy")

        def argmax(a, *args, **kw):
            r = real_np.argmax(a, *args, **kw)
            cur = rec.chunks[-1]
            t = real_np.sort(real_np.asarray(a, dtype=np.float64))
            cur["argmax"].append((int(r), float((t[-1] - t[-2]) / t[-1]) if t.size > 1 else 1.0))
            return r

        def argpartition(a, kth, *args, **kw):
            r = real_np.argpartition(a, kth, *args, **kw)
            rec.chunks[-1]["argpartition"].append((np.array(r), kth))
            return r

        def eigh(a, *args, **kw):
            rec.chunks[-1]["eigh"] += 1
            rec.chunks[-1]["cands"].append([])
            return real_eigh(a, *args, **kw)

        def rel_entr(c, c_):
            r = real_rel(c, c_)
            c_ = np.asarray(c_)
            cap = 1.0 / (1 - rec.eps) / len(c_)
            rec.chunks[-1]["cands"][-1].append((float(np.sum(r)), int(np.sum(c_ == cap))))
            return r

        proxy.__getattr__ = lambda name: getattr(real_np, name)
        proxy.argmax = argmax
        proxy.argpartition = argpartition
        ref.np, ref.eigh, ref.rel_entr = proxy, eigh, rel_entr
        self._restore = (real_np, real_eigh, real_rel)

        inner = {"filterL2_": ref.filterL2_, "ex_noregret_": ref.ex_noregret_}

        def wrap(fn):
            def w(samples, eps, *args, **kw):
                rec.eps = eps
                rec.chunks.append({"n": len(samples), "argmax": [], "argpartition": [], "eigh": 0, "cands": []})
                return fn(samples, eps, *args, **kw)
            return w
        ref.filterL2_ = wrap(inner["filterL2_"])
        ref.ex_noregret_ = wrap(inner["ex_noregret_"])
        self._inner = inner

    def uninstall(self):
        self.ref.np, self.ref.eigh, self.ref.rel_entr = self._restore
        self.ref.filterL2_ = self._inner["filterL2_"]
        self.ref.ex_noregret_ = self._inner["ex_noregret_"]


def pack(chunks, mode, n):
    trace = np.full((len(chunks), 1 + 2 * n), -1, dtype=np.int32)
    margin = np.full((len(chunks), n), np.nan)
    for i, ch in enumerate(chunks):
        if mode == 0:
            alive = list(range(ch["n"]))
            dec = [alive.pop(j) for j, _ in ch["argmax"]]
            mar = [m for _, m in ch["argmax"]]
            flags = np.ones(n, np.int32)
            flags[dec] = 0
            flags[ch["n"]:] = 0
        else:
            # the pre-filter's argpartition(metric, -f)[:-f] keeps all but the f last
            (order, kth), = ch["argpartition"]
            kept = np.sort(order[:kth])
            flags = np.zeros(n, np.int32)
            flags[kept] = 1
            dec, mar = [], []
            for cands in ch["cands"]:
                if not cands:        # the early-exit iteration: eigh ran, no projection
                    continue
                kls = [k for k, _ in cands]
                b = int(np.argmin(kls))   # first minimum, as the reference's strict '<'
                dec.append(cands[b][1])
                s = np.sort(kls)
                mar.append(float((s[1] - s[0]) / max(abs(s[0]), 1e-300)) if len(s) > 1 else 1.0)
        trace[i, 0] = len(dec)
        trace[i, 1:1 + len(dec)] = dec
        trace[i, 1 + n:1 + 2 * n] = flags
        margin[i, :len(mar)] = mar
    return trace, margin


def bench_rows(n, d, seed):
    return (0.01 * np.random.default_rng(seed).standard_normal((n, d))).astype(np.float32)


def main():
    only = sys.argv[1:]
    ref = load_reference()
    c4 = np.load(os.path.join(HERE, "filterL2_n128_c4.npz"))["x"].reshape(128, -1)
    c5 = np.load(os.path.join(HERE, "mom_filterL2_n512_c5.npz"))["x"].reshape(512, -1)
    pc5 = dict(PC, delta=float(np.exp(-26)))
    cases = [
        ("trace_filterL2_c4", "filterL2", 0, PC, c4),
        ("trace_filterL2_bench", "filterL2", 0, PC, bench_rows(128, 4000, 91)),
        ("trace_ex_noregret_c4", "ex_noregret", 1, PC, c4),
        ("trace_ex_noregret_bench", "ex_noregret", 1, PC, bench_rows(128, 3000, 92)),
        ("trace_mom_filterL2_c5", "mom_filterL2", 0, pc5, c5),
        ("trace_mom_filterL2_bench", "mom_filterL2", 0, pc5, bench_rows(512, 2000, 93)),
    ]
    for name, func, mode, p, x in cases:
        if only and not any(o in name for o in only):
            continue
        rec = _Recorder(ref)
        rec.install()
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                args = [list(x), p["eps"], p["sigma"], p["expansion"], p["itv"]]
                if func == "mom_filterL2":
                    out = ref.mom_filterL2(*args, p["delta"])
                else:
                    out = getattr(ref, func)(*args)
        finally:
            rec.uninstall()
        n = rec.chunks[0]["n"]
        trace, margin = pack(rec.chunks, mode, n)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, func=np.array(func), params=np.array(json.dumps(p)), x=x, out=np.asarray(out),
                            trace=trace, margin=margin)
        print("wrote %s: %d chunks, iters %s, min margin %.2e" % (
            name, len(rec.chunks), trace[:, 0].tolist(), np.nanmin(margin)), flush=True)


if __name__ == "__main__":
    main()
