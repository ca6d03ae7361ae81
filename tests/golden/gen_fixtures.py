"""Generate the golden fixtures in tests/golden/*.npz from the LIVE reference.

Runs only in the build container, where the reference is mounted read-only at
/root/reference.  It imports ``src/robust_estimator.py`` with the two shims
recorded in SURVEY.md §8(c):

  1. ``cvxpy`` is imported at robust_estimator.py:32 but never used and is not
     installed here -> an empty module is placed in sys.modules;
  2. scipy 1.15 removed ``eigh(eigvals=...)`` (the reference pins scipy 1.4.1,
     requirements.txt:3) -> ``robust_estimator.eigh`` is wrapped to map
     ``eigvals=(lo, hi)`` onto ``subset_by_index=[lo, hi]``.

Only data (inputs, outputs, indices) is written; no reference source or
bytecode is copied.  Usage:  python tests/golden/gen_fixtures.py
"""
from __future__ import annotations

import json
import os
import sys
import time
import types
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
sys.path.insert(0, HERE)
from synth import make_clients, make_convnet_round, CONVNET_MNIST_SHAPES  # noqa: E402


def load_reference():
    if not os.path.isdir(REF_SRC):
        raise SystemExit("gen_fixtures.py needs the reference at %s; it is never run on the GPU box" % REF_SRC)
    sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))
    sys.path.insert(0, REF_SRC)
    import robust_estimator as ref  # noqa: E402
    from scipy.linalg import eigh as _eigh

    def eigh_compat(a, *args, eigvals=None, **kw):
        if eigvals is not None:
            kw["subset_by_index"] = list(eigvals)
        return _eigh(a, *args, **kw)

    ref.eigh = eigh_compat
    return ref


def save(name, func, params, x, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez(path, func=np.array(func), params=np.array(json.dumps(params)),
             x=np.asarray(x), **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote %-40s %8.1f KB" % (name, os.path.getsize(path) / 1024.0))


def run_case(ref, name, func, params, clients, call):
    t = time.time()
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            res = call()
    except Exception as e:  # record the reference's failure class
        save(name, func, params, np.array(clients), error=np.array(type(e).__name__))
        return
    extra = {}
    if isinstance(res, tuple):
        out, idx = res
        extra["index"] = np.array(idx)
        res = out
    if isinstance(res, list):
        res = np.array(res)
    save(name, func, params, np.array(clients), out=res, **extra)
    _ = t


def _none_exit_sigma(ref, xs, eps, expansion, itv):
    """A sigma at which ex_noregret's projection is infeasible at iteration 0
    (projected_c is None) and the next iteration -- weights=None, i.e. the
    unweighted mean -- takes the early exit (robust_estimator.py:65-72, 99),
    so the reference returns np.average(samples, weights=None).  Iteration 0
    (weights = ones) evaluates the same statistics up to rounding, so the window
    is the rounding gap between the two top eigenvalues: found by bisection on
    the reference's own outcome; None if that gap has the wrong sign."""
    def outcome(sigma):
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                out = ref.ex_noregret(xs, eps, sigma, expansion, itv)
        except TypeError:
            return "typeerror", None
        return "value", out
    lo, hi = 1e-12, 10.0            # lo: TypeError, hi: exit at iteration 0
    if outcome(lo)[0] != "typeerror" or outcome(hi)[0] != "value":
        return None
    for _ in range(200):
        mid = np.sqrt(lo * hi) if hi / lo > 1.0 + 1e-9 else 0.5 * (lo + hi)
        if mid in (lo, hi):
            break
        if outcome(mid)[0] == "typeerror":
            lo = mid
        else:
            hi = mid
    # hi is the smallest sigma (to the bisection's resolution) that returns; it
    # exits at iteration 1 iff the result is the fp32 (unweighted) mean
    # (a weighted fp64 average is practically never fp32-exact on every coordinate)
    res = outcome(hi)[1]
    if res is None or not np.all(np.asarray(res, np.float64) == np.asarray(res, np.float32)):
        return None
    return hi


def degenerate_cases(ref):
    """Round 4: the reference's behaviour on degenerate inputs.
      * krum with NaN / inf clients: the NaN distances sort last (argsort), a
        NaN score is np.argmin's answer (the FIRST NaN), inf - inf = NaN;
      * bulyan(..., 'median') with a NaN client: every distance to the NaN
        median is NaN, no strict minimum -> AssertionError (:308);
        trimmedmean / krum modes with the same client;
      * ex_noregret with an infeasible capped-simplex projection (cap
        1/((1-eps) n') >= 1 -> break at i = 0, projected_c = None, :78-99):
        TypeError at the next multiplicative update (:75), or -- when the next
        iteration (weights=None) exits early -- the unweighted mean (:71-72)."""
    out = []
    xs = make_clients(12, (30,), 90)
    xs[5][7] = np.nan
    out.append(("krum_nan_client_n12_f2", "krum", {"f": 2}, xs, (lambda xs=xs: ref.krum(xs, 2))))
    out.append(("krum__nan_client_n12_f2", "krum_", {"f": 2}, xs, (lambda xs=xs: ref.krum_(xs, 2))))
    xs = make_clients(12, (30,), 91)
    xs[8][1] = np.nan
    xs[3][20] = np.nan
    out.append(("krum_nan_two_n12_f2", "krum", {"f": 2}, xs, (lambda xs=xs: ref.krum(xs, 2))))
    xs = make_clients(12, (30,), 92)
    xs[2][3] = np.inf
    xs[9][3] = np.inf           # inf - inf = NaN: d(2, 9) is NaN, d(2 or 9, others) inf
    xs[4][10] = -np.inf
    out.append(("krum_inf_clients_n12_f2", "krum", {"f": 2}, xs, (lambda xs=xs: ref.krum(xs, 2))))
    out.append(("krum__inf_clients_n12_f2", "krum_", {"f": 2}, xs, (lambda xs=xs: ref.krum_(xs, 2))))
    xs = make_clients(128, (300,), 93, byz=20)
    xs[77][150] = np.nan
    out.append(("krum_nan_client_n128_f20", "krum", {"f": 20}, xs, (lambda xs=xs: ref.krum(xs, 20))))
    xs = make_clients(300, (64,), 94, byz=30)
    xs[211][5] = np.nan
    out.append(("krum_nan_client_n300_f30", "krum", {"f": 30}, xs, (lambda xs=xs: ref.krum(xs, 30))))
    xs = make_clients(30, (40,), 95, byz=3)
    xs[10][4] = np.nan
    out.append(("mom_krum_nan_client_n30_f3", "mom_krum", {"f": 3}, xs, (lambda xs=xs: ref.mom_krum(xs, 3))))
    xs = make_clients(24, (40,), 96, byz=5)
    xs[7][13] = np.nan
    for mode in ("median", "trimmedmean", "krum"):
        out.append(("bulyan_%s_nan_client_n24_f5" % mode, "bulyan", {"f": 5, "aggsubfunc": mode}, xs,
                    (lambda xs=xs, mode=mode: ref.bulyan(xs, 5, aggsubfunc=mode))))
    xs = make_clients(24, (40,), 97, byz=5)
    xs[11][2] = np.inf
    out.append(("bulyan_median_inf_client_n24_f5", "bulyan", {"f": 5, "aggsubfunc": "median"}, xs,
                (lambda xs=xs: ref.bulyan(xs, 5, aggsubfunc="median"))))
    # ex_noregret, eps = 0.5, n = 4: f = 2, n' = 2, T = int(2 eps n') = 2,
    # cap = 1/((1 - 0.5) 2) = 1 -> clip_norm = 0 -> projected_c = None at iteration 0
    pn = {"eps": 0.5, "sigma": 1e-5, "expansion": 20, "itv": 20}
    xs = make_clients(4, (20,), 98)
    out.append(("ex_noregret_none_typeerror", "ex_noregret", pn, xs,
                (lambda xs=xs, p=pn: ref.ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]))))
    for seed in range(99, 160):
        xs = make_clients(4, (20,), seed)
        sig = _none_exit_sigma(ref, xs, 0.5, 20, 20)
        if sig is not None:
            pe = {"eps": 0.5, "sigma": float(sig), "expansion": 20, "itv": 20}
            out.append(("ex_noregret_none_exit", "ex_noregret", pe, xs,
                        (lambda xs=xs, p=pe: ref.ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]))))
            break
    return out


def main():
    ref = load_reference()
    cases = []

    # ---- coordinate-wise: median / trimmed_mean / average ----------------
    cw_shapes = [(1, (7,), 1), (2, (5,), 2), (3, (4, 3), 3), (12, (50,), 4), (100, (30, 30), 5),
                 (128, (600,), 6), (129, (100,), 7), (512, (64,), 8), (128, (1,), 9), (16, (33,), 10)]
    for n, shp, seed in cw_shapes:
        xs = make_clients(n, shp, seed)
        cases.append(("median_n%d_%s" % (n, "x".join(map(str, shp))), "median", {}, xs,
                      (lambda xs=xs: ref.median(xs))))
        cases.append(("trimmed_mean_n%d_%s" % (n, "x".join(map(str, shp))), "trimmed_mean", {"beta": 0.1}, xs,
                      (lambda xs=xs: ref.trimmed_mean(xs))))
    for beta in (0.0, 0.2, 0.45):
        xs = make_clients(40, (77,), 11)
        cases.append(("trimmed_mean_beta%g" % beta, "trimmed_mean", {"beta": beta}, xs,
                      (lambda xs=xs, beta=beta: ref.trimmed_mean(xs, beta))))
    # NaN / inf / ties
    xs = make_clients(20, (40,), 12)
    xs[3][5] = np.nan
    xs[7][9] = np.nan
    xs[8][9] = np.nan
    xs[1][10] = np.nan
    xs[2][10] = np.nan
    xs[4][10] = np.nan   # 3 NaNs at coord 10 > b=2 -> NaN; 2 at coord 9 trimmed
    xs[5][11] = np.inf
    xs[6][12] = -np.inf
    xs[9][13] = np.inf
    xs[10][13] = -np.inf
    cases.append(("median_nan_inf", "median", {}, xs, (lambda xs=xs: ref.median(xs))))
    cases.append(("trimmed_mean_nan_inf", "trimmed_mean", {"beta": 0.1}, xs, (lambda xs=xs: ref.trimmed_mean(xs))))
    rng = np.random.default_rng(13)
    ties = [rng.integers(-3, 4, size=(25,)).astype(np.float32) for _ in range(31)]
    cases.append(("median_ties", "median", {}, ties, (lambda xs=ties: ref.median(xs))))
    cases.append(("trimmed_mean_ties", "trimmed_mean", {"beta": 0.1}, ties, (lambda xs=ties: ref.trimmed_mean(xs))))

    # ---- Krum / MoM-Krum ---------------------------------------------------
    for n, f, shp, seed, kw in [(5, 1, (6,), 20, {}), (12, 2, (3, 7), 21, {}), (30, 5, (64,), 22, {"byz": 5}),
                                (10, 9, (8,), 23, {}), (10, 8, (8,), 24, {}),
                                (64, 10, (200,), 25, {"byz": 10, "identical_byz": True}),
                                (128, 20, (300,), 26, {"byz": 20})]:
        xs = make_clients(n, shp, seed, **kw)
        cases.append(("krum_n%d_f%d" % (n, f), "krum", {"f": f}, xs, (lambda xs=xs, f=f: ref.krum(xs, f))))
        cases.append(("krum__n%d_f%d" % (n, f), "krum_", {"f": f}, xs, (lambda xs=xs, f=f: ref.krum_(xs, f))))
    for n, f, seed in [(30, 3, 30), (100, 20, 31), (128, 20, 32)]:
        xs = make_clients(n, (120,), seed, byz=f)
        cases.append(("mom_krum_n%d_f%d" % (n, f), "mom_krum", {"f": f}, xs, (lambda xs=xs, f=f: ref.mom_krum(xs, f))))

    # ---- Bulyan --------------------------------------------------------------
    for n, f, shp, seed, kw in [(24, 5, (40,), 40, {}), (30, 5, (12, 10), 41, {"byz": 5}),
                                (45, 10, (90,), 42, {"byz": 10}), (40, 9, (70,), 43, {"byz": 9, "identical_byz": True}),
                                (100, 20, (300,), 44, {"byz": 20})]:
        xs = make_clients(n, shp, seed, **kw)
        for mode in ("krum", "median", "trimmedmean"):
            cases.append(("bulyan_%s_n%d_f%d" % (mode, n, f), "bulyan", {"f": f, "aggsubfunc": mode}, xs,
                          (lambda xs=xs, f=f, mode=mode: ref.bulyan(xs, f, aggsubfunc=mode))))
    # 2f < N < 4f: beta = theta - 2f < 0, so argsort(...)[:beta] drops -beta values
    # from the far end (Python slice semantics); keep 0 is the mean of an empty slice
    for n, f, shp, seed in [(30, 8, (60,), 46), (40, 12, (55,), 47), (30, 10, (20,), 48)]:
        xs = make_clients(n, shp, seed, byz=f)
        for mode in ("krum", "median", "trimmedmean"):
            cases.append(("bulyan_%s_n%d_f%d_negbeta" % (mode, n, f), "bulyan", {"f": f, "aggsubfunc": mode}, xs,
                          (lambda xs=xs, f=f, mode=mode: ref.bulyan(xs, f, aggsubfunc=mode))))
    xs = make_clients(10, (5,), 45)
    cases.append(("bulyan_theta0", "bulyan", {"f": 5, "aggsubfunc": "trimmedmean"}, xs,
                  (lambda xs=xs: ref.bulyan(xs, 5, aggsubfunc="trimmedmean"))))

    # ---- spectral filters ----------------------------------------------------
    for tag, n, shp, seed, kw, params in [
        ("exit", 30, (40,), 50, {"byz": 5}, {"eps": 0.2, "sigma": 0.02, "expansion": 20, "itv": 20}),
        ("noexit", 30, (40,), 51, {"byz": 5}, {"eps": 0.2, "sigma": 1e-5, "expansion": 20, "itv": 20}),
        ("sqrt_itv", 40, (7, 9), 52, {"byz": 8}, {"eps": 0.2, "sigma": 0.02, "expansion": 20, "itv": None}),
        ("ragged", 24, (53,), 53, {"byz": 4}, {"eps": 0.2, "sigma": 0.02, "expansion": 20, "itv": 16}),
    ]:
        xs = make_clients(n, shp, seed, **kw)
        cases.append(("filterL2_%s" % tag, "filterL2", params, xs,
                      (lambda xs=xs, p=params: ref.filterL2(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]))))
        cases.append(("ex_noregret_%s" % tag, "ex_noregret", params, xs,
                      (lambda xs=xs, p=params: ref.ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]))))
    for tag, n, seed, params in [
        ("ok", 40, 60, {"eps": 0.2, "sigma": 0.02, "expansion": 20, "itv": 25, "delta": float(np.exp(-2))}),
        ("empty_bucket", 128, 61, {"eps": 0.2, "sigma": 1e-5, "expansion": 20, "itv": 25, "delta": float(np.exp(-30))}),
    ]:
        xs = make_clients(n, (50,), seed, byz=int(0.2 * n))
        cases.append(("mom_filterL2_%s" % tag, "mom_filterL2", params, xs,
                      (lambda xs=xs, p=params: ref.mom_filterL2(xs, p["eps"], p["sigma"], p["expansion"], p["itv"], p["delta"]))))
        cases.append(("mom_ex_noregret_%s" % tag, "mom_ex_noregret", params, xs,
                      (lambda xs=xs, p=params: ref.mom_ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"], p["delta"]))))

    only = sys.argv[1:]   # optional name filters: regenerate only matching fixtures
    # ex_noregret with ceil(eps*n) = 0: argpartition(..., -0)[:-0] keeps nothing -> ValueError
    xs = make_clients(20, (30,), 54, byz=3)
    p0 = {"eps": 0.0, "sigma": 0.02, "expansion": 20, "itv": 15}
    cases.append(("ex_noregret_f0", "ex_noregret", p0, xs,
                  (lambda xs=xs, p=p0: ref.ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]))))

    # ---- BASELINE configs at their client counts (a few chunks / columns of d) ----
    # C3 bulyan N=128 f=20 (theta 88, beta 48); C4 filterl2 / ex_noregret N=128 with
    # simulate.py's eps = malnum/nworker = 0.2, sigma 1e-5, itv 1000; C5 mom_filterL2
    # N=512 with delta = e^-26 (128 buckets of 4)
    xs = make_clients(128, (1500,), 80, byz=20)
    for mode in ("median", "trimmedmean", "krum"):
        cases.append(("bulyan_%s_n128_f20_c3" % mode, "bulyan", {"f": 20, "aggsubfunc": mode}, xs,
                      (lambda xs=xs, mode=mode: ref.bulyan(xs, 20, aggsubfunc=mode))))
    pc4 = {"eps": 0.2, "sigma": 1e-5, "expansion": 20, "itv": 1000}
    xs = make_clients(128, (1300,), 81, byz=20)
    cases.append(("filterL2_n128_c4", "filterL2", pc4, xs,
                  (lambda xs=xs, p=pc4: ref.filterL2(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]))))
    cases.append(("ex_noregret_n128_c4", "ex_noregret", pc4, xs,
                  (lambda xs=xs, p=pc4: ref.ex_noregret(xs, p["eps"], p["sigma"], p["expansion"], p["itv"]))))
    pc5 = dict(pc4, delta=float(np.exp(-26)))
    xs = make_clients(512, (1200,), 82, byz=100)
    cases.append(("mom_filterL2_n512_c5", "mom_filterL2", pc5, xs,
                  (lambda xs=xs, p=pc5: ref.mom_filterL2(xs, p["eps"], p["sigma"], p["expansion"], p["itv"],
                                                         p["delta"]))))

    cases += degenerate_cases(ref)

    for name, func, params, xs, call in cases:
        if only and not any(o in name for o in only):
            continue
        run_case(ref, name, func, params, xs, call)
    # ---- the scalar Bulyan helpers (robust_estimator.py:259-275) -------------
    if not only or any(o in "bulyan_coord" for o in only):
        rng = np.random.default_rng(49)
        arrs, betas = [], []
        for theta, kind in [(1, "n"), (2, "n"), (7, "n"), (10, "n"), (60, "n"), (88, "n"), (100, "n"), (13, "int"),
                            (40, "int"), (20, "nan"), (24, "nan0"), (16, "inf"), (130, "n"), (200, "int")]:
            a = rng.standard_normal(theta).astype(np.float32).astype(np.float64)
            if kind == "int":
                a = rng.integers(-3, 4, size=theta).astype(np.float64)
            elif kind == "nan":
                a[5] = np.nan
            elif kind == "nan0":
                a[0] = np.nan
            elif kind == "inf":
                a[3] = np.inf
            for beta in sorted({theta - 40, theta // 2, -3, 0, theta, theta + 5, 1}):
                arrs.append(a)
                betas.append(beta)
        mi, rows, one = [], [], []
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for a, beta in zip(arrs, betas):
                m, row = ref.bulyan_median(a)
                mi.append(int(m))
                rows.append(np.asarray(row, dtype=np.float64))
                one.append(float(ref.bulyan_one_coordinate(a, beta)))
        flat = np.concatenate(arrs)
        lens = np.array([len(a) for a in arrs])
        np.savez(os.path.join(HERE, "bulyan_coord.npz"), values=flat, lens=lens, betas=np.array(betas),
                 median_index=np.array(mi), rows=np.concatenate(rows), one=np.array(one))
        print("wrote bulyan_coord (%d cases)" % len(arrs))
    if only:
        return

    # ---- C1 plumbing: one round of the ConvNet layers at N=100 ------------
    seed = 70
    layers = make_convnet_round(100, seed)
    outs = {}
    for agg, fn in (("median", ref.median), ("trimmedmean", ref.trimmed_mean)):
        outs[agg] = np.concatenate([fn(lay).ravel() for lay in layers]).astype(np.float32)
    kr = [ref.krum(lay, 20)[1] for lay in layers]
    np.savez(os.path.join(HERE, "c1_convnet_n100.npz"), seed=np.array(seed), n=np.array(100),
             shapes=np.array(json.dumps(CONVNET_MNIST_SHAPES)), median=outs["median"],
             trimmedmean=outs["trimmedmean"], krum_index=np.array(kr),
             x_checksum=np.array([float(np.sum(np.stack(l).astype(np.float64))) for l in layers]))
    print("wrote c1_convnet_n100")


if __name__ == "__main__":
    main()
