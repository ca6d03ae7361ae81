"""Shared definition of the dispatch fixtures (gen_dispatch_fixtures.py writes
them from the live reference; tests/test_dispatch*.py replay them).

Two configurations of the simulate.py dispatch:
  A  the simulate.py defaults (nworker = perround = 100, malnum = 20,
     buckets = 10, tau = 10, sigma = 1e-5), small ConvNet-like layers;
  B  a sub-sampled round (nworker = 50, perround = 40, malnum = 5) with a
     small tau so that the clipping of the two stateful aggregators is
     active, and MoM bucket counts that leave empty buckets (the reference
     raises ValueError).
Every aggregator runs ``rounds`` consecutive rounds from the same initial
state, so the stateful ``prev_average_grad`` of iclr2022_bucketing /
icml2021_history and the momentum form of their local updates carry over.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# simulate.py:76 — the 14 --agg names, in that order
AGGS = ["average", "ex_noregret", "filterl2", "krum", "median", "trimmedmean", "bulyankrum",
        "bulyantrimmedmean", "bulyanmedian", "mom_filterl2", "mom_ex_noregret", "iclr2022_bucketing",
        "icml2021_history", "clustering"]
# simulate.py:192-194: these two aggregators see momentum-form local updates
MOMENTUM_AGGS = ("iclr2022_bucketing", "icml2021_history")

CONFIGS = [
    {"name": "A", "nworker": 100, "perround": 100, "malnum": 20, "sigma": 1e-5, "buckets": 10, "tau": 10.0,
     "beta": 0.9, "rounds": 2, "np_seed": 5, "data_seed": 700,
     "shapes": [[3, 1, 5, 5], [3], [8, 24], [8], [4, 8], [4]]},
    {"name": "B", "nworker": 50, "perround": 40, "malnum": 5, "sigma": 1e-5, "buckets": 7, "tau": 0.02,
     "beta": 0.9, "rounds": 3, "np_seed": 6, "data_seed": 800,
     "shapes": [[2, 1, 4, 4], [2], [6, 20], [6], [3, 6], [3]]},
]


def layer_shapes(cfg):
    return [tuple(s) for s in cfg["shapes"]]


def total_size(cfg):
    return int(sum(int(np.prod(s)) for s in cfg["shapes"]))


def round_inputs(cfg, r):
    """(nworker, D) float32 local updates of round r: benign N(0, 0.01) plus a
    shared drift, clients 0..malnum-1 Byzantine at -10x the benign mean (the
    reference's mal_index = range(malnum), simulate.py:81)."""
    from synth import make_rows
    return make_rows(cfg["nworker"], total_size(cfg), cfg["data_seed"] + r, byz=cfg["malnum"])


def initial_params(cfg):
    rng = np.random.default_rng(cfg["data_seed"] + 99)
    return (0.1 * rng.standard_normal(total_size(cfg))).astype(np.float32)


def fixture_path(cfg):
    return os.path.join(HERE, "dispatch_%s.npz" % cfg["name"])


def load_fixture(cfg):
    return np.load(fixture_path(cfg), allow_pickle=False)


def round_args(cfg, agg):
    import types
    return types.SimpleNamespace(agg=agg, malnum=cfg["malnum"], nworker=cfg["nworker"], perround=cfg["perround"],
                                 sigma=cfg["sigma"], buckets=cfg["buckets"], tau=cfg["tau"], beta=cfg["beta"])


def _flat(arrs):
    out = []
    for a in arrs:
        if hasattr(a, "detach"):
            a = a.detach().cpu().numpy()
        out.append(np.asarray(a, dtype=np.float64).ravel())
    return np.concatenate(out)


def replay(cfg, agg, fx, round_fn, device=None):
    """Replay the fixture's rounds for ``agg`` through ``round_fn(agg,
    local_grads, choices, args, params)`` (which aggregates AND applies the
    update to ``params``, returning ``average_grad``), with the same caller
    steps gen_dispatch_fixtures.py ran around the reference block.  Yields one
    dict per round: out / params / choices / grads (flat float64), or
    {"error": class name}.  ``device``: keep local_grads and params as torch
    tensors there (device-resident calling convention)."""
    import torch
    shapes = layer_shapes(cfg)
    sizes = [int(np.prod(s)) for s in shapes]
    np.random.seed(cfg["np_seed"])
    local_grads = [[np.zeros(s) for s in shapes] for _ in range(cfg["nworker"])]
    if device is not None:
        local_grads = [[torch.from_numpy(g).to(device) for g in row] for row in local_grads]
    flat0 = fx["params0"]
    params, off = [], 0
    for s, n in zip(shapes, sizes):
        t = torch.from_numpy(flat0[off:off + n].reshape(s).copy())
        params.append(torch.nn.Parameter(t.to(device) if device is not None else t))
        off += n
    args = round_args(cfg, agg)
    for r in range(cfg["rounds"]):
        x = fx["x_r%d" % r]
        choices = np.random.choice(cfg["nworker"], cfg["perround"], replace=False)
        for c in choices:
            off = 0
            for li, (s, n) in enumerate(zip(shapes, sizes)):
                upd = x[c, off:off + n].reshape(s)
                if device is not None:
                    upd = torch.from_numpy(upd.copy()).to(device)
                if agg in MOMENTUM_AGGS:
                    local_grads[c][li] = (1 - args.beta) * upd + args.beta * local_grads[c][li]
                else:
                    local_grads[c][li] = upd.copy() if device is None else upd
                off += n
        try:
            avg = round_fn(agg, local_grads, choices, args, params)
        except Exception as e:
            yield {"round": r, "error": type(e).__name__, "exc": e}
            return
        rec = {"round": r, "out": _flat(avg), "params": _flat(params), "choices": np.asarray(choices).copy(),
               "dtypes": [str(a.dtype).replace("torch.", "") for a in avg]}
        if agg in MOMENTUM_AGGS:
            rec["grads"] = np.stack([_flat(local_grads[c]) for c in choices])
        yield rec
