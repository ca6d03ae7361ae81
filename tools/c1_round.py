#!/usr/bin/env python3
"""C1 round timing: one round of simulate.py's loop
body around the aggregation, MNIST ConvNet shapes (8 layers, D = 319,520),
N = nworker = perround = 100, malnum = 20, on one MI355X.

Local training is emulated by one device add of a fixed per-client update to
the parameters (identical in both flows; no MNIST here).  Two flows:

  host   the reference's data movement: per client and layer
         ``params_copy.cpu().numpy() - p.cpu().numpy()`` (simulate.py:193-194)
         into host ``local_grads``, parameters restored (:196-199),
         dispatch.aggregate on the host lists (pinned stack + H2D + kernels +
         D2H), then ``p.data.sub_(torch.from_numpy(avg).to(device))`` (:400-404);
  store  srfl_amd.store.ClientStore: one record launch per client (delta +
         restore), dispatch.aggregate_and_apply on the store (device row
         gather + kernels + one apply launch); nothing crosses PCIe.

Prints one JSON object per aggregator: round_ms for both flows and the
aggregation-only share of the store flow.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import srfl_loader  # noqa: E402

srfl_loader.load()
from srfl_amd import dispatch, store as st  # noqa: E402

CONVNET = [(30, 1, 5, 5), (30,), (30, 30, 5, 5), (30,), (200, 1470), (200,), (10, 200), (10,)]
AGGS = ["average", "median", "trimmedmean", "krum", "clustering", "bulyankrum", "bulyantrimmedmean",
        "filterl2", "ex_noregret", "mom_filterl2", "iclr2022_bucketing", "icml2021_history"]
MOMENTUM = ("iclr2022_bucketing", "icml2021_history")


def sync():
    torch.cuda.synchronize()


def make(n):
    g = torch.Generator(device="cpu").manual_seed(0)
    params = [torch.nn.Parameter((0.1 * torch.randn(s, generator=g)).cuda()) for s in CONVNET]
    D = sum(p.numel() for p in params)
    upd = (1e-3 * torch.randn(n, D, generator=g)).cuda()
    upd[:20] *= -10.0
    return params, upd


def train(params, upd_row):
    """Stand-in for client c's local SGD: params += its update."""
    off = 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            p.add_(upd_row[off:off + n].view(p.shape))
            off += n


def host_round(agg, params, upd, args, state, lg):
    copy = [p.detach().clone() for p in params]
    copy_np = [c.cpu().numpy() for c in copy]
    choices = np.arange(args.nworker)
    for c in choices:
        train(params, upd[c])
        cur = [p.detach().cpu().numpy() for p in params]
        for l in range(len(params)):
            d = copy_np[l] - cur[l]
            lg[c][l] = (1 - args.beta) * d + args.beta * lg[c][l] if agg in MOMENTUM else d
        with torch.no_grad():
            for p, c0 in zip(params, copy):
                p.copy_(c0)
    avg = dispatch.aggregate(agg, lg, choices, args, state)
    dispatch.apply_update(params, avg)


def store_round(agg, params, upd, args, state, S):
    choices = np.arange(args.nworker)
    S.snapshot()
    for c in choices:
        train(params, upd[c])
        S.record(c)
    sync()
    t0 = time.perf_counter()
    dispatch.aggregate_and_apply(agg, params, S.local_grads, choices, args, state)
    sync()
    return time.perf_counter() - t0


def timed(fn, reps):
    out = []
    for _ in range(reps):
        sync()
        t0 = time.perf_counter()
        r = fn()
        sync()
        out.append((time.perf_counter() - t0, r))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--aggs", default=",".join(AGGS))
    a = ap.parse_args()
    n = 100
    for agg in a.aggs.split(","):
        args = dispatch.RoundArgs(agg=agg, nworker=n, perround=n, malnum=20)
        params, upd = make(n)
        lg = [[np.zeros(s) for s in CONVNET] for _ in range(n)]
        state = dispatch.DispatchState()
        host_round(agg, params, upd, args, state, lg)                      # warm-up
        h = timed(lambda: host_round(agg, params, upd, args, state, lg), a.reps)
        params, upd = make(n)
        S = st.ClientStore(params, n, momentum=agg in MOMENTUM)
        state = dispatch.DispatchState()
        store_round(agg, params, upd, args, state, S)
        s = timed(lambda: store_round(agg, params, upd, args, state, S), a.reps)
        rec = {"workload": "C1 round, ConvNet D=319520, N=100, f=20", "agg": agg,
               "host_round_ms": round(1e3 * min(t for t, _ in h), 3),
               "store_round_ms": round(1e3 * min(t for t, _ in s), 3),
               "store_aggregate_apply_ms": round(1e3 * min(r for _, r in s), 3)}
        rec["speedup"] = round(rec["host_round_ms"] / rec["store_round_ms"], 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
