"""Case table for the DBA harness's Helper aggregators (src/DBA/helper.py,
SURVEY.md §8(f).4), shared by gen_dba_fixtures.py (which runs the live
reference in the build container) and the tests (which only read the .npz).

A case is one aggregation call: N client update dicts over the layers of a
small CNN-like model (DBA_LAYERS), num_samples per client, a Helper method with
its keyword arguments, the Helper.params it reads, and the Python ``random``
seed set before the call (sharding / bucketing shuffle with it).
"""
from __future__ import annotations

import os

import numpy as np

from synth import make_rows

HERE = os.path.dirname(os.path.abspath(__file__))

DBA_LAYERS = [("conv.weight", (3, 1, 3, 3)), ("conv.bias", (3,)), ("fc1.weight", (8, 12)), ("fc1.bias", (8,)),
              ("fc2.weight", (4, 8)), ("fc2.bias", (4,))]
D = int(sum(np.prod(s) for _, s in DBA_LAYERS))   # 170

# name -> (method, kwargs, N, byz, params overrides, rounds)
CASES = {
    "mean_n24": ("fed_avg", {}, 24, 5, {}, 1),
    "median_n24": ("median", {}, 24, 5, {}, 1),
    "median_n25": ("median", {}, 25, 5, {}, 1),
    "trimmedmean_n24_b02": ("trimmed_mean", {"beta": 0.2}, 24, 5, {}, 1),
    "trimmedmean_n25_b01": ("trimmed_mean", {"beta": 0.1}, 25, 5, {}, 1),
    "krum_n24_f5": ("krum", {"f": 5}, 24, 5, {}, 1),
    "krum_n25_f0": ("krum", {"f": 0}, 25, 5, {}, 1),
    "momkrum_n24_f5": ("mom_krum", {"f": 5}, 24, 5, {}, 1),
    "momkrum_n25_f5": ("mom_krum", {"f": 5}, 25, 5, {}, 1),
    "bulyankrum_n24_f5": ("bulyan_krum", {"f": 5}, 24, 5, {}, 1),
    "bulyankrum_n25_f2": ("bulyan_krum", {"f": 2}, 25, 2, {}, 1),
    "bulyanmedian_n25_f5": ("bulyan_median", {"f": 5}, 25, 5, {}, 1),
    "bulyanmedian_n24_f5": ("bulyan_median", {"f": 5}, 24, 5, {}, 1),
    "bulyantrimmed_n25_f5": ("bulyan_trimmed_mean", {"f": 5}, 25, 5, {}, 1),
    "filterl2_n24": ("filterl2", {"sigma": 1e-5, "expansion": 20, "itv": None}, 24, 5, {}, 1),
    "exnoregret_n24": ("ex_noregret", {"eps": 1. / 5, "sigma": 1e-5, "expansion": 20, "itv": 1000}, 24, 5, {}, 1),
    "exnoregret_n24_sqrt": ("ex_noregret", {"eps": 1. / 5, "sigma": 1e-5, "expansion": 20, "itv": None}, 24, 5,
                            {}, 1),
    "history_n24": ("history", {}, 24, 5, {}, 2),
    "geomed_n24": ("geometric_median_update", {"maxiter": 4}, 24, 5, {}, 1),
    "mean_sharded_n100": ("fed_avg", {}, 100, 20, {"sharding": True}, 1),
    "median_sharded_n100": ("median", {}, 100, 20, {"sharding": True}, 1),
    "bucketing_n100": ("bucketing", {}, 100, 20, {}, 2),
    "sharding_n25": ("fed_avg", {}, 25, 5, {"sharding": True}, 1),   # 50 shards of 1 > 25 clients: IndexError
    # FoolsGold (helper.py:291-325, 1321-1417): updates carry per-layer gradient LISTS; SGD step on the model
    "foolsgold_n24": ("foolsgold_update", {}, 24, 5, {"fg_use_memory": False}, 2),
    "foolsgold_mem_n24": ("foolsgold_update", {}, 24, 5, {"fg_use_memory": True}, 2),
    # 2f < N < 4f: beta < 0, torch slicing [:beta] drops -beta values (keep 0 -> mean of nothing, NaN)
    "bulyankrum_n30_f8_negbeta": ("bulyan_krum", {"f": 8}, 30, 8, {}, 1),
    "bulyanmedian_n30_f8_negbeta": ("bulyan_median", {"f": 8}, 30, 8, {}, 1),
    "bulyantrimmed_n40_f12_negbeta": ("bulyan_trimmed_mean", {"f": 12}, 40, 12, {}, 1),
    "bulyanmedian_n30_f10_negbeta": ("bulyan_median", {"f": 10}, 30, 10, {}, 1),
    # a NaN coordinate in one client (case_rows injects it): torch.median propagates it, every distance
    # of the round is NaN and ``assert min_index != None`` fails (helper.py:1047 / :1119)
    "bulyanmedian_nan_n24_f5": ("bulyan_median", {"f": 5}, 24, 5, {}, 1),
    "bulyantrimmed_nan_n24_f5": ("bulyan_trimmed_mean", {"f": 5}, 24, 5, {}, 1),
    "bulyankrum_nan_n24_f5": ("bulyan_krum", {"f": 5}, 24, 5, {}, 1),
}

BASE_PARAMS = {"eta": 1, "sharding": False, "shard_size": 0.2, "adversary_list": [0, 1, 2, 3, 4],
               "poisoning_per_batch": 20, "batch_size": 64, "diff_privacy": False,
               "lr": 0.1, "momentum": 0.9, "decay": 0.0005}


def case_rows(name, rnd=0):
    """(N, D) float32 client updates and the (N,) num_samples of round ``rnd``."""
    _, _, n, byz, _, _ = CASES[name]
    seed = 1000 + 97 * list(CASES).index(name) + rnd
    x = make_rows(n, D, seed, byz=byz)
    if "_nan_" in name:
        x[7, 13] = np.nan
    ns = np.random.default_rng(seed + 1).integers(200, 600, size=n).astype(np.int64)
    return x, ns


def case_params(name):
    p = dict(BASE_PARAMS)
    p.update(CASES[name][4])
    return p


def case_seed(name):
    return 7 + list(CASES).index(name)


def fixture_path(name):
    return os.path.join(HERE, "dba_%s.npz" % name)
