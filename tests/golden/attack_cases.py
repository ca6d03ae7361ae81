"""Shared definition of the attack fixtures (gen_attack_fixtures.py writes them
from the live reference src/attack.py; tests/test_attack*.py replay them).
SURVEY.md §8(f).2: the attack-side callers of the aggregation path.

Cases (m clients, small ConvNet-like layers, updates from synth.make_rows):
  krum_A   m = 30, mal_index = range(6)          (simulate.py:81 convention)
  krum_B   m = 40, scattered mal_index, lower_bound 1e-5
  krum_C   m = 12, one malicious client (the search may fail -> smallest lambda)
  tm_A     m = 30, mal_index = range(6), b = 1.5 (simulate.py:220)
  tm_B     m = 20, scattered mal_index, b = 2 (the default), random state
           advanced by an odd number of words first
  xie_A    m = 30, choices = 20 of 30, mal_index = range(6), weight 1
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

SHAPES = [[3, 1, 5, 5], [3], [8, 24], [8], [4, 8], [4]]

CASES = [
    {"name": "krum_A", "func": "attack_krum", "m": 30, "mal": list(range(6)), "lower_bound": 1e-8, "seed": 901},
    {"name": "krum_B", "func": "attack_krum", "m": 40, "mal": [1, 4, 9, 16, 25, 36, 39], "lower_bound": 1e-5,
     "seed": 902},
    {"name": "krum_C", "func": "attack_krum", "m": 12, "mal": [5], "lower_bound": 1e-8, "seed": 903},
    {"name": "tm_A", "func": "attack_trimmedmean", "m": 30, "mal": list(range(6)), "b": 1.5, "py_seed": 11,
     "pre_words": 0, "seed": 904},
    {"name": "tm_B", "func": "attack_trimmedmean", "m": 20, "mal": [0, 3, 7, 19], "b": 2, "py_seed": 12,
     "pre_words": 37, "seed": 905},
    {"name": "xie_A", "func": "attack_xie", "m": 30, "mal": list(range(6)), "perround": 20, "weight": 1,
     "seed": 906},
    # bulyan_attack_krum (attack.py:264-308), target_layer / target_idx defaults and a non-default target
    {"name": "bkrum_A", "func": "bulyan_attack_krum", "m": 30, "mal": list(range(6)), "lower_bound": 1e-8,
     "target_layer": 0, "target_idx": 0, "seed": 907},
    {"name": "bkrum_B", "func": "bulyan_attack_krum", "m": 24, "mal": [2, 5, 11, 23], "lower_bound": 1e-5,
     "target_layer": 3, "target_idx": 1, "seed": 908},
]


def layer_sizes():
    return [int(np.prod(s)) for s in SHAPES]


def case_inputs(case):
    """(m, D) float32 client updates and (D,) float32 parameters."""
    from synth import make_rows
    D = sum(layer_sizes())
    x = make_rows(case["m"], D, case["seed"])
    p = (0.1 * np.random.default_rng(case["seed"] + 1).standard_normal(D)).astype(np.float32)
    return x, p


def split_layers(flat):
    out, off = [], 0
    for s, n in zip(SHAPES, layer_sizes()):
        out.append(flat[off:off + n].reshape(s))
        off += n
    return out


def case_clients(case):
    x, p = case_inputs(case)
    return [[a.copy() for a in split_layers(x[c])] for c in range(case["m"])], split_layers(p)


def case_choices(case):
    return np.random.default_rng(case["seed"] + 2).choice(case["m"], case["perround"], replace=False)


def fixture_path(case):
    return os.path.join(HERE, "attack_%s.npz" % case["name"])


def load_fixture(case):
    return np.load(fixture_path(case), allow_pickle=False)
