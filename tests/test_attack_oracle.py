"""CPU pin of the attack oracle against the golden fixtures
written by the live reference (tests/golden/gen_attack_fixtures.py), and of
the device kernel's three-phase Mersenne Twister decomposition against
Python's own ``random``."""
from __future__ import annotations

import os
import random
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))
from attack_cases import CASES, case_clients, case_choices, load_fixture  # noqa: E402
from oracle import attacks_np as orc  # noqa: E402


def _flat(arrs):
    return np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in arrs])


def _cases(func):
    return [c for c in CASES if c["func"] == func]


@pytest.mark.parametrize("case", _cases("bulyan_attack_krum"), ids=lambda c: c["name"])
def test_bulyan_attack_krum_oracle_matches_reference(case):
    fx = load_fixture(case)
    grads, params = case_clients(case)
    shapes = [p.shape for p in params]
    for idx in range(len(params)):
        orc.bulyan_attack_krum(shapes, grads, case["mal"], idx, case["lower_bound"], case["target_layer"],
                               case["target_idx"])
    for k, c in enumerate(case["mal"]):
        np.testing.assert_array_equal(_flat(grads[c]), fx["mal_out"][k])


@pytest.mark.parametrize("case", _cases("attack_krum"), ids=lambda c: c["name"])
def test_attack_krum_oracle_matches_reference(case):
    fx = load_fixture(case)
    grads, params = case_clients(case)
    for idx in range(len(params)):
        orc.attack_krum(grads, case["mal"], idx, case["lower_bound"])
    for k, c in enumerate(case["mal"]):
        np.testing.assert_array_equal(_flat(grads[c]), fx["mal_out"][k])
    benign = [c for c in range(case["m"]) if c not in set(case["mal"])]
    np.testing.assert_array_equal(np.stack([_flat(grads[c]) for c in benign]), fx["benign_out"])


@pytest.mark.parametrize("case", _cases("attack_trimmedmean"), ids=lambda c: c["name"])
def test_attack_trimmedmean_oracle_matches_reference(case):
    fx = load_fixture(case)
    grads, params = case_clients(case)
    rng = random.Random()
    rng.setstate((3, tuple(int(v) for v in fx["state_in"]), None))
    orc.attack_trimmedmean(params, grads, case["mal"], b=case["b"], rng=rng)
    for k, c in enumerate(case["mal"]):
        np.testing.assert_array_equal(_flat(grads[c]), fx["mal_out"][k])
    assert rng.getstate()[1] == tuple(int(v) for v in fx["state_out"])
    assert list(fx["mal_dtypes"]) == ["float64"] * len(params)


@pytest.mark.parametrize("case", _cases("attack_xie"), ids=lambda c: c["name"])
def test_attack_xie_oracle_matches_reference(case):
    fx = load_fixture(case)
    grads, _ = case_clients(case)
    choices = case_choices(case)
    np.testing.assert_array_equal(choices, fx["choices"])
    orc.attack_xie(grads, case["weight"], choices, case["mal"])
    for k, c in enumerate(case["mal"]):
        np.testing.assert_array_equal(_flat(grads[c]), fx["mal_out"][k])
    assert grads[case["mal"][0]] is grads[case["mal"][-1]]   # one shared list, like the reference


@pytest.mark.parametrize("seed,pre,n", [(1, 0, 5000), (2, 1, 1300), (3, 623, 700), (4, 624, 624), (5, 1001, 3),
                                        (6, 5, 0)])
def test_mt19937_three_phase_twist_equals_python_random(seed, pre, n):
    rng = random.Random(seed)
    for _ in range(pre):
        rng.getrandbits(32)
    words, state = orc.mt19937_phased(rng.getstate()[1], n)
    want = np.array([rng.getrandbits(32) for _ in range(n)], dtype=np.uint32)
    np.testing.assert_array_equal(words, want)
    assert state == rng.getstate()[1]
