"""GPU parity of the attack-side callers (srfl_amd.attack)
against the live reference's outputs (tests/golden/attack_*.npz) and the
CPU oracle (oracle/attacks_np.py).

Bars: bit-exact malicious rows for all three attacks (attack_krum's lambda
decision included), bit-exact Mersenne Twister words, and the Python random
state after attack_trimmedmean equal to the reference's.  Both calling
conventions: numpy local_grads (host) and CUDA tensors (device)."""
from __future__ import annotations

import random

import numpy as np
import pytest
import torch

from attack_cases import CASES, case_clients, case_choices, load_fixture
from oracle import attacks_np as orc

pytestmark = pytest.mark.gpu


def _flat(arrs):
    out = []
    for a in arrs:
        if isinstance(a, torch.Tensor):
            a = a.detach().cpu().numpy()
        out.append(np.asarray(a, dtype=np.float64).ravel())
    return np.concatenate(out)


def _cases(func):
    return [c for c in CASES if c["func"] == func]


class _Net:
    def __init__(self, params, device=None):
        self._p = [torch.nn.Parameter(torch.from_numpy(p.copy()).to(device) if device else torch.from_numpy(p.copy()))
                   for p in params]

    def parameters(self):
        return iter(self._p)


def _to_dev(grads):
    return [[torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in row] for row in grads]


@pytest.mark.parametrize("seed,pre,n", [(1, 0, 5000), (2, 1, 1301), (3, 623, 700), (4, 624, 624), (5, 1001, 3),
                                        (7, 17, 200000)])
def test_mt19937_words_equal_python_random(seed, pre, n):
    from srfl_amd import attack
    rng = random.Random(seed)
    for _ in range(pre):
        rng.getrandbits(32)
    words, state = attack.mt19937_words(rng.getstate()[1], n, torch.device("cuda"))
    got = words.cpu().numpy().view(np.uint32)
    want = np.array([rng.getrandbits(32) for _ in range(n)], dtype=np.uint32)
    np.testing.assert_array_equal(got, want)
    assert state == rng.getstate()[1]


@pytest.mark.parametrize("device", [False, True], ids=["host", "device"])
@pytest.mark.parametrize("case", _cases("bulyan_attack_krum"), ids=lambda c: c["name"])
def test_bulyan_attack_krum_matches_reference(case, device):
    """attack.py:264-308 (not called by simulate.py): the live reference's rows,
    the target layer's ones-direction and the other layers' zero (-0.0) rows."""
    from srfl_amd import attack
    fx = load_fixture(case)
    grads, params = case_clients(case)
    if device:
        grads = _to_dev(grads)
    net = _Net(params)
    for idx in range(len(params)):
        ret = attack.bulyan_attack_krum(net, grads, case["mal"], idx, lower_bound=case["lower_bound"],
                                        target_layer=case["target_layer"], target_idx=case["target_idx"])
        assert ret is grads
    for k, c in enumerate(case["mal"]):
        got = _flat(grads[c])
        np.testing.assert_array_equal(got, fx["mal_out"][k])
        np.testing.assert_array_equal(np.signbit(got), np.signbit(fx["mal_out"][k]))
        assert all((a.dtype == torch.float64) if device else (a.dtype == np.float64) for a in grads[c])
    benign = [c for c in range(case["m"]) if c not in set(case["mal"])]
    np.testing.assert_array_equal(np.stack([_flat(grads[c]) for c in benign]), fx["benign_out"])


@pytest.mark.parametrize("device", [False, True], ids=["host", "device"])
@pytest.mark.parametrize("case", _cases("attack_krum"), ids=lambda c: c["name"])
def test_attack_krum_matches_reference(case, device):
    from srfl_amd import attack
    fx = load_fixture(case)
    grads, params = case_clients(case)
    if device:
        grads = _to_dev(grads)
    net = _Net(params)
    for idx in range(len(params)):
        ret = attack.attack_krum(net, grads, case["mal"], idx, lower_bound=case["lower_bound"])
        assert ret is grads
    for k, c in enumerate(case["mal"]):
        np.testing.assert_array_equal(_flat(grads[c]), fx["mal_out"][k])
        assert all((a.dtype == torch.float64) if device else (a.dtype == np.float64) for a in grads[c])
    benign = [c for c in range(case["m"]) if c not in set(case["mal"])]
    np.testing.assert_array_equal(np.stack([_flat(grads[c]) for c in benign]), fx["benign_out"])


def test_attack_krum_lambda_and_pick_vs_oracle_larger_layer():
    """m = 48 clients, d = 20000: lambda, the pick's class and the malicious
    row against the oracle's loop (which re-runs krum per lambda)."""
    from srfl_amd import attack
    from synth import make_rows
    m, d = 48, 20000
    x = make_rows(m, d, 4242)
    mal = list(range(0, 48, 5))
    grads = [[x[c].copy()] for c in range(m)]
    lam_ref, row_ref = orc.attack_krum([[x[c].copy()] for c in range(m)], mal, 0, 1e-8)
    X = torch.from_numpy(x).cuda()
    mask = torch.tensor([1 if c in mal else 0 for c in range(m)], dtype=torch.int32, device="cuda")
    benign = torch.tensor([c for c in range(m) if c not in mal], dtype=torch.int32, device="cuda")
    row, lam, pick = attack.attack_krum_layer(X, mask, benign, 1e-8)
    assert float(lam.item()) == lam_ref
    np.testing.assert_array_equal(row.cpu().numpy(), row_ref)
    attack.attack_krum(None, grads, mal, 0)
    for c in mal:
        np.testing.assert_array_equal(grads[c][0], row_ref)


@pytest.mark.parametrize("device", [False, True], ids=["host", "device"])
@pytest.mark.parametrize("case", _cases("attack_trimmedmean"), ids=lambda c: c["name"])
def test_attack_trimmedmean_matches_reference(case, device):
    from srfl_amd import attack
    fx = load_fixture(case)
    grads, params = case_clients(case)
    if device:
        grads = _to_dev(grads)
    net = _Net(params, "cuda" if device else None)
    saved = random.getstate()
    try:
        random.setstate((3, tuple(int(v) for v in fx["state_in"]), None))
        ret = attack.attack_trimmedmean(net, grads, case["mal"], b=case["b"])
        assert ret is grads
        assert random.getstate()[1] == tuple(int(v) for v in fx["state_out"])
    finally:
        random.setstate(saved)
    for k, c in enumerate(case["mal"]):
        np.testing.assert_array_equal(_flat(grads[c]), fx["mal_out"][k])
    benign = [c for c in range(case["m"]) if c not in set(case["mal"])]
    np.testing.assert_array_equal(np.stack([_flat(grads[c]) for c in benign]), fx["benign_out"])


def test_attack_trimmedmean_large_vs_oracle_and_continuation():
    """D = 300000 elements (600000 words, many twists) against the oracle, and
    the next draw after the call equals the reference module's next draw."""
    from srfl_amd import attack
    from synth import make_rows
    m, D = 9, 300000
    x = make_rows(m, D, 77)
    p = (0.1 * np.random.default_rng(78).standard_normal(D)).astype(np.float32)
    mal = [2, 5]
    want = [[x[c].copy()] for c in range(m)]
    rng = random.Random(99)
    orc.attack_trimmedmean([p], want, mal, b=1.5, rng=rng)
    grads = [[x[c].copy()] for c in range(m)]
    saved = random.getstate()
    try:
        random.setstate(random.Random(99).getstate())
        attack.attack_trimmedmean(_Net([p]), grads, mal, b=1.5)
        assert random.random() == rng.random()
    finally:
        random.setstate(saved)
    for c in mal:
        np.testing.assert_array_equal(grads[c][0], want[c][0])


@pytest.mark.parametrize("device", [False, True], ids=["host", "device"])
@pytest.mark.parametrize("case", _cases("attack_xie"), ids=lambda c: c["name"])
def test_attack_xie_matches_reference(case, device):
    from srfl_amd import attack
    fx = load_fixture(case)
    grads, _ = case_clients(case)
    if device:
        grads = _to_dev(grads)
    choices = case_choices(case)
    ret = attack.attack_xie(grads, case["weight"], choices, case["mal"])
    assert ret is grads
    for k, c in enumerate(case["mal"]):
        np.testing.assert_array_equal(_flat(grads[c]), fx["mal_out"][k])
    assert grads[case["mal"][0]] is grads[case["mal"][-1]]


def test_attack_errors_match_reference_classes():
    from srfl_amd import attack
    grads, params = case_clients(CASES[3])
    with pytest.raises(ValueError):
        attack.attack_trimmedmean(_Net(params), grads, list(range(CASES[3]["m"])))


def test_attack_krum_many_clients_vs_oracle():
    """m = 600 clients (distance lists longer than 512: numpy's pairwise sum one
    split level deeper), lambda and the malicious row against the oracle."""
    from srfl_amd import attack
    from synth import make_rows
    m, d = 600, 48
    x = make_rows(m, d, 4343)
    mal = list(range(0, m, 7))
    lam_ref, row_ref = orc.attack_krum([[x[c].copy()] for c in range(m)], mal, 0, 1e-8)
    X = torch.from_numpy(x).cuda()
    mask = torch.tensor([1 if c in mal else 0 for c in range(m)], dtype=torch.int32, device="cuda")
    benign = torch.tensor([c for c in range(m) if c not in mal], dtype=torch.int32, device="cuda")
    row, lam, pick = attack.attack_krum_layer(X, mask, benign, 1e-8)
    assert float(lam.item()) == lam_ref
    np.testing.assert_array_equal(row.cpu().numpy(), row_ref)
