"""GPU parity of the device-resident client-update store (srfl_amd.store,
csrc/store.hip): the step either side of the aggregation.

* record / momentum / apply kernels bit-exact against what the reference
  computes after its per-layer D2H (numpy float32 minus, numpy's promotion of
  the momentum form) and against torch's own ``p.data.sub_`` of the aggregate
  (simulate.py:187-199, 400-404);
* the ``--agg`` dispatch on store-backed ``local_grads`` (rows gathered on the
  device, icml2021_history's clipped rows written back into the store, the
  update applied in one launch) against the reference's own dispatch fixtures
  (tests/golden/dispatch_*.npz), with the tolerances of test_gpu_dispatch;
* ``fl_round`` end to end with real local SGD on the device against the
  reference's host flow (D2H of every client's layers, numpy aggregation by the
  oracle, ``sub_`` of the numpy aggregate).
"""
from __future__ import annotations

import random
import types
import warnings

import numpy as np
import pytest
import torch

from dispatch_cases import AGGS, CONFIGS, MOMENTUM_AGGS, layer_shapes, load_fixture, round_args, _flat
from oracle import attacks_np, robust_np as orc
from test_gpu_dispatch import _check

pytestmark = pytest.mark.gpu

CONVNET = [(30, 1, 5, 5), (30,), (30, 30, 5, 5), (30,), (200, 1470), (200,), (10, 200), (10,)]   # C1, D=319520


def _params(shapes, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [torch.nn.Parameter((0.1 * torch.randn(s, generator=g)).cuda()) for s in shapes]


def _perturb(params, seed, scale=1e-3):
    g = torch.Generator(device="cpu").manual_seed(seed)
    with torch.no_grad():
        for p in params:
            p.add_((scale * torch.randn(p.shape, generator=g)).cuda())


def test_record_delta_bit_exact_and_restores():
    from srfl_amd import store as st
    params = _params(CONVNET, 1)
    S = st.ClientStore(params, nworker=5)
    assert S.D == 319520
    copy_np = [p.detach().cpu().numpy() for p in params]
    S.snapshot()
    for c in (3, 0):
        _perturb(params, 10 + c)
        cur_np = [p.detach().cpu().numpy() for p in params]
        S.record(c)
        for l, (a, b) in enumerate(zip(copy_np, cur_np)):
            got = S.local_grads[c][l].cpu().numpy()
            assert got.dtype == np.float32
            np.testing.assert_array_equal(got, a - b)            # simulate.py:193-194 after the D2H
        for p, a in zip(params, copy_np):                          # restored, :196-199
            np.testing.assert_array_equal(p.detach().cpu().numpy(), a)
    np.testing.assert_array_equal(S.U[1].cpu().numpy(), 0.0)       # never written: np.zeros


@pytest.mark.parametrize("beta", [0.9, 0.5, 0.0])
def test_record_momentum_bit_exact(beta):
    from srfl_amd import store as st
    params = _params(CONVNET[:4], 2)
    S = st.ClientStore(params, nworker=3, momentum=True, beta=beta)
    rng = np.random.default_rng(3)
    prev = [rng.standard_normal(s) * 1e-3 for s in CONVNET[:4]]     # float64, like np.zeros + rounds
    for l, v in enumerate(S.local_grads[2]):
        v.copy_(torch.from_numpy(prev[l]))
    copy_np = [p.detach().cpu().numpy() for p in params]
    S.snapshot()
    _perturb(params, 4)
    cur_np = [p.detach().cpu().numpy() for p in params]
    S.record(2)
    for l in range(4):
        want = (1 - beta) * (copy_np[l] - cur_np[l]) + beta * prev[l]   # simulate.py:190-191 in numpy
        got = S.local_grads[2][l].cpu().numpy()
        assert got.dtype == want.dtype == np.float64
        np.testing.assert_array_equal(got, want)
    # a replaced entry (an attack's output) feeds the momentum, then the view is back
    rep = torch.full(CONVNET[1], 0.25, dtype=torch.float64, device="cuda")
    S.local_grads[2][1] = rep
    S.snapshot()
    S.record(2)
    assert S.intact([2])
    want = np.float32(1 - beta) * np.zeros(CONVNET[1], np.float32) + beta * np.full(CONVNET[1], 0.25)
    np.testing.assert_array_equal(S.local_grads[2][1].cpu().numpy(), want)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_apply_matches_torch_sub(dtype):
    from srfl_amd import store as st
    params = _params(CONVNET, 5)
    ref = [p.detach().clone() for p in params]
    S = st.ClientStore(params, nworker=1)
    rng = np.random.default_rng(6)
    flat = (rng.standard_normal(S.D) * 1e-2).astype(dtype)
    S.apply(torch.from_numpy(flat).cuda())
    for l, r in enumerate(ref):
        lo, hi = S.seg[l], S.seg[l + 1]
        r.sub_(torch.from_numpy(flat[lo:hi].reshape(CONVNET[l])).cuda())   # simulate.py:400-404
        np.testing.assert_array_equal(params[l].detach().cpu().numpy(), r.cpu().numpy())


def test_store_rejects_bad_input():
    from srfl_amd import store as st
    with pytest.raises(RuntimeError):
        st.ClientStore([torch.zeros(3)], 2)
    with pytest.raises(TypeError):
        st.ClientStore([torch.zeros(3, dtype=torch.float64, device="cuda")], 2)
    S = st.ClientStore([torch.zeros(3, device="cuda")], 2)
    with pytest.raises(IndexError):
        S.record(2)
    with pytest.raises(ValueError):
        S.apply(torch.zeros(4, device="cuda"))


# ---------------------------------------------------------------------------
# the dispatch on store-backed local_grads vs the reference's fixtures
# ---------------------------------------------------------------------------
def _replay_store(cfg, agg, fx):
    """tests/golden/dispatch_cases.replay with the updates written into a
    ClientStore's rows (momentum form on the device for the two stateful
    aggregators) and the round run by aggregate_and_apply on the store."""
    from srfl_amd import dispatch, store as st
    shapes = layer_shapes(cfg)
    sizes = [int(np.prod(s)) for s in shapes]
    np.random.seed(cfg["np_seed"])
    flat0 = fx["params0"]
    params, off = [], 0
    for s, n in zip(shapes, sizes):
        params.append(torch.nn.Parameter(torch.from_numpy(flat0[off:off + n].reshape(s).copy()).cuda()))
        off += n
    S = st.ClientStore(params, cfg["nworker"], momentum=agg in MOMENTUM_AGGS, beta=cfg["beta"])
    lg = S.local_grads
    args = round_args(cfg, agg)
    state = dispatch.DispatchState()
    for r in range(cfg["rounds"]):
        x = fx["x_r%d" % r]
        choices = np.random.choice(cfg["nworker"], cfg["perround"], replace=False)
        for c in choices:
            off = 0
            for li, (s, n) in enumerate(zip(shapes, sizes)):
                upd = torch.from_numpy(x[c, off:off + n].reshape(s).copy()).cuda()
                v = lg[c][li]
                v.copy_((1 - args.beta) * upd + args.beta * v if agg in MOMENTUM_AGGS else upd)
                off += n
        assert S.intact(choices)
        try:
            avg = dispatch.aggregate_and_apply(agg, params, lg, choices, args, state)
        except Exception as e:
            yield {"round": r, "error": type(e).__name__, "exc": e}
            return
        assert S.intact(choices)      # history's clipped rows went back into the store
        rec = {"round": r, "out": _flat(avg), "params": _flat(params), "choices": np.asarray(choices).copy(),
               "dtypes": [str(a.dtype).replace("torch.", "") for a in avg]}
        if agg in MOMENTUM_AGGS:
            rec["grads"] = np.stack([_flat(lg[c]) for c in choices])
        yield rec


@pytest.mark.parametrize("cfg", CONFIGS, ids=[c["name"] for c in CONFIGS])
@pytest.mark.parametrize("agg", AGGS)
def test_dispatch_store_matches_reference(cfg, agg):
    fx = load_fixture(cfg)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _check(cfg, agg, fx, _replay_store(cfg, agg, fx), host=False)


# ---------------------------------------------------------------------------
# fl_round: real local training on the device vs the reference's host flow
# ---------------------------------------------------------------------------
class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = torch.nn.Linear(20, 16)
        self.fc2 = torch.nn.Linear(16, 4)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


def _data(nworker):
    g = torch.Generator(device="cpu").manual_seed(11)
    xs = torch.randn(nworker, 3, 8, 20, generator=g).cuda()      # 3 batches of 8 per client
    ys = torch.randint(0, 4, (nworker, 3, 8), generator=g).cuda()
    return xs, ys


EXACT = ("average", "median", "trimmedmean", "krum", "clustering")


@pytest.mark.parametrize("agg,attack", [("average", "noattack"), ("median", "noattack"),
                                        ("trimmedmean", "noattack"), ("krum", "noattack"),
                                        ("clustering", "noattack"), ("bulyantrimmedmean", "noattack"),
                                        ("filterl2", "noattack"), ("icml2021_history", "noattack"),
                                        ("iclr2022_bucketing", "noattack"), ("median", "xie"),
                                        ("trimmedmean", "trimmedmean")])
def test_fl_round_matches_host_flow(agg, attack):
    from srfl_amd import dispatch, store as st
    torch.manual_seed(0)
    net = _Net().cuda()
    nworker, malnum = 24, 4
    args = types.SimpleNamespace(agg=agg, malnum=malnum, nworker=nworker, perround=nworker, sigma=1e-5,
                                 buckets=6, tau=0.05, beta=0.9)
    momentum = agg in MOMENTUM_AGGS
    params = list(net.parameters())
    S = st.ClientStore(params, nworker, momentum=momentum, beta=args.beta)
    state = dispatch.DispatchState()
    xs, ys = _data(nworker)
    opt = torch.optim.SGD(params, lr=0.05)
    crit = torch.nn.CrossEntropyLoss()
    host_lg = [[np.zeros(tuple(p.shape)) for p in params] for _ in range(nworker)]
    prev = None
    mal_index = list(range(malnum))
    np.random.seed(21)
    for rnd in range(2):
        choices = np.random.choice(nworker, nworker, replace=False)
        copy_np = [p.detach().cpu().numpy() for p in params]

        def local_update(c):
            for b in range(3):
                opt.zero_grad()
                crit(net(xs[c, b]), ys[c, b]).backward()
                opt.step()
            cur = [p.detach().cpu().numpy() for p in params]                 # the reference's D2H
            for l in range(len(params)):
                d = copy_np[l] - cur[l]
                host_lg[c][l] = (1 - args.beta) * d + args.beta * host_lg[c][l] if momentum else d

        random_state = random.getstate()
        np_state = np.random.get_state()
        host_choices = choices.copy()
        flat = st.fl_round(net, S, choices, local_update, args, state, attack=attack, mal_index=mal_index)
        # the reference's host flow on the captured updates, from the same RNG states
        if attack == "xie":
            attacks_np.attack_xie(host_lg, 1, host_choices, mal_index)
        elif attack == "trimmedmean":
            rs = random.Random()
            rs.setstate(random_state)
            attacks_np.attack_trimmedmean(copy_np, host_lg, mal_index, b=1.5, rng=rs)
        np.random.set_state(np_state)
        want, prev = orc.dispatch_round(agg, host_lg, host_choices, args, prev)
        np.testing.assert_array_equal(choices, host_choices)
        want_flat = np.concatenate([np.asarray(w, dtype=np.float64).ravel() for w in want])
        got = flat.cpu().numpy().astype(np.float64)
        if agg in EXACT and attack != "trimmedmean":
            np.testing.assert_array_equal(got, want_flat)
            expect = [torch.from_numpy(a).cuda().sub_(torch.from_numpy(np.asarray(w)).cuda())
                      for a, w in zip(copy_np, want)]
            for p, e in zip(params, expect):
                np.testing.assert_array_equal(p.detach().cpu().numpy(), e.cpu().numpy())
        else:
            np.testing.assert_allclose(got, want_flat, rtol=0, atol=2e-5 * max(np.abs(want_flat).max(), 1e-30))
        if momentum:
            for c in choices:
                np.testing.assert_allclose(_flat(S.local_grads[c]), _flat(host_lg[c]), rtol=0, atol=1e-12)


def test_gan_layers_from_store_byte_identical(tmp_path):
    """formats.save_gan_layers on store-backed local_grads (one device gather +
    one copy per layer) writes the same bytes as the reference's np.save of the
    host list (simulate_gan.py:306-313)."""
    import io
    from srfl_amd import formats, store as st
    params = _params(CONVNET, 9)
    S = st.ClientStore(params, nworker=6)
    S.snapshot()
    for c in range(6):
        _perturb(params, 30 + c)
        S.record(c)
    choices = np.array([4, 1, 5, 0])
    host = [[t.cpu().numpy() for t in S.local_grads[c]] for c in range(6)]
    for idx, p in enumerate(formats.save_gan_layers(S.local_grads, choices, 2, str(tmp_path))):
        buf = io.BytesIO()
        np.save(buf, [host[c][idx] for c in choices])
        with open(p, "rb") as f:
            assert f.read() == buf.getvalue()
