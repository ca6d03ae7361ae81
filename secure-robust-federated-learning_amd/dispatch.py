"""The per-layer aggregation dispatch of the reference's training loop
(src/simulate.py:231-404) on the MI355X.

In the reference this is an if/elif chain inside ``main()``: for each of the 14
``--agg`` names (simulate.py:76) it gathers, per layer ``idx``,
``[local_grads[c][idx] for c in choices]``, calls the aggregator on that list
and stores the result in ``average_grad[idx]``; then every parameter takes
``params[idx].data.sub_(average_grad[idx])`` (simulate.py:400-404).  Two
aggregators are inline and stateful: ``iclr2022_bucketing`` (:335-366) and
``icml2021_history`` (:367-388) keep ``prev_average_grad`` across rounds, and
history clips ``local_grads`` in place.

Here one round is staged ONCE: the chosen clients' layers become one
client-major ``N x D`` device matrix (D = all layers concatenated, a segment
table holds the layer offsets; one pinned H2D copy for host arrays, device
copies for device tensors).  Then

* coordinate-wise aggregators (average / median / trimmedmean) run as ONE
  launch over all D columns (they are per coordinate, so layer boundaries do
  not matter);
* MoM bucket means (clustering, mom_filterl2, mom_ex_noregret) are computed
  once over all D columns;
* per-layer aggregators (Krum, Bulyan, the spectral filters) run on column
  slices of that matrix (no copies: the row stride is D);
* the two stateful aggregators run the k7 clipping kernels with the norm taken
  across the segment table, ``prev_average_grad`` stays on the device.

``aggregate`` returns ``average_grad`` in the reference's convention (numpy
arrays of the layer shapes and numpy's dtypes for numpy inputs, device tensors
for device inputs; Krum returns the chosen client's own object).
``aggregate_and_apply`` is the device-resident round: the aggregate never
leaves the GPU and is subtracted from the parameters in place.
"""
from __future__ import annotations

import numpy as np
import torch

from . import engine

# simulate.py:76
AGG_NAMES = ("average", "ex_noregret", "filterl2", "krum", "median", "trimmedmean", "bulyankrum",
             "bulyantrimmedmean", "bulyanmedian", "mom_filterl2", "mom_ex_noregret", "iclr2022_bucketing",
             "icml2021_history", "clustering")
_BULYAN = {"bulyankrum": "krum", "bulyanmedian": "median", "bulyantrimmedmean": "trimmedmean"}
_STATEFUL = ("iclr2022_bucketing", "icml2021_history")


class RoundArgs:
    """The ``args`` fields the dispatch reads, with simulate.py:59-78 defaults."""

    def __init__(self, agg="average", nworker=100, perround=100, malnum=20, sigma=1e-5, buckets=10, tau=10.,
                 beta=0.9):
        self.agg = agg
        self.nworker = nworker
        self.perround = perround
        self.malnum = malnum
        self.sigma = sigma
        self.buckets = buckets
        self.tau = tau
        self.beta = beta


class DispatchState:
    """Cross-round state of the dispatch: ``prev_average_grad`` (simulate.py:132),
    kept on the device as one flat float64 vector over all layers."""

    def __init__(self):
        self.prev = None

    @property
    def prev_average_grad(self):
        return self.prev


class StagedRound:
    """The chosen clients' layers as one (N, D) device matrix plus the segment
    table (layer offsets) and what is needed to hand results back."""

    def __init__(self, X, seg, shapes, layer_dtypes, device_io):
        self.X = X
        self.seg = seg
        self.shapes = shapes
        self.layer_dtypes = layer_dtypes
        self.device_io = device_io

    @property
    def nlayers(self):
        return len(self.shapes)

    def cols(self, layer):
        return self.X[:, self.seg[layer]:self.seg[layer + 1]]


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("srfl_amd.dispatch needs an MI355X (HIP device); no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def stage_round(local_grads, choices, dtype=torch.float32):
    """Stack ``local_grads[c][l]`` for c in ``choices`` into (N, D) on the device."""
    choices = [int(c) for c in choices]
    store = getattr(local_grads, "store", None)
    if store is not None and store.intact(choices):
        # device-resident local_grads (store.py): one gather of the chosen rows
        ldt = np.float64 if store.dtype == torch.float64 else np.float32
        return StagedRound(store.stage(choices, dtype), list(store.seg), list(store.shapes),
                           [np.dtype(ldt)] * len(store.shapes), True)
    first = local_grads[choices[0]]
    device_io = isinstance(first[0], torch.Tensor) and first[0].is_cuda
    shapes = [tuple(t.shape) for t in first]
    sizes = [int(np.prod(s, dtype=np.int64)) for s in shapes]
    seg = [0]
    for s in sizes:
        seg.append(seg[-1] + s)
    D = seg[-1]
    n = len(choices)
    layer_dtypes = []
    for l in range(len(shapes)):
        dts = {np.dtype(_np_dtype(local_grads[c][l])) for c in choices}
        layer_dtypes.append(np.result_type(*dts))
    if device_io:
        dev = first[0].device
        X = torch.empty((n, D), dtype=dtype, device=dev)
        for l in range(len(shapes)):
            cols = torch.stack([local_grads[c][l].reshape(-1) for c in choices])
            X[:, seg[l]:seg[l + 1]].copy_(cols)
        return StagedRound(X, seg, shapes, layer_dtypes, True)
    host = torch.empty((n, D), dtype=dtype, pin_memory=True)
    h = host.numpy()
    for i, c in enumerate(choices):
        for l in range(len(shapes)):
            h[i, seg[l]:seg[l + 1]] = np.asarray(local_grads[c][l]).reshape(-1)
    X = host.to(_device(), non_blocking=True)
    return StagedRound(X, seg, shapes, layer_dtypes, False)


def _np_dtype(a):
    if isinstance(a, torch.Tensor):
        return {torch.float64: np.float64, torch.float16: np.float16}.get(a.dtype, np.float32)
    return np.asarray(a).dtype


def _stage_dtype(agg, local_grads, choices):
    """fp64 staging only for the two stateful aggregators when their inputs are
    fp64 (they always are in the reference: momentum over np.zeros, :192-194)."""
    if agg not in _STATEFUL:
        return torch.float32
    c0 = int(choices[0])
    return torch.float64 if any(np.dtype(_np_dtype(t)) == np.float64 for t in local_grads[c0]) else torch.float32


# ---------------------------------------------------------------------------
# one round on the device: flat (D,) aggregate, or per-layer objects for Krum
# ---------------------------------------------------------------------------
def _device_round(agg, st, args, state, local_grads, choices):
    """Returns (flat device vector over D or None, per-layer Krum picks or None)."""
    X, seg = st.X, st.seg
    f = int(args.malnum)
    eps = args.malnum * 1. / args.nworker
    if agg == "average":
        return engine.average(X), None
    if agg == "median":
        return engine.median(X), None
    if agg == "trimmedmean":
        return engine.trimmed_mean(X), None
    if agg == "krum":
        orders = [engine.krum_select(st.cols(l), f, 1, scores=False)[0] for l in range(st.nlayers)]
        return None, torch.cat(orders)
    if agg == "clustering":
        out = torch.empty(seg[-1], dtype=torch.float32, device=X.device)
        for l in range(st.nlayers):
            out[seg[l]:seg[l + 1]] = engine.mom_krum(st.cols(l), f)[0]
        return out, None
    if agg in _BULYAN:
        out = torch.empty(seg[-1], dtype=torch.float64, device=X.device)
        status = torch.zeros(st.nlayers, dtype=torch.int32, device=X.device)
        for l in range(st.nlayers):
            out[seg[l]:seg[l + 1]] = engine.bulyan(st.cols(l), f, _BULYAN[agg], status=status[l:l + 1])
        if agg != "bulyankrum":   # one read back per round (robust_estimator.py:308, 321)
            engine.check_bulyan_status(status, "bulyan(%s)" % _BULYAN[agg])
        return out, None
    if agg in ("filterl2", "ex_noregret", "mom_filterl2", "mom_ex_noregret"):
        src = X
        if agg.startswith("mom_"):
            num, size = engine.mom_bucket_count(int(X.shape[0]), eps, np.exp(-50 + args.malnum))
            src = engine.bucket_means(X, size, num)
        fn = engine.filter_l2 if agg.endswith("filterl2") else engine.ex_noregret
        out = torch.empty(seg[-1], dtype=torch.float64, device=X.device)
        for l in range(st.nlayers):
            out[seg[l]:seg[l + 1]] = fn(src[:, seg[l]:seg[l + 1]], eps=eps, sigma=args.sigma)
        return out, None
    if agg == "iclr2022_bucketing":
        prev = state.prev
        width = int(args.perround) // int(args.buckets)
        W = engine.window_means(X, 1, width, int(args.buckets))
        out = engine.clipped_mean(W, prev, engine.clip_scales(W, prev, seg, args.tau))
        state.prev = out.clone()
        return out, None
    if agg == "icml2021_history":
        prev = state.prev
        clipped = torch.empty((int(X.shape[0]), seg[-1]), dtype=torch.float64, device=X.device)
        out = engine.clipped_mean(X, prev, engine.clip_scales(X, prev, seg, args.tau), clipped=clipped)
        state.prev = out.clone()
        _write_back(local_grads, choices, st, clipped)
        return out, None
    raise ValueError("unknown aggregator %r (simulate.py:76 lists %s)" % (agg, ", ".join(AGG_NAMES)))


def _write_back(local_grads, choices, st, clipped):
    """simulate.py:380 stores the clipped float64 rows into local_grads."""
    store = getattr(local_grads, "store", None)
    if store is not None and store.intact(choices):
        store.store_rows([int(c) for c in choices], clipped)
        return
    if st.device_io:
        for i, c in enumerate(choices):
            for l in range(st.nlayers):
                local_grads[int(c)][l] = clipped[i, st.seg[l]:st.seg[l + 1]].view(st.shapes[l])
        return
    h = clipped.cpu().numpy()
    for i, c in enumerate(choices):
        for l in range(st.nlayers):
            local_grads[int(c)][l] = h[i, st.seg[l]:st.seg[l + 1]].reshape(st.shapes[l])


def _prepare(agg, local_grads, choices, state):
    if agg not in AGG_NAMES:
        raise ValueError("unknown aggregator %r (simulate.py:76 lists %s)" % (agg, ", ".join(AGG_NAMES)))
    if agg in _STATEFUL and state is None:
        raise ValueError("%s is stateful: pass a DispatchState that lives across rounds" % agg)
    first_call = agg in _STATEFUL and state.prev is None
    if first_call and agg == "iclr2022_bucketing":
        # simulate.py:338-342: on the first round `choices` is shuffled in place,
        # once per parameter tensor, by numpy's global RNG
        for _ in range(len(local_grads[int(choices[0])])):
            np.random.shuffle(choices)
    st = stage_round(local_grads, choices, _stage_dtype(agg, local_grads, choices))
    if first_call:
        state.prev = torch.zeros(st.seg[-1], dtype=torch.float64, device=st.X.device)
    return st


_OUT_KIND = {"average": "input", "median": "input", "trimmedmean": "input", "clustering": "input"}


def aggregate(agg, local_grads, choices, args, state=None):
    """One round of simulate.py:231-398: returns ``average_grad`` (one entry per
    layer).  ``local_grads[c][l]`` are numpy arrays or device tensors;
    ``choices`` is the round's client array (shuffled in place on the first
    iclr2022_bucketing round, like the reference)."""
    st = _prepare(agg, local_grads, choices, state)
    flat, picks = _device_round(agg, st, args, state, local_grads, choices)
    if picks is not None:   # Krum: the chosen client's own object per layer
        idx = picks.cpu().tolist()
        return [local_grads[int(choices[i])][l] for l, i in enumerate(idx)]
    if st.device_io:
        return [flat[st.seg[l]:st.seg[l + 1]].view(st.shapes[l]) for l in range(st.nlayers)]
    host = flat.cpu().numpy()
    res = []
    for l in range(st.nlayers):
        a = host[st.seg[l]:st.seg[l + 1]].reshape(st.shapes[l])
        if _OUT_KIND.get(agg) == "input":
            a = a.astype(st.layer_dtypes[l], copy=False)
        res.append(a)
    return res


def apply_update(params, average_grad):
    """simulate.py:400-404: params[idx].data.sub_(average_grad[idx])."""
    with torch.no_grad():
        for p, g in zip(params, average_grad):
            if not isinstance(g, torch.Tensor):
                g = torch.from_numpy(np.asarray(g))
            p.data.sub_(g.to(p.device))


def aggregate_flat(agg, local_grads, choices, args, state=None):
    """One round's aggregate as a flat (D,) device vector over all layers
    (Krum's per-layer picks gathered on the device); nothing leaves the GPU."""
    st = _prepare(agg, local_grads, choices, state)
    flat, picks = _device_round(agg, st, args, state, local_grads, choices)
    if picks is not None:
        flat = torch.empty(st.seg[-1], dtype=torch.float32, device=st.X.device)
        for l in range(st.nlayers):
            lo, hi = st.seg[l], st.seg[l + 1]
            engine.gather_rows(st.cols(l), picks[l:l + 1], out=flat[lo:hi].view(1, hi - lo))
    return flat, st


def aggregate_and_apply(agg, params, local_grads, choices, args, state=None):
    """Device-resident round: aggregate and subtract from ``params`` without the
    aggregate leaving the GPU (Krum's pick is gathered on the device too).
    Returns the per-layer device aggregates."""
    flat, st = aggregate_flat(agg, local_grads, choices, args, state)
    store = getattr(local_grads, "store", None)
    views = [flat[st.seg[l]:st.seg[l + 1]].view(st.shapes[l]) for l in range(st.nlayers)]
    params = list(params)
    if store is not None and len(params) == len(store.params) and all(a is b for a, b in zip(params, store.params)):
        store.apply(flat)          # one launch over the whole network (csrc/store.hip)
    else:
        apply_update(params, views)
    return views
