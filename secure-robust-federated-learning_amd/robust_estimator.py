"""Drop-in replacement of the reference module ``robust_estimator``
(src/robust_estimator.py), computed on the MI355X by libsra.

Same names, signatures, defaults and return types as the reference (SURVEY.md
§8(b)).  ``samples`` may be

* a list of same-shape numpy arrays (the reference's calling convention,
  simulate.py:277-279): results come back as numpy arrays of the layer shape
  in the dtype numpy would return;
* a list of torch tensors, or one (N, *shape) torch tensor, on the GPU: the
  result stays on the GPU as a torch tensor (no host round trip).

Arithmetic is fp32 on the device.  Inputs numpy promotes to float64 (an
attack's float64 rows, reference src/attack.py:197,260) are computed in fp32
and returned as float64 (tolerance stated in DESIGN.md).
"""
from __future__ import annotations

import numpy as np
import torch

from . import engine

ITV = 1000        # reference robust_estimator.py:40
MAX_ITER = 100    # reference robust_estimator.py:39


class _Staged:
    """An (N, D) float32 device matrix plus what is needed to hand results back."""

    def __init__(self, X, shape, np_dtype, device_io, n):
        self.X = X
        self.shape = shape
        self.np_dtype = np_dtype
        self.device_io = device_io
        self.n = n

    def result(self, vec, dtype=None):
        """Return a flat device vector in the caller's convention."""
        if self.device_io:
            return vec.reshape(self.shape)
        out = vec.detach().to("cpu").numpy().reshape(self.shape)
        want = dtype if dtype is not None else self.np_dtype
        return out.astype(want, copy=False)


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("srfl_amd.robust_estimator needs an MI355X (HIP device); no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _stage(samples):
    """Stack the caller's samples into one (N, D) float32 device matrix."""
    if isinstance(samples, torch.Tensor):
        if samples.dim() < 1:
            raise ValueError("samples must have a leading client axis")
        n = samples.shape[0]
        shape = tuple(samples.shape[1:])
        X = samples.reshape(n, -1)
        device_io = samples.is_cuda
        if not device_io:
            X = X.to(_device())
        return _Staged(X.to(torch.float32).contiguous(), shape, _np_dtype(samples.dtype), device_io, n)
    seq = list(samples)
    if not seq:
        raise ValueError("need at least one sample")
    if isinstance(seq[0], torch.Tensor):
        shape = tuple(seq[0].shape)
        X = torch.stack([t.reshape(-1) for t in seq])
        device_io = X.is_cuda
        if not device_io:
            X = X.to(_device())
        return _Staged(X.to(torch.float32).contiguous(), shape, _np_dtype(seq[0].dtype), device_io, len(seq))
    arr = np.array(seq)                       # the reference's own stacking (robust_estimator.py:224)
    n = arr.shape[0]
    shape = arr.shape[1:]
    res_dtype = np.result_type(arr.dtype, np.float32) if arr.dtype.kind != "f" else arr.dtype
    host = torch.empty((n, int(np.prod(shape, dtype=np.int64))), dtype=torch.float32, pin_memory=True)
    host.numpy()[...] = arr.reshape(n, -1)
    X = host.to(_device(), non_blocking=True)
    return _Staged(X, shape, res_dtype, False, n)


def _np_dtype(tdtype):
    return {torch.float64: np.float64, torch.float16: np.float16}.get(tdtype, np.float32)


# ---------------------------------------------------------------------------
# coordinate-wise
# ---------------------------------------------------------------------------
def median(samples):
    """robust_estimator.py:220-221 (np.median(samples, axis=0))."""
    st = _stage(samples)
    return st.result(engine.median(st.X))


def trimmed_mean(samples, beta=0.1):
    """robust_estimator.py:223-232."""
    st = _stage(samples)
    return st.result(engine.trimmed_mean(st.X, beta))


def average(samples):
    """The inline ``--agg average`` of simulate.py:235-244 (np.average(axis=0))."""
    st = _stage(samples)
    return st.result(engine.average(st.X))


# ---------------------------------------------------------------------------
# Krum family
# ---------------------------------------------------------------------------
def krum_(samples, f):
    """robust_estimator.py:234-244: the list of per-client Krum scores."""
    st = _stage(samples)
    _, scores = engine.krum_select(st.X, f, 1, scores=True)
    if st.device_io:
        return scores
    # numpy returns float64 metrics for float64 rows (an attack's promoted rows,
    # attack.py:197/260); the distances themselves are the fp32 Gram route's
    # (near-tie picks can differ from float64 BLAS norms)
    typ = np.dtype(st.np_dtype).type
    return [typ(v) for v in scores.cpu().numpy()]


def krum(samples, f):
    """robust_estimator.py:246-249: (the chosen sample itself, its index).
    Like the reference, the returned array IS the caller's object."""
    st = _stage(samples)
    order, _ = engine.krum_select(st.X, f, 1, scores=False)
    idx = int(order.cpu()[0])
    return samples[idx], idx


def mom_krum(samples, f, bucket_size=3):
    """robust_estimator.py:251-257 (``--agg clustering``)."""
    st = _stage(samples)
    row, _ = engine.mom_krum(st.X, f, bucket_size)
    return st.result(row)


# ---------------------------------------------------------------------------
# Bulyan
# ---------------------------------------------------------------------------
def _coord64(arr):
    """One coordinate's values as a (theta, 1) float64 device column; returns
    (column, device_io)."""
    if isinstance(arr, torch.Tensor):
        col = arr.reshape(-1, 1).to(dtype=torch.float64)
        io = arr.is_cuda
        return (col if io else col.to(_device())).contiguous(), io
    a = np.asarray(arr, dtype=np.float64).reshape(-1, 1)
    return torch.from_numpy(np.ascontiguousarray(a)).to(_device()), False


def bulyan_median(arr):
    """robust_estimator.py:259-270: (index of the value with the smallest total
    distance to the others -- np.argmin of numpy's pairwise row sums, the first
    NaN if any -- and that value's float64 distance row)."""
    col, io = _coord64(arr)
    _, mi, mr = engine.bulyan_coordinates(col, 0, median_index=True, median_row=True)
    if io:
        return mi[0], mr[:, 0]
    return np.int64(mi.cpu()[0]), mr[:, 0].cpu().numpy()


def bulyan_one_coordinate(arr, beta):
    """robust_estimator.py:272-275: mean of arr[np.argsort(distances)[:beta]]
    (Python slice semantics for beta < 0; equal distances take the smaller
    value first -- numpy's unstable argsort leaves that order undefined)."""
    col, io = _coord64(arr)
    out, _, _ = engine.bulyan_coordinates(col, int(beta))
    return out[0] if io else np.float64(out.cpu()[0])


def bulyan(grads, f, aggsubfunc="trimmedmean"):
    """robust_estimator.py:277-332 (float64 result, like the reference)."""
    st = _stage(grads)
    return st.result(engine.bulyan(st.X, f, aggsubfunc), dtype=np.float64)


# ---------------------------------------------------------------------------
# spectral filters
# ---------------------------------------------------------------------------
def filterL2_(samples, eps=0.2, sigma=1, expansion=20):
    """robust_estimator.py:144-177 on one (n, k) chunk."""
    st = _stage(samples)
    k = int(st.X.shape[1])
    return st.result(engine.filter_l2(st.X, eps, sigma, expansion, itv=k), dtype=np.float64)


def filterL2(samples, eps=0.2, sigma=1, expansion=20, itv=ITV):
    """robust_estimator.py:180-208."""
    st = _stage(samples)
    return st.result(engine.filter_l2(st.X, eps, sigma, expansion, itv), dtype=np.float64)


def mom_filterL2(samples, eps=0.2, sigma=1, expansion=20, itv=ITV, delta=np.exp(-30)):
    """robust_estimator.py:210-218."""
    st = _stage(samples)
    return st.result(engine.mom_filter_l2(st.X, eps, sigma, expansion, itv, delta), dtype=np.float64)


def _noregret_dtype(info):
    """The reference's result dtype: every chunk float64 (np.average with
    weights), except that a chunk whose projection was infeasible returns the
    plain float32 mean (robust_estimator.py:65, 101) -- np.concatenate keeps
    float32 only when every chunk did."""
    return np.float32 if info["chunks"] and info["unweighted_chunks"] == info["chunks"] else np.float64


def ex_noregret_(samples, eps=1. / 12, sigma=1, expansion=20, dis_threshold=0.7):
    """robust_estimator.py:42-102 on one (n, k) chunk."""
    st = _stage(samples)
    k = int(st.X.shape[1])
    info = {}
    out = engine.ex_noregret(st.X, eps, sigma, expansion, itv=k, info=info)
    return st.result(out, dtype=_noregret_dtype(info))


def ex_noregret(samples, eps=1. / 12, sigma=1, expansion=20, itv=ITV):
    """robust_estimator.py:104-133."""
    st = _stage(samples)
    info = {}
    out = engine.ex_noregret(st.X, eps, sigma, expansion, itv, info=info)
    return st.result(out, dtype=_noregret_dtype(info))


def mom_ex_noregret(samples, eps=0.2, sigma=1, expansion=20, itv=ITV, delta=np.exp(-30)):
    """robust_estimator.py:135-142."""
    st = _stage(samples)
    info = {}
    out = engine.mom_ex_noregret(st.X, eps, sigma, expansion, itv, delta, info=info)
    return st.result(out, dtype=_noregret_dtype(info))
