"""Device-level engine API: aggregators over a device-resident N x d fp32
matrix (client-major, row stride ``X.stride(0)``), launched on the current
HIP stream through libsra.so.

These are the building blocks behind the reference-compatible module
``robust_estimator`` (list-of-arrays in, array out) and behind ``bench.py``
(device-resident timing).  Nothing here synchronises the stream or touches the
host except where a data-dependent host decision is unavoidable (documented
per function).
"""
from __future__ import annotations

import torch

from . import _lib


def _stream_ptr(device=None):
    """hipStream_t of torch's current stream on ``device`` (as an int)."""
    return torch.cuda.current_stream(device).cuda_stream


def as_matrix(X):
    """Validate an (N, d) CUDA float32 matrix with unit column stride."""
    if not isinstance(X, torch.Tensor) or not X.is_cuda:
        raise TypeError("engine ops need a CUDA (HIP) tensor, got %r" % type(X))
    if X.dtype != torch.float32:
        raise TypeError("engine ops compute in float32, got %s" % X.dtype)
    if X.dim() != 2:
        raise ValueError("expected an (N, d) matrix, got shape %s" % (tuple(X.shape),))
    if X.shape[1] > 1 and X.stride(1) != 1:
        X = X.contiguous()
    n, d = X.shape
    ldx = X.stride(0) if n > 1 else d
    return X, int(n), int(d), int(max(ldx, d))


def _out(X, d, out):
    if out is None:
        return torch.empty(d, dtype=torch.float32, device=X.device)
    if out.dtype != torch.float32 or out.numel() < d or not out.is_contiguous():
        raise ValueError("out must be a contiguous float32 tensor with >= d elements")
    return out


def average(X, out=None):
    """Sequential-sum mean over clients (simulate.py:235-244)."""
    X, n, d, ldx = as_matrix(X)
    out = _out(X, d, out)
    _lib.call("sra_average_f32", X.data_ptr(), n, d, ldx, out.data_ptr(), _stream_ptr(X.device))
    return out


def median(X, out=None):
    """Coordinate-wise median, numpy semantics (robust_estimator.py:220-221)."""
    X, n, d, ldx = as_matrix(X)
    out = _out(X, d, out)
    _lib.call("sra_median_f32", X.data_ptr(), n, d, ldx, out.data_ptr(), _stream_ptr(X.device))
    return out


def trim_count(n, beta):
    """b = int(N * beta), evaluated in Python floats like robust_estimator.py:226."""
    return int(n * beta)


def trimmed_mean(X, beta=0.1, out=None):
    """Coordinate-wise trimmed mean (robust_estimator.py:223-232), bit-exact."""
    X, n, d, ldx = as_matrix(X)
    out = _out(X, d, out)
    _lib.call("sra_trimmed_mean_f32", X.data_ptr(), n, d, ldx, trim_count(n, beta), out.data_ptr(),
              _stream_ptr(X.device))
    return out
