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

import numpy as np
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
    X = _unit_rows(X)
    n, d = X.shape
    ldx = X.stride(0) if n > 1 else d
    return X, int(n), int(d), int(ldx)


def _unit_rows(X):
    """A view the kernels can walk as rows[i * ldx + j]: unit column stride and
    non-overlapping rows (ldx >= d).  Expanded (stride 0) or overlapping views
    (unfold / as_strided) would make the kernels read past the real storage,
    so they are copied."""
    n, d = X.shape
    if (d > 1 and X.stride(1) != 1) or (n > 1 and X.stride(0) < d):
        X = X.contiguous()
    return X


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


# ---------------------------------------------------------------------------
# pairwise L2 / Krum family
# ---------------------------------------------------------------------------
def _workspace(nbytes, device):
    """Caller-owned workspace (torch's caching allocator: no hipMalloc per call)."""
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def gram(X):
    """Centred Gram (N x N float64) of the client rows (k2, MFMA)."""
    X, n, d, ldx = as_matrix(X)
    G = torch.empty((n, n), dtype=torch.float64, device=X.device)
    nb = _lib.query_bytes("sra_gram_workspace_bytes", n, d)
    ws = _workspace(nb, X.device)
    _lib.call("sra_gram_f32", X.data_ptr(), n, d, ldx, G.data_ptr(), ws.data_ptr(), nb, _stream_ptr(X.device))
    return G


def krum_select(X, f, rounds=1, scores=True):
    """Run `rounds` Krum selections (f fixed) on device.

    Returns (order int32 tensor of length `rounds`, scores float32 tensor of
    the N round-0 scores or None).  No host synchronisation."""
    X, n, d, ldx = as_matrix(X)
    order = torch.empty(rounds, dtype=torch.int32, device=X.device)
    sc = torch.empty(n, dtype=torch.float32, device=X.device) if scores else None
    nb = _lib.query_bytes("sra_krum_workspace_bytes", n, d)
    ws = _workspace(nb, X.device)
    _lib.call("sra_krum_select_f32", X.data_ptr(), n, d, ldx, int(f), int(rounds), order.data_ptr(),
              sc.data_ptr() if sc is not None else None, ws.data_ptr(), nb, _stream_ptr(X.device))
    return order, sc


def krum_from_gram(G, f, rounds=1, scores=True):
    """Krum selections from a precomputed (e.g. all-reduced) Gram."""
    n = int(G.shape[0])
    order = torch.empty(rounds, dtype=torch.int32, device=G.device)
    sc = torch.empty(n, dtype=torch.float32, device=G.device) if scores else None
    nb = _lib.query_bytes("sra_krum_from_gram_workspace_bytes", n)
    ws = _workspace(nb, G.device)
    _lib.call("sra_krum_from_gram", G.contiguous().data_ptr(), n, int(f), int(rounds), order.data_ptr(),
              sc.data_ptr() if sc is not None else None, ws.data_ptr(), nb, _stream_ptr(G.device))
    return order, sc


def krum_pair_sq(X, bucket_size=1):
    """Class-coded sums of squared fp32 differences over X's columns (nb x nb
    float64, i < j; NaN / +inf where the reference's norm is NaN / inf) of the
    clients (bucket_size 1) or of the means of consecutive buckets: one
    shard's contribution to the sharded Krum family's exact route."""
    X, n, d, ldx = as_matrix(X)
    nb = -(-n // int(bucket_size))
    A = torch.empty((nb, nb), dtype=torch.float64, device=X.device)
    nbytes = _lib.query_bytes("sra_krum_pair_sq_workspace_bytes", n, int(bucket_size))
    ws = _workspace(nbytes, X.device)
    _lib.call("sra_krum_pair_sq_f32", X.data_ptr(), n, d, ldx, int(bucket_size), A.data_ptr(), ws.data_ptr(), nbytes,
              _stream_ptr(X.device))
    return A


def krum_from_pairs(A, f, rounds=1, scores=True):
    """Krum selections from (summed) krum_pair_sq sums: the exact route."""
    n = int(A.shape[0])
    order = torch.empty(rounds, dtype=torch.int32, device=A.device)
    sc = torch.empty(n, dtype=torch.float32, device=A.device) if scores else None
    nb = _lib.query_bytes("sra_krum_from_pairs_workspace_bytes", n)
    ws = _workspace(nb, A.device)
    _lib.call("sra_krum_from_pairs", A.contiguous().data_ptr(), n, int(f), int(rounds), order.data_ptr(),
              sc.data_ptr() if sc is not None else None, ws.data_ptr(), nb, _stream_ptr(A.device))
    return order, sc


def gather_rows(X, rows, out=None):
    """out[r] = X[rows[r]] with `rows` a device int32 tensor (no host sync)."""
    X, n, d, ldx = as_matrix(X)
    k = int(rows.numel())
    if out is None:
        out = torch.empty((k, d), dtype=torch.float32, device=X.device)
    _lib.call("sra_gather_rows_f32", X.data_ptr(), n, d, ldx, rows.data_ptr(), k, out.data_ptr(), out.stride(0),
              _stream_ptr(X.device))
    return out


def row_fault_count(reset=True):
    """Device row indices found outside their matrix (clamped) since the last
    reset (sra_row_fault_count); synchronous.  Non-zero means a bug."""
    import ctypes
    c = ctypes.c_uint32(0)
    _lib.call("sra_row_fault_count", int(bool(reset)), ctypes.byref(c))
    return int(c.value)


def krum(X, f):
    """Device Krum: (chosen row as a device copy (d,), order int32 tensor (1,))."""
    order, _ = krum_select(X, f, 1, scores=False)
    return gather_rows(X, order)[0], order


def bucket_means(X, bucket_size, nbuckets, out=None):
    """Means of consecutive buckets of clients (np.mean order), (B, d)."""
    X, n, d, ldx = as_matrix(X)
    if out is None:
        out = torch.empty((nbuckets, d), dtype=torch.float32, device=X.device)
    _lib.call("sra_bucket_mean_f32", X.data_ptr(), n, d, ldx, int(bucket_size), int(nbuckets), out.data_ptr(),
              out.stride(0), _stream_ptr(X.device))
    return out


MOM_KRUM_FUSED_MAX_BUCKETS = 192


def gram_buckets(X, bucket_size=3):
    """Centred Gram (B x B float64) of the means of consecutive buckets of
    clients, B = ceil(N / bucket_size): without writing the means up to 192
    buckets of at most 4 clients (sra_gram_buckets_f32), else the Gram of the
    materialised means (sra_bucket_mean_f32 + sra_gram_f32, B <= 8192)."""
    X, n, d, ldx = as_matrix(X)
    nb = -(-n // bucket_size)
    if not (1 <= bucket_size <= 4 and nb <= MOM_KRUM_FUSED_MAX_BUCKETS):
        return gram(bucket_means(X, bucket_size, nb))
    G = torch.empty((nb, nb), dtype=torch.float64, device=X.device)
    nbytes = _lib.query_bytes("sra_gram_workspace_bytes", nb, d)
    ws = _workspace(nbytes, X.device)
    _lib.call("sra_gram_buckets_f32", X.data_ptr(), n, d, ldx, int(bucket_size), G.data_ptr(), ws.data_ptr(), nbytes,
              _stream_ptr(X.device))
    return G


def mom_krum(X, f, bucket_size=3, fused=True):
    """robust_estimator.mom_krum on device: Krum over ceil(N/3) bucket means.
    Returns (the chosen bucket's mean row (d,), order int32 (1,) = its bucket).
    Up to 192 buckets of at most 4 clients the bucket means are never written
    (sra_mom_krum_f32); otherwise, or with fused=False, they are materialised
    (sra_bucket_mean_f32) and scored by krum()."""
    X, n, d, ldx = as_matrix(X)
    nb = -(-n // bucket_size)
    if fused and 1 <= bucket_size <= 4 and nb <= MOM_KRUM_FUSED_MAX_BUCKETS:
        out = torch.empty(d, dtype=torch.float32, device=X.device)
        order = torch.empty(1, dtype=torch.int32, device=X.device)
        nbytes = _lib.query_bytes("sra_mom_krum_workspace_bytes", n, d, int(bucket_size))
        ws = _workspace(nbytes, X.device)
        _lib.call("sra_mom_krum_f32", X.data_ptr(), n, d, ldx, int(f), int(bucket_size), order.data_ptr(),
                  out.data_ptr(), ws.data_ptr(), nbytes, _stream_ptr(X.device))
        return out, order
    B = bucket_means(X, bucket_size, nb)
    row, order = krum(B, f)
    return row, order


# ---------------------------------------------------------------------------
# Bulyan
# ---------------------------------------------------------------------------
BULYAN_MODES = {"krum": 0, "median": 1, "trimmedmean": 2}


def bulyan(X, f, aggsubfunc="trimmedmean", selected=False, check=True, status=None):
    """robust_estimator.bulyan on device: float64 (d,) aggregate.
    With selected=True also returns the theta chosen clients (krum mode).
    check=True reads the selection status back (one host synchronisation) and
    raises AssertionError where the reference's ``assert min_index != None``
    fails (robust_estimator.py:308, 321): a median / trimmed-mean round whose
    distances are all NaN / inf, e.g. bulyan(..., 'median') with a NaN client.
    Krum mode has no such assert and never reads back.  status: a device int32
    slot to write the status into instead (no read back: a caller running
    several layers checks them once with check_bulyan_status)."""
    X, n, d, ldx = as_matrix(X)
    if aggsubfunc not in BULYAN_MODES:
        raise ValueError("aggsubfunc must be one of %s" % sorted(BULYAN_MODES))
    mode = BULYAN_MODES[aggsubfunc]
    theta = n - 2 * int(f)
    out = torch.empty(d, dtype=torch.float64, device=X.device)
    sel = torch.empty(max(theta, 1), dtype=torch.int32, device=X.device) if selected else None
    own = status is None
    if own:
        status = torch.empty(1, dtype=torch.int32, device=X.device)
    nb = _lib.query_bytes("sra_bulyan_workspace_bytes", n, d, int(f), mode)
    ws = _workspace(nb, X.device)
    _lib.call("sra_bulyan_f32", X.data_ptr(), n, d, ldx, int(f), mode, out.data_ptr(),
              sel.data_ptr() if sel is not None else None, status.data_ptr(), ws.data_ptr(), nb,
              _stream_ptr(X.device))
    if own and check and mode != 0:
        check_bulyan_status(status, "bulyan(%s)" % aggsubfunc)
    return (out, sel) if selected else out


def check_bulyan_status(status, what="bulyan"):
    """One read back of the status slots of one or more Bulyan calls."""
    if int(status.max().item()) == 1:
        raise AssertionError("%s: a selection round found no finite distance (min_index is None)" % what)


def bulyan_round(X, rows, nr, aggsubfunc, agg, dist, dba=False):
    """One Bulyan selection round (median / trimmedmean) over rows[:nr] of a
    (shard of a) layer: fills agg (d float32) and dist (nr float64, squared
    distances over this block's columns).  No host synchronisation."""
    X, n, d, ldx = as_matrix(X)
    mode = BULYAN_MODES[aggsubfunc]
    nb = _lib.query_bytes("sra_bulyan_round_workspace_bytes", n, d)
    ws = _workspace(nb, X.device)
    _lib.call("sra_bulyan_round_f32", X.data_ptr(), n, d, ldx, rows.data_ptr(), int(nr), mode, int(bool(dba)),
              agg.data_ptr(), dist.data_ptr(), ws.data_ptr(), nb, _stream_ptr(X.device))


def bulyan_pick(dist, rows, nr, rows_next, status=None):
    """Remove the first strict minimum of dist[:nr] from rows[:nr] into rows_next."""
    _lib.call("sra_bulyan_pick", dist.data_ptr(), rows.data_ptr(), int(nr), rows_next.data_ptr(),
              status.data_ptr() if status is not None else None, _stream_ptr(dist.device))


def bulyan_stage(S, beta):
    """The per-coordinate Bulyan stage over the rows of a (theta, d) float32
    device matrix in selection order (robust_estimator.py:324-330): (d,)
    float64.  beta = theta - 2f (Python slice semantics when negative)."""
    S, theta, d, lds = as_matrix(S)
    out = torch.empty(d, dtype=torch.float64, device=S.device)
    nb = _lib.query_bytes("sra_bulyan_stage_workspace_bytes", theta, d)
    ws = _workspace(nb, S.device)
    _lib.call("sra_bulyan_stage_f32", S.data_ptr(), theta, d, lds, int(beta), out.data_ptr(), ws.data_ptr(), nb,
              _stream_ptr(S.device))
    return out


def bulyan_coordinates(A, beta, median_index=False, median_row=False):
    """The per-coordinate Bulyan stage over the columns of a (theta, d) float64
    device matrix (robust_estimator.py:259-275 for every column): returns the
    (d,) float64 means, plus the median indices (int64) and distance rows
    ((theta, d) float64) when asked."""
    if not isinstance(A, torch.Tensor) or not A.is_cuda or A.dtype != torch.float64 or A.dim() != 2:
        raise TypeError("bulyan_coordinates takes a (theta, d) float64 CUDA tensor")
    A = _unit_rows(A)
    theta, d = A.shape
    lda = A.stride(0) if theta > 1 else d
    out = torch.empty(d, dtype=torch.float64, device=A.device)
    mi = torch.empty(d, dtype=torch.int64, device=A.device) if median_index else None
    mr = torch.empty((theta, d), dtype=torch.float64, device=A.device) if median_row else None
    _lib.call("sra_bulyan_coordinate_f64", A.data_ptr(), int(theta), int(d), int(lda), int(beta), out.data_ptr(),
              mi.data_ptr() if mi is not None else None, mr.data_ptr() if mr is not None else None, int(d),
              _stream_ptr(A.device))
    return out, mi, mr

# ---------------------------------------------------------------------------
# spectral filters
# ---------------------------------------------------------------------------
ITV = 1000


def chunk_width(d, itv):
    """robust_estimator.py:116-117, 192-193: itv None -> floor(sqrt(d))."""
    if itv is None:
        import math
        return int(math.floor(math.sqrt(d)))
    return int(itv)


def _filter(X, mode, eps, sigma, expansion, itv, check, out=None, info=None):
    """info (a dict, optional): ``unweighted_chunks`` = the chunks whose result
    is ex_noregret's plain fp32 mean after an infeasible projection
    (projected_c = None, robust_estimator.py:99-101), ``chunks`` = all chunks
    (one host synchronisation)."""
    X, n, d, ldx = as_matrix(X)
    if out is None:
        out = torch.empty(d, dtype=torch.float64, device=X.device)
    elif out.dtype != torch.float64 or out.numel() != d or not out.is_contiguous() or out.device != X.device:
        raise ValueError("out must be a contiguous float64 (d,) tensor on X's device")
    status = torch.zeros(2, dtype=torch.int32, device=X.device)
    w = chunk_width(d, itv)
    nb = _lib.query_bytes("sra_filter_workspace_bytes", n, d, w)
    ws = _workspace(nb, X.device)
    _lib.call("sra_filter_f32", X.data_ptr(), n, d, ldx, int(mode), w, float(eps), float(sigma),
              float(expansion), out.data_ptr(), status.data_ptr(), ws.data_ptr(), nb, _stream_ptr(X.device))
    _filter_status(status, mode, check, info, d, w)
    return out


def _filter_status(status, mode, check, info, d, w):
    if check or info is not None:
        st = status.cpu().tolist()
        if check and st[0] == 2:
            raise TypeError("ex_noregret: no feasible capped-simplex projection (projected_c is None), and the "
                            "next (unweighted) iteration does not exit: unsupported operand type(s) for *: "
                            "'NoneType' and 'float'")
        if info is not None:
            info["unweighted_chunks"] = int(st[1])
            info["chunks"] = -(-d // w)


FILTER_TRACE_STRIDE = 1 + 2 * 128


def filter_trace(X, mode, eps, sigma, expansion, itv):
    """Run a filter (mode 0 filterL2, 1 ex_noregret) and return (out, trace):
    trace is a host int32 (nchunks, 1 + 2n) array [iterations completed,
    decision per iteration (-1 unused), active flag per client] -- the layout
    of oracle.robust_np.trace_array (sra_filter_trace_f32, include/sra.h)."""
    X, n, d, ldx = as_matrix(X)
    out = torch.empty(d, dtype=torch.float64, device=X.device)
    status = torch.zeros(2, dtype=torch.int32, device=X.device)
    w = chunk_width(d, itv)
    nch = -(-d // w)
    half = max(n, 128)   # rows of 1 + 2 max(N, 128) int32 (include/sra.h)
    tr = torch.full((nch, 1 + 2 * half), -1, dtype=torch.int32, device=X.device)
    nb = _lib.query_bytes("sra_filter_workspace_bytes", n, d, w)
    ws = _workspace(nb, X.device)
    _lib.call("sra_filter_trace_f32", X.data_ptr(), n, d, ldx, int(mode), w, float(eps), float(sigma),
              float(expansion), out.data_ptr(), status.data_ptr(), tr.data_ptr(), ws.data_ptr(), nb,
              _stream_ptr(X.device))
    tr = tr.cpu().numpy()
    return out, np.concatenate([tr[:, :1 + n], tr[:, 1 + half:1 + half + n]], axis=1)


FILTER_DEBUG_DOUBLES = 128 * 128 + 256 * 144


def filter_debug(X, mode, eps, sigma, expansion, itv):
    """Run a filter and return (out, G0, records) for chunk 0: G0 the centred
    chunk Gram (n x n fp64), records an (iters, 144) array of [weights(128),
    lambda, lanczos_steps, ritz_residual, checks, active, w'Gw, restarts,
    second_gs_passes, cycles, 7 unused]."""
    X, n, d, ldx = as_matrix(X)
    out = torch.empty(d, dtype=torch.float64, device=X.device)
    status = torch.zeros(2, dtype=torch.int32, device=X.device)
    dbg = torch.full((FILTER_DEBUG_DOUBLES,), float("nan"), dtype=torch.float64, device=X.device)
    w = chunk_width(d, itv)
    nb = _lib.query_bytes("sra_filter_workspace_bytes", n, d, w)
    ws = _workspace(nb, X.device)
    _lib.call("sra_filter_debug_f32", X.data_ptr(), n, d, ldx, int(mode), w, float(eps),
              float(sigma), float(expansion), out.data_ptr(), status.data_ptr(), dbg.data_ptr(),
              ws.data_ptr(), nb, _stream_ptr(X.device))
    dbg = dbg.cpu()
    G = dbg[:128 * 128].reshape(128, 128)[:n, :n].clone()
    recs = dbg[128 * 128:].reshape(256, 144)
    return out, G, recs


def filter_l2(X, eps=0.2, sigma=1, expansion=20, itv=ITV, check=True, out=None):
    """robust_estimator.filterL2 on device: float64 (d,) (into ``out`` when given)."""
    return _filter(X, 0, eps, sigma, expansion, itv, check, out)


def ex_noregret(X, eps=1. / 12, sigma=1, expansion=20, itv=ITV, check=True, out=None, info=None):
    """robust_estimator.ex_noregret on device: float64 (d,) (into ``out`` when given)."""
    return _filter(X, 1, eps, sigma, expansion, itv, check, out, info)


def mom_bucket_count(n, eps, delta):
    """robust_estimator.py:136-137 / 211-212, evaluated with numpy's float64
    floor/log/ceil exactly as the reference (int() truncates a log(1/delta)
    that lands one ulp below an integer)."""
    import numpy as np
    num = int(np.floor(eps * n) + np.log(1. / delta))
    size = int(np.ceil(n * 1. / num))
    return num, size


def _mom_filter(X, mode, eps, sigma, expansion, itv, delta, check, out, info=None):
    """The MoM forms (robust_estimator.py:135-142, 210-218): up to 128 buckets
    in one call whose chunk-Gram loads form the bucket means (sra_mom_filter_f32,
    the bucket matrix never written whole); more buckets through the bucket
    kernel and the N > 128 filter."""
    n = int(X.shape[0])
    num, size = mom_bucket_count(n, eps, delta)
    if num > 128:
        return _filter(bucket_means(X, size, num), mode, eps, sigma, expansion, itv, check, out, info)
    X, n, d, ldx = as_matrix(X)
    if out is None:
        out = torch.empty(d, dtype=torch.float64, device=X.device)
    elif out.dtype != torch.float64 or out.numel() != d or not out.is_contiguous() or out.device != X.device:
        raise ValueError("out must be a contiguous float64 (d,) tensor on X's device")
    status = torch.zeros(2, dtype=torch.int32, device=X.device)
    w = chunk_width(d, itv)
    nb = _lib.query_bytes("sra_mom_filter_workspace_bytes", num, d, w)
    ws = _workspace(nb, X.device)
    _lib.call("sra_mom_filter_f32", X.data_ptr(), n, d, ldx, int(mode), w, int(size), int(num), float(eps),
              float(sigma), float(expansion), out.data_ptr(), status.data_ptr(), ws.data_ptr(), nb,
              _stream_ptr(X.device))
    _filter_status(status, mode, check, info, d, w)
    return out


def mom_filter_l2(X, eps=0.2, sigma=1, expansion=20, itv=ITV, delta=2.718281828459045 ** -30, check=True,
                  out=None):
    return _mom_filter(X, 0, eps, sigma, expansion, itv, delta, check, out)


def mom_ex_noregret(X, eps=0.2, sigma=1, expansion=20, itv=ITV, delta=2.718281828459045 ** -30, check=True,
                    out=None, info=None):
    return _mom_filter(X, 1, eps, sigma, expansion, itv, delta, check, out, info)


# ---------------------------------------------------------------------------
# cross-layer-norm clipping (k7): iclr2022_bucketing / icml2021_history
# ---------------------------------------------------------------------------
_SUFFIX = {torch.float32: "f32", torch.float64: "f64"}


def as_rows(X):
    """Validate an (k, d) CUDA float32/float64 matrix with unit column stride."""
    if not isinstance(X, torch.Tensor) or not X.is_cuda:
        raise TypeError("engine ops need a CUDA (HIP) tensor, got %r" % type(X))
    if X.dtype not in _SUFFIX:
        raise TypeError("clipping ops take float32 or float64 rows, got %s" % X.dtype)
    if X.dim() != 2:
        raise ValueError("expected a (k, d) matrix, got shape %s" % (tuple(X.shape),))
    X = _unit_rows(X)
    k, d = X.shape
    ld = X.stride(0) if k > 1 else d
    return X, int(k), int(d), int(ld)


def window_means(X, stride, width, nwin, out=None):
    """out[w] = mean of rows [w*stride, min(w*stride+width, N)) in X's precision
    (sequential sum / count, numpy's np.average(axis=0)); (nwin, d)."""
    X, n, d, ldx = as_rows(X)
    if out is None:
        out = torch.empty((nwin, d), dtype=X.dtype, device=X.device)
    _lib.call("sra_window_mean_" + _SUFFIX[X.dtype], X.data_ptr(), n, d, ldx, int(stride), int(width), int(nwin),
              out.data_ptr(), out.stride(0), _stream_ptr(X.device))
    return out


def _seg_table(seg, d):
    import ctypes
    seg = [int(s) for s in seg] if seg is not None else [0, d]
    arr = (ctypes.c_int64 * len(seg))(*seg)
    return arr, len(seg) - 1


def clip_scales(M, prev, seg, tau, norms=False, running=False):
    """scale[r] = min(1, tau / ||M[r] - prev||) with the norm across the layer
    segments ``seg`` (offsets, host ints) as simulate.py:352-356 / 374-378
    evaluate it.  Returns the (k,) fp64 device tensor (and the norms).
    running=True: the DBA harness's rule instead, norm = sqrt(norm + ||layer||^2)
    after every layer (src/DBA/helper.py:753-759)."""
    M, k, d, ldm = as_rows(M)
    prev = prev.reshape(-1)
    if prev.dtype != torch.float64 or prev.numel() != d or not prev.is_contiguous():
        raise ValueError("prev must be a contiguous float64 vector of d elements")
    arr, nseg = _seg_table(seg, d)
    nb = _lib.query_bytes("sra_clip_workspace_bytes", k, arr, nseg)
    ws = _workspace(nb, M.device)
    scale = torch.empty(k, dtype=torch.float64, device=M.device)
    nrm = torch.empty(k, dtype=torch.float64, device=M.device) if norms else None
    if running and M.dtype != torch.float32:
        raise TypeError("the running-norm (DBA) clip rule takes float32 rows")
    fn = "sra_clip_scale_running_f32" if running else "sra_clip_scale_" + _SUFFIX[M.dtype]
    _lib.call(fn, M.data_ptr(), k, d, ldm, prev.data_ptr(), arr, nseg, float(tau),
              scale.data_ptr(), nrm.data_ptr() if nrm is not None else None, ws.data_ptr(), nb,
              _stream_ptr(M.device))
    return (scale, nrm) if norms else scale


def clipped_mean(M, prev, scale, clipped=None, out=None):
    """out = mean_r (M[r] - prev) * scale[r] in fp64 (sequential over r); the
    clipped rows are written to ``clipped`` ((k, d) fp64) when given."""
    M, k, d, ldm = as_rows(M)
    prev = prev.reshape(-1)
    if out is None:
        out = torch.empty(d, dtype=torch.float64, device=M.device)
    ldc = 0
    if clipped is not None:
        if clipped.dtype != torch.float64 or tuple(clipped.shape) != (k, d) or clipped.stride(1) != 1:
            raise ValueError("clipped must be a (k, d) float64 matrix with unit column stride")
        ldc = clipped.stride(0) if k > 1 else d
    _lib.call("sra_clipped_mean_" + _SUFFIX[M.dtype], M.data_ptr(), k, d, ldm, prev.data_ptr(), scale.data_ptr(),
              clipped.data_ptr() if clipped is not None else None, ldc, out.data_ptr(), _stream_ptr(M.device))
    return out


def bucketing(X, prev, seg, buckets, tau):
    """iclr2022_bucketing (simulate.py:343-364) over the rows of X, already in
    (shuffled) choices order: overlapping windows X[b : b + N//buckets], clip
    each window mean against prev by its cross-layer norm, mean over windows."""
    n = int(X.shape[0])
    W = window_means(X, 1, n // int(buckets), int(buckets))
    return clipped_mean(W, prev, clip_scales(W, prev, seg, tau))


def history(X, prev, seg, tau, clipped=None):
    """icml2021_history (simulate.py:374-386): clip every row against prev by
    its cross-layer norm (written to ``clipped`` when given), mean over rows."""
    return clipped_mean(X, prev, clip_scales(X, prev, seg, tau), clipped=clipped)


# ---------------------------------------------------------------------------
# DBA harness primitives (k10, src/DBA/helper.py)
# ---------------------------------------------------------------------------
def order_stat(X, k, out=None):
    """s_k of every column (ascending; a NaN anywhere gives NaN).  k = (N-1)//2
    is torch.median's lower median (helper.py:561)."""
    X, n, d, ldx = as_matrix(X)
    out = _out(X, d, out)
    _lib.call("sra_order_stat_f32", X.data_ptr(), n, d, ldx, int(k), out.data_ptr(), _stream_ptr(X.device))
    return out


def rows_sum_div(X, divisor, out=None):
    """(sequential fp32 sum of the rows of X) / divisor, torch's in-place
    ``+=`` then ``/=`` rounding (helper.py:859-863, 1157-1163)."""
    X, n, d, ldx = as_matrix(X)
    out = _out(X, d, out)
    _lib.call("sra_rows_sum_div_f32", X.data_ptr(), n, d, ldx, float(divisor), out.data_ptr(), _stream_ptr(X.device))
    return out


def weighted_sum(X, w, out=None):
    """sum_r fl32(w[r] * X[r]) accumulated in row order (helper.py:1212-1219);
    ``w`` a device float32 vector of N weights."""
    X, n, d, ldx = as_matrix(X)
    if w.dtype != torch.float32 or w.numel() != n or not w.is_cuda:
        raise ValueError("w must be a device float32 vector of N weights")
    w = w.contiguous()
    out = _out(X, d, out)
    _lib.call("sra_weighted_sum_f32", X.data_ptr(), n, d, ldx, w.data_ptr(), out.data_ptr(), _stream_ptr(X.device))
    return out


def bulyan_dba(X, f, aggsubfunc="trimmedmean", selected=False, check=True, status=None):
    """Helper.bulyan_krum / bulyan_median / bulyan_trimmed_mean selection rules
    (helper.py:942-1137) with the shared per-coordinate stage; float64 (d,).
    check=True raises AssertionError where helper.py's ``assert min_index !=
    None`` fails (:1047, :1119): a round whose distances are all NaN / inf.
    status: as for bulyan()."""
    X, n, d, ldx = as_matrix(X)
    if aggsubfunc not in BULYAN_MODES:
        raise ValueError("aggsubfunc must be one of %s" % sorted(BULYAN_MODES))
    mode = BULYAN_MODES[aggsubfunc]
    theta = n - 2 * int(f)
    out = torch.empty(d, dtype=torch.float64, device=X.device)
    sel = torch.empty(max(theta, 1), dtype=torch.int32, device=X.device) if selected else None
    own = status is None
    if own:
        status = torch.empty(1, dtype=torch.int32, device=X.device)
    nb = _lib.query_bytes("sra_bulyan_workspace_bytes", n, d, int(f), mode)
    ws = _workspace(nb, X.device)
    _lib.call("sra_bulyan_dba_f32", X.data_ptr(), n, d, ldx, int(f), mode, out.data_ptr(),
              sel.data_ptr() if sel is not None else None, status.data_ptr(), ws.data_ptr(), nb,
              _stream_ptr(X.device))
    if own and check and mode != 0:
        check_bulyan_status(status, "bulyan_dba(%s)" % aggsubfunc)
    return (out, sel) if selected else out
