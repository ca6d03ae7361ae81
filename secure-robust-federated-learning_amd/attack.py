"""The attack-side callers of the aggregation path on the MI355X
(src/attack.py), with the reference's names, arguments
and in-place semantics:

* ``attack_krum(network, local_grads, mal_index, param_index, lower_bound=1e-8,
  upper_bound=1e-3)``  (attack.py:202-262, called per layer at simulate.py:224-225)
* ``attack_trimmedmean(network, local_grads, mal_index, b=2)``  (attack.py:157-198,
  simulate.py:220 with b=1.5)
* ``attack_xie(local_grads, weight, choices, mal_index)``  (attack.py:362-372)
* ``bulyan_attack_krum(network, local_grads, mal_index, param_index, lower_bound=1e-8,
  upper_bound=1e-3, target_layer=0, target_idx=0)``  (attack.py:264-308; defined
  by the reference but not called by simulate.py)

Each mutates ``local_grads`` in place and returns it, like the reference.  The
d-dependent work runs in libsra.so (csrc/attack.hip); ``local_grads`` entries
may be numpy arrays (staged through pinned memory) or CUDA tensors (results
stay on the device).  attack_trimmedmean draws from Python's ``random`` module
exactly as the reference's per-element ``random.uniform`` calls do: the
Mersenne Twister stream is generated on the device from ``random.getstate()``
and the module's state is advanced to where the reference would leave it.
"""
from __future__ import annotations

import random

import numpy as np
import torch

from . import _lib, engine


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("srfl_amd.attack needs an MI355X (HIP device); no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _on_device(a):
    return isinstance(a, torch.Tensor) and a.is_cuda


def _stack(arrays, dtype, dev):
    """(len(arrays), numel) matrix of the flattened arrays on the device."""
    if all(_on_device(a) for a in arrays):
        return torch.stack([a.reshape(-1).to(dtype) for a in arrays])
    n = int(np.prod(np.shape(arrays[0]), dtype=np.int64))
    host = torch.empty((len(arrays), n), dtype=dtype, pin_memory=True)
    h = host.numpy()
    for i, a in enumerate(arrays):
        h[i] = (a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)).reshape(-1)
    return host.to(dev, non_blocking=True)


def _i32(values, dev):
    return torch.tensor(list(values), dtype=torch.int32, device=dev)


def _emit(flat, shape, like_device):
    """A result layer in the caller's convention (device tensor or numpy)."""
    if like_device:
        return flat.reshape(shape).clone()
    return flat.reshape(shape).cpu().numpy()


# ---------------------------------------------------------------------------
# attack_krum
# ---------------------------------------------------------------------------
def attack_krum_layer(X, mal_mask, benign_rows, lower_bound=1e-8):
    """Device core of attack_krum for one layer: X (m, d) float32 CUDA matrix of
    all clients, ``mal_mask`` / ``benign_rows`` int32 CUDA tensors.  Returns
    (malicious layer value (d,) float64, lambda (1,) float64, krum's pick (1,)
    int32), all on the device, no host synchronisation."""
    X, m, d, ldx = engine.as_matrix(X)
    nb = _lib.query_bytes("sra_attack_krum_workspace_bytes", m, d, float(lower_bound))
    ws = engine._workspace(nb, X.device)
    row = torch.empty(d, dtype=torch.float64, device=X.device)
    lam = torch.empty(1, dtype=torch.float64, device=X.device)
    pick = torch.empty(1, dtype=torch.int32, device=X.device)
    _lib.call("sra_attack_krum_f32", X.data_ptr(), m, d, ldx, mal_mask.data_ptr(), benign_rows.data_ptr(),
              int(benign_rows.numel()), float(lower_bound), row.data_ptr(), lam.data_ptr(), pick.data_ptr(),
              ws.data_ptr(), nb, engine._stream_ptr(X.device))
    return row, lam, pick


def attack_krum(network, local_grads, mal_index, param_index, lower_bound=1e-8, upper_bound=1e-3):
    """attack.py:202-262.  ``network`` and ``upper_bound`` are accepted for the
    reference's signature; the reference reads only the layer shape from the
    former and overwrites the latter with 1.0 (:237)."""
    m = len(local_grads)
    mal = {int(i) for i in mal_index}
    benign = [c for c in range(m) if c not in mal]
    layer = [local_grads[c][param_index] for c in range(m)]
    shape = tuple(np.shape(layer[0]))
    dev_io = _on_device(layer[0])
    if not mal:
        return local_grads            # the loop runs, but there is no row to write
    if not benign:
        # average_sign = sign(zeros): every row is -lambda * 0, krum picks row 0 at lambda = 1
        for kk in mal_index:
            z = -1.0 * np.zeros(shape)
            local_grads[kk][param_index] = torch.from_numpy(z).to(layer[0].device) if dev_io else z
        return local_grads
    dev = layer[0].device if dev_io else _device()
    X = _stack(layer, torch.float32, dev)
    mask = _i32((1 if c in mal else 0 for c in range(m)), dev)
    row, _, _ = attack_krum_layer(X, mask, _i32(benign, dev), lower_bound)
    for kk in mal_index:
        local_grads[kk][param_index] = _emit(row, shape, dev_io)
    return local_grads


def bulyan_attack_krum(network, local_grads, mal_index, param_index, lower_bound=1e-8, upper_bound=1e-3,
                       target_layer=0, target_idx=0):
    """attack.py:264-308: attack_krum's lambda search with the direction
    attack_vec[param_index] in place of the benign sign: ones when
    ``param_index == target_idx`` and ``target_layer`` indexes a benign client
    (the reference adds 1 once, for the loop's c == target_layer), zeros
    otherwise.  The malicious rows become -lambda * attack_vec[param_index]
    (float64).  ``network`` gives the layer's shape; ``upper_bound`` is
    overwritten with 1.0 by the reference (:286)."""
    m = len(local_grads)
    mal = {int(i) for i in mal_index}
    benign = [c for c in range(m) if c not in mal]
    params = [p.data if hasattr(p, "data") else p for p in network.parameters()]
    shape = tuple(params[param_index].shape)
    ones = param_index == target_idx and 0 <= int(target_layer) < len(benign)
    layer = [local_grads[c][param_index] for c in range(m)]
    dev_io = _on_device(layer[0])
    if not mal:
        return local_grads            # the loop runs, but there is no row to write
    if not benign:
        # attack_vec is all zeros: every row is -lambda * 0, krum picks row 0 at lambda = 1
        for kk in mal_index:
            z = -1.0 * np.zeros(shape)
            local_grads[kk][param_index] = torch.from_numpy(z).to(layer[0].device) if dev_io else z
        return local_grads
    dev = layer[0].device if dev_io else _device()
    X = _stack(layer, torch.float32, dev)
    Xm, mm, d, ldx = engine.as_matrix(X)
    direction = (torch.ones if ones else torch.zeros)(d, dtype=torch.float32, device=dev)
    mask = _i32((1 if c in mal else 0 for c in range(m)), dev)
    rows = _i32(benign, dev)
    nb = _lib.query_bytes("sra_attack_krum_workspace_bytes", mm, d, float(lower_bound))
    ws = engine._workspace(nb, dev)
    row = torch.empty(d, dtype=torch.float64, device=dev)
    lam = torch.empty(1, dtype=torch.float64, device=dev)
    pick = torch.empty(1, dtype=torch.int32, device=dev)
    _lib.call("sra_attack_krum_dir_f32", Xm.data_ptr(), mm, d, ldx, mask.data_ptr(), rows.data_ptr(),
              int(rows.numel()), direction.data_ptr(), float(lower_bound), row.data_ptr(), lam.data_ptr(),
              pick.data_ptr(), ws.data_ptr(), nb, engine._stream_ptr(dev))
    for kk in mal_index:
        local_grads[kk][param_index] = _emit(row, shape, dev_io)
    return local_grads


# ---------------------------------------------------------------------------
# attack_trimmedmean
# ---------------------------------------------------------------------------
def mt19937_words(state, nwords, device):
    """Python ``random`` stream on the device: ``state`` = random.getstate()[1]
    (624 words + position).  Returns (words (nwords,) uint32 bits in an int32
    tensor, the advanced state tuple for random.setstate)."""
    st = torch.from_numpy(np.asarray(state, dtype=np.uint32).view(np.int32).copy()).to(device)
    words = torch.empty(max(int(nwords), 1), dtype=torch.int32, device=device)
    st_out = torch.empty(625, dtype=torch.int32, device=device)
    _lib.call("sra_mt19937_words", st.data_ptr(), int(nwords), words.data_ptr(), st_out.data_ptr(),
              engine._stream_ptr(device))
    new_state = tuple(int(v) for v in st_out.cpu().numpy().view(np.uint32))
    return words[:nwords], new_state


def attack_trimmedmean(network, local_grads, mal_index, b=2):
    """attack.py:157-198: every malicious client's update becomes
    ``p - u`` with ``u`` drawn per element between the benign extreme of
    ``p - x`` and ``b`` times it (the side chosen by the sign of the benign
    sum); ``p`` = the network's current parameters."""
    m = len(local_grads)
    mal = {int(i) for i in mal_index}
    benign = [c for c in range(m) if c not in mal]
    if not benign:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    params = [p.data if hasattr(p, "data") else p for p in network.parameters()]
    shapes = [tuple(p.shape) for p in params]
    sizes = [int(np.prod(s, dtype=np.int64)) for s in shapes]
    seg = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(seg[-1])
    dev_io = _on_device(local_grads[benign[0]][0])
    dev = local_grads[benign[0]][0].device if dev_io else _device()
    X = _stack([_flat_client(local_grads[c]) for c in benign], torch.float32, dev)
    P = torch.cat([p.detach().reshape(-1).to(device=dev, dtype=torch.float32) for p in params])
    version, internal, gauss_next = random.getstate()
    words, new_state = mt19937_words(internal, 2 * D, dev)
    out = torch.empty(D, dtype=torch.float64, device=dev)
    rows = _i32(range(len(benign)), dev)
    _lib.call("sra_attack_trimmedmean_f32", X.data_ptr(), D, int(X.stride(0)), rows.data_ptr(), len(benign),
              P.data_ptr(), words.data_ptr(), float(b), out.data_ptr(), engine._stream_ptr(dev))
    random.setstate((version, new_state, gauss_next))
    for c in mal_index:
        for idx in range(len(shapes)):
            local_grads[c][idx] = _emit(out[seg[idx]:seg[idx + 1]], shapes[idx], dev_io)
    return local_grads


def _flat_client(layers):
    if all(_on_device(t) for t in layers):
        return torch.cat([t.reshape(-1).to(torch.float32) for t in layers])
    return np.concatenate([(t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)).reshape(-1)
                           .astype(np.float32, copy=False) for t in layers])


# ---------------------------------------------------------------------------
# attack_xie
# ---------------------------------------------------------------------------
def attack_xie(local_grads, weight, choices, mal_index):
    """attack.py:362-372: every malicious client gets the SAME list object
    ``[-weight * sum_{benign chosen} local_grads[j][i] / len(choices)]``."""
    mal = {int(i) for i in mal_index}
    rows_idx = [int(j) for j in choices if int(j) not in mal]
    attack_vec = []
    for i, pp in enumerate(local_grads[0]):
        dev_io = _on_device(pp)
        dev = pp.device if dev_io else _device()
        is64 = (pp.dtype == torch.float64) if isinstance(pp, torch.Tensor) else np.asarray(pp).dtype == np.float64
        dt = torch.float64 if is64 else torch.float32
        shape = tuple(np.shape(pp))
        d = int(np.prod(shape, dtype=np.int64))
        if rows_idx:
            X = _stack([local_grads[j][i] for j in rows_idx], dt, dev)
            ldx = int(X.stride(0))
        else:
            X = torch.zeros((1, d), dtype=dt, device=dev)
            ldx = d
        out = torch.empty(d, dtype=dt, device=dev)
        rows = _i32(range(len(rows_idx)), dev) if rows_idx else torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("sra_attack_xie_f64" if is64 else "sra_attack_xie_f32", X.data_ptr(), d, ldx, rows.data_ptr(),
                  len(rows_idx), float(weight), len(choices), out.data_ptr(), engine._stream_ptr(dev))
        attack_vec.append(_emit(out, shape, dev_io))
    for i in mal_index:
        local_grads[i] = attack_vec
    return local_grads
