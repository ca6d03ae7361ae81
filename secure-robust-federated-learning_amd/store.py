"""Device-resident client updates: the step either side of the aggregation path
(src/simulate.py:127-131, 139-229, 400-404).

The reference keeps ``local_grads[c][idx]`` as host numpy arrays: every chosen
client trains on the GPU, then each layer's update crosses PCIe
(``params_copy[idx].data.cpu().numpy() - p.data.cpu().numpy()``, :193-194), the
aggregator restacks the layers on the host, and the aggregate crosses back
(``p.data.sub_(torch.from_numpy(avg).to(device))``, :400-404).

``ClientStore`` holds the same ``local_grads`` as ONE ``nworker x D`` device
matrix (D = all parameters, a segment table holds the layer offsets) and hands
out ``local_grads[c][idx]`` as views of its rows, so the reference's code that
reads ``local_grads`` (the attacks, the ``--agg`` dispatch) runs unchanged on
device tensors and nothing crosses PCIe:

* ``snapshot()``  -- params_copy (:146-148), one launch over the whole network;
* ``record(c)``   -- client c's update ``params_copy - params`` (or the momentum
  form of :187-191) written into row c, and the parameters restored (:196-199),
  one launch;
* ``dispatch.aggregate`` on ``store.local_grads`` stages the round with one
  row gather instead of a host stack + H2D;
* ``apply(flat)`` -- ``params -= aggregate`` (:400-404), one launch.

``fl_round`` strings these together like the body of simulate.py's round loop.
All arithmetic is in libsra.so (csrc/store.hip); there is no CPU path.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, engine


class StoreGrads(list):
    """``local_grads`` whose entries are views of a ``ClientStore``'s rows."""

    store = None


class ClientStore:
    """``local_grads`` for ``nworker`` clients of ``network`` on the device.

    ``momentum=True`` is the iclr2022_bucketing / icml2021_history form
    (simulate.py:187-191): rows are float64 (the reference's momentum is a
    float32 * float + float64 sum over ``np.zeros`` and stays float64); otherwise
    rows are float32 (the reference assigns the float32 difference, :193-194).
    Unwritten rows are zero, like ``np.zeros(p.data.shape)`` (:127-131)."""

    def __init__(self, params, nworker, momentum=False, beta=0.9):
        params = [p for p in params]
        if not params:
            raise ValueError("ClientStore needs at least one parameter tensor")
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError("ClientStore needs parameters on an MI355X (HIP) device; no CPU fallback")
        for p in params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                raise TypeError("ClientStore needs contiguous float32 parameters on one device")
        self.params = params
        self.device = dev
        self.nworker = int(nworker)
        self.momentum = bool(momentum)
        self.beta = float(beta)
        self.one_minus_beta = float(np.float32(1 - self.beta))
        self.shapes = [tuple(p.shape) for p in params]
        seg = [0]
        for p in params:
            seg.append(seg[-1] + p.numel())
        self.seg = seg
        self.D = seg[-1]
        self.dtype = torch.float64 if self.momentum else torch.float32
        self.U = torch.zeros((self.nworker, self.D), dtype=self.dtype, device=dev)
        self.snap = torch.empty(self.D, dtype=torch.float32, device=dev)
        self._seg_dev = torch.tensor(seg, dtype=torch.int64, device=dev)
        self._ptr_host = None
        self._ptrs = None
        self._views = [self._row_views(c) for c in range(self.nworker)]
        self.local_grads = StoreGrads(list(v) for v in self._views)
        self.local_grads.store = self

    # -- parameter table ----------------------------------------------------
    def _row_views(self, c):
        row = self.U[c]
        return [row[self.seg[l]:self.seg[l + 1]].view(self.shapes[l]) for l in range(len(self.shapes))]

    def _table(self):
        """Device array of the parameters' addresses, rebuilt if any moved."""
        ptrs = [p.data_ptr() for p in self.params]
        if ptrs != self._ptr_host:
            self._ptrs = torch.tensor(np.asarray(ptrs, dtype=np.uint64).view(np.int64), device=self.device)
            self._ptr_host = ptrs
        return self._ptrs.data_ptr(), self._seg_dev.data_ptr(), len(self.params), self.D

    def _stream(self):
        return engine._stream_ptr(self.device)

    # -- the round ----------------------------------------------------------
    def snapshot(self):
        """params_copy (simulate.py:146-148) as one flat float32 vector."""
        _lib.call("sra_params_flatten_f32", *self._table(), self.snap.data_ptr(), self._stream())
        return self.snap

    def record(self, c):
        """Client ``c`` finished local training: write its update into row c and
        restore the parameters from the snapshot (simulate.py:187-199)."""
        c = int(c)
        if not 0 <= c < self.nworker:
            raise IndexError("client %d out of range [0, %d)" % (c, self.nworker))
        row = self.U[c]
        if self.momentum:
            self._sync_row(c)   # the momentum reads local_grads[c] as the caller left it
            _lib.call("sra_record_momentum_f64", *self._table(), self.snap.data_ptr(), self.one_minus_beta,
                      self.beta, row.data_ptr(), self._stream())
        else:
            _lib.call("sra_record_delta_f32", *self._table(), self.snap.data_ptr(), row.data_ptr(), self._stream())
        # the reference assigns fresh arrays to local_grads[c][idx]
        self.local_grads[c] = list(self._views[c])

    def _sync_row(self, c):
        """Copy into row c any layer the caller replaced (an attack's output)."""
        cur = self.local_grads[c]
        for l, v in enumerate(self._views[c]):
            t = cur[l] if l < len(cur) else v
            if t is v:
                continue
            if not isinstance(t, torch.Tensor):
                t = torch.from_numpy(np.asarray(t))
            v.copy_(t.to(device=self.device, dtype=self.dtype).view(v.shape))

    def intact(self, choices):
        """True when ``local_grads[c]`` for every chosen c are still this
        store's row views (nothing replaced them since ``record``)."""
        for c in choices:
            cur = self.local_grads[int(c)]
            views = self._views[int(c)]
            if len(cur) != len(views) or any(a is not b for a, b in zip(cur, views)):
                return False
        return True

    def rows(self, choices):
        return torch.as_tensor(np.asarray(choices, dtype=np.int64), device=self.device)

    def stage(self, choices, dtype):
        """The round's (N, D) matrix: one gather of the chosen rows."""
        X = self.U.index_select(0, self.rows(choices))
        return X if X.dtype == dtype else X.to(dtype)

    def store_rows(self, choices, M):
        """local_grads[c] = M[i] for the i-th chosen client (icml2021_history's
        in-place clipping, simulate.py:380), keeping the views."""
        self.U.index_copy_(0, self.rows(choices), M.to(self.dtype))
        for c in choices:
            self.local_grads[int(c)] = list(self._views[int(c)])

    def apply(self, flat):
        """params -= flat (simulate.py:400-404) in one launch; ``flat`` is the
        (D,) float32 or float64 aggregate over all layers."""
        if flat.device != self.device or flat.numel() != self.D or not flat.is_contiguous():
            raise ValueError("apply needs a contiguous (%d,) tensor on %s" % (self.D, self.device))
        if flat.dtype == torch.float64:
            _lib.call("sra_apply_update_f64", *self._table(), flat.data_ptr(), self._stream())
        elif flat.dtype == torch.float32:
            _lib.call("sra_apply_update_f32", *self._table(), flat.data_ptr(), self._stream())
        else:
            raise TypeError("aggregate must be float32 or float64, got %s" % flat.dtype)


def fl_round(network, store, choices, local_update, args, state=None, attack="noattack", mal_index=()):
    """One round of simulate.py's loop (:139-404) with device-resident updates.

    ``local_update(c)`` runs client c's local training on ``network`` (the
    reference's inner loops, :175-186); the store records the update and
    restores the parameters.  ``attack`` is one of the reference's post-training
    attacks (:218-229: ``trimmedmean`` with b=1.5, ``krum`` per layer, ``xie``),
    run on the device by ``srfl_amd.attack``.  The aggregate is subtracted from
    the parameters in place and returned as the flat (D,) device vector."""
    from . import attack as atk, dispatch

    store.snapshot()
    for c in choices:
        local_update(int(c))
        store.record(int(c))
    lg = store.local_grads
    if attack == "trimmedmean":
        atk.attack_trimmedmean(network, lg, mal_index, b=1.5)
    elif attack == "krum":
        for idx in range(len(store.shapes)):
            atk.attack_krum(network, lg, mal_index, idx)
    elif attack == "xie":
        atk.attack_xie(lg, 1, choices, mal_index)
    elif attack != "noattack":
        raise ValueError("attack %r is not a post-training attack of simulate.py:218-229" % attack)
    flat, _ = dispatch.aggregate_flat(args.agg, lg, choices, args, state)
    store.apply(flat)
    return flat
