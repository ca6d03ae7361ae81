"""Drop-in for the aggregation methods of the DBA harness's ``Helper``
(src/DBA/helper.py:251-1173, dispatched by src/DBA/main.py:184-240; SURVEY.md
§8(f).4), on the engine's HIP kernels.

The DBA harness carries its own torch re-implementations of the robust
aggregators, with semantics that differ from src/robust_estimator.py:

* ``median`` is torch.median's LOWER median (helper.py:561) -> ``sra_order_stat_f32``;
* ``krum`` picks a client PER LAYER (helper.py:705-714);
* ``mom_krum``'s buckets alias one dict and divide by count + 1 (helper.py:857-863),
  so every layer ends as the last bucket's sum / (size + 1) -> ``sra_rows_sum_div_f32``;
* ``bulyan_krum`` counts the zero self-distance among the nearest (helper.py:976-980),
  ``bulyan_median`` selects with the lower median -> ``sra_bulyan_dba_f32``;
* ``history`` / ``bucketing`` re-root the running norm after every layer
  (helper.py:753-757) -> ``sra_clip_scale_running_f32``;
* ``geometric_median_update`` (RFA / Weiszfeld) averages with torch's
  ``w * p`` then ``add_`` rounding -> ``sra_weighted_sum_f32``;
* ``sharding`` shuffles with Python's ``random`` and averages 50 shards.

``HelperAggregation`` holds the state those methods read (``params``,
``history_prev_average_grad``, ``history_tau``) and keeps the reference's
method names, signatures, return values and exceptions; ``updates`` is the
``{name: (num_samples, {layer: tensor})}`` dict of DBA/main.py:181.  Client
updates are stacked once into a client-major (N, D) float32 matrix on the HIP
device; every reduction over clients runs in libsra.  There is no CPU
fallback.  ``foolsgold_update`` keeps the reference's behaviour exactly: its
FoolsGold weighting (helper.py:1388-1417) ends in ``return wv,alpha(base)``,
which raises NameError on every call, so the weights are computed on the
device (``foolsgold_weights``, kept on ``self.fg.last``) and the same NameError
is raised; the model is never updated, as in the reference.
"""
from __future__ import annotations

import copy
import math
import random

import numpy as np
import torch

from . import engine

ITV = 1000                 # helper.py:26
SHARD_BUCKETS = 50         # helper.py:1151


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("srfl_amd.dba needs an MI355X (HIP device); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


class _Staged:
    """Client updates of one call as an (N, D) float32 device matrix."""

    def __init__(self, samples):
        first = samples[0]
        self.keys = list(first.keys())
        self.shapes = [tuple(first[k].shape) for k in self.keys]
        self.dtypes = [first[k].dtype for k in self.keys]
        sizes = [int(np.prod(s, dtype=np.int64)) for s in self.shapes]
        self.seg = [0]
        for s in sizes:
            self.seg.append(self.seg[-1] + s)
        dev = _device()
        rows = [torch.cat([torch.as_tensor(s[k]).reshape(-1).float() for k in self.keys]) for s in samples]
        self.X = torch.stack(rows).to(dev, non_blocking=True)

    @property
    def n(self):
        return int(self.X.shape[0])

    def cols(self, l):
        return self.X[:, self.seg[l]:self.seg[l + 1]]

    def split(self, vec):
        """{layer: view of vec reshaped} in the staged layer order."""
        return {k: vec[self.seg[l]:self.seg[l + 1]].reshape(self.shapes[l]) for l, k in enumerate(self.keys)}


class FoolsGoldState:
    """The FoolsGold object of helper.py:1321-1326 (per-client feature memory)."""

    def __init__(self, use_memory=False):
        self.memory = None
        self.memory_dict = dict()
        self.wv_history = []
        self.use_memory = use_memory
        self.last = None


def foolsgold_weights(F):
    """FoolsGold.foolsgold (helper.py:1388-1417) on a device float64 (N, k)
    feature matrix: cosine similarity (rows at unit L2 norm, zero rows kept;
    sklearn's cosine_similarity) minus the identity, pardoning
    cs[i][j] *= maxcs[i] / maxcs[j] where maxcs[i] < maxcs[j], then the
    clip / rescale / logit of the weights.  Returns (wv, alpha) on the device."""
    n = int(F.shape[0])
    eye = torch.eye(n, dtype=torch.float64, device=F.device)
    nrm = torch.sqrt((F * F).sum(dim=1))
    nrm = torch.where(nrm == 0, torch.ones_like(nrm), nrm)
    U = F / nrm[:, None]
    cs = U @ U.T - eye
    maxcs = cs.max(dim=1).values
    pard = (maxcs[:, None] < maxcs[None, :]) & (eye == 0)
    cs = torch.where(pard, cs * maxcs[:, None] / maxcs[None, :], cs)
    top = cs.max(dim=1).values
    wv = (1 - top).clamp(min=0, max=1)
    alpha = top
    wv = wv / wv.max()
    wv = torch.where(wv == 1, torch.full_like(wv, .99), wv)
    wv = torch.log(wv / (1 - wv)) + 0.5
    wv = torch.where(torch.isinf(wv).double() + wv > 1, torch.ones_like(wv), wv)
    wv = torch.where(wv < 0, torch.zeros_like(wv), wv)
    return wv, alpha


class HelperAggregation:
    """The aggregation methods of src/DBA/helper.py ``Helper`` on the engine."""

    def __init__(self, params=None):
        self.params = dict(params or {})
        self.params.setdefault("eta", 1)
        self.params.setdefault("sharding", False)
        self.params.setdefault("shard_size", 0.2)
        self.params.setdefault("diff_privacy", False)
        self.history_prev_average_grad = None
        self.history_tau = 10.
        self.fg = FoolsGoldState(use_memory=self.params.get("fg_use_memory", False))

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _collect(updates):
        """helper.py:252-260: names, num_samples, update dicts in dict order."""
        names, alphas, samples = [], [], []
        for name, data in updates.items():
            samples.append(data[1])
            alphas.append(data[0])
            names.append(name)
        return names, alphas, samples

    def _apply(self, target_model, chosen):
        """helper.py:283-288: data += chosen * eta, cast to the parameter's type."""
        for name, data in target_model.state_dict().items():
            upd = chosen[name] * self.params["eta"]
            if upd.device != data.device:
                upd = upd.to(data.device)
            if upd.dtype != data.dtype:
                upd = upd.type_as(data)
            data.add_(upd)

    def dp_noise(self, param, sigma):
        """helper.py dp_noise: N(0, sigma) noise of the parameter's shape."""
        return torch.empty(param.shape, dtype=torch.float32, device=param.device).normal_(0, sigma)

    def _staged(self, samples, shard=None):
        shard = self.params["sharding"] if shard is None else shard
        st = _Staged(samples)
        if shard:
            st.X = self._shard_matrix(st.X)
        return st

    # ----------------------------------------------------------------- sharding
    @staticmethod
    def _shard_matrix(X):
        """helper.py:1139-1166 on the staged rows: random.shuffle(samples) (the
        module-level Python RNG, consumed exactly as the reference does), then
        50 shards of ceil(N/50) consecutive clients, each averaged
        (sequential fp32 sum / count, sra_bucket_mean_f32)."""
        n = int(X.shape[0])
        order = list(range(n))
        random.shuffle(order)
        bs = int(np.ceil(n * 1. / SHARD_BUCKETS))
        if (SHARD_BUCKETS - 1) * bs >= n:
            raise IndexError("list index out of range")   # samples[begin_index] of an empty shard (:1156)
        rows = torch.tensor(order, dtype=torch.int32, device=X.device)
        return engine.bucket_means(engine.gather_rows(X, rows), bs, SHARD_BUCKETS)

    def sharding(self, samples, eps=0.2, delta=np.exp(-5)):
        """helper.py:1139: list of 50 shard-average update dicts."""
        st = _Staged(samples)
        S = self._shard_matrix(st.X)
        return [st.split(S[i]) for i in range(S.shape[0])]

    # -------------------------------------------------------- coordinate-wise
    def fed_avg(self, target_model, updates):
        """helper.py:251-289: mean over clients (sra_average_f32)."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        self._apply(target_model, st.split(engine.average(st.X)))
        return True

    def median(self, target_model, updates):
        """helper.py:529-569: torch.median lower median (sra_order_stat_f32)."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        self._apply(target_model, st.split(engine.order_stat(st.X, (st.n - 1) // 2)))
        return True

    def trimmed_mean(self, target_model, updates, beta=0.1):
        """helper.py:892-930: mean of s[b : N-b], b = int(N*beta)."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        self._apply(target_model, st.split(engine.trimmed_mean(st.X, beta)))
        return True

    # ------------------------------------------------------------------- Krum
    def krum(self, target_model, updates, f=0):
        """helper.py:676-720: a Krum pick per layer (self excluded, N-f-2
        nearest); the layer takes its chosen client's values."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        chosen = {}
        for l, k in enumerate(st.keys):
            Xl = st.cols(l)
            order, _ = engine.krum_select(Xl, f, 1, scores=False)
            chosen[k] = engine.gather_rows(Xl, order)[0].reshape(st.shapes[l])
        self._apply(target_model, chosen)
        return True

    def mom_krum(self, target_model, updates, f=0, bucket_size=3):
        """helper.py:833-890.  All buckets are one aliased dict (:859), so every
        Krum score is 0 and the result is the last bucket's sum / (size + 1)."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        nb = int(np.ceil(st.n * 1. / bucket_size))
        lo, hi = (nb - 1) * bucket_size, min(nb * bucket_size, st.n)
        self._apply(target_model, st.split(engine.rows_sum_div(st.X[lo:hi], hi - lo + 1)))
        return True

    # ----------------------------------------------------------------- Bulyan
    def _bulyan(self, target_model, updates, f, mode):
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        if st.n - 2 * f <= 0:
            raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")   # helper.py:985 / 1035
        chosen = {}
        status = torch.zeros(len(st.keys), dtype=torch.int32, device=st.X.device)
        for l, k in enumerate(st.keys):
            out = engine.bulyan_dba(st.cols(l), f, mode, status=status[l:l + 1])
            chosen[k] = out.float().reshape(st.shapes[l])
        if mode != "krum":   # helper.py:1047 / :1119, one read back per round
            engine.check_bulyan_status(status, "bulyan_dba(%s)" % mode)
        self._apply(target_model, chosen)
        return True

    def bulyan_krum(self, target_model, updates, f=20):
        """helper.py:942-992."""
        return self._bulyan(target_model, updates, f, "krum")

    def bulyan_median(self, target_model, updates, f=20):
        """helper.py:994-1050."""
        return self._bulyan(target_model, updates, f, "median")

    def bulyan_trimmed_mean(self, target_model, updates, f=20):
        """helper.py:1053-1137."""
        return self._bulyan(target_model, updates, f, "trimmedmean")

    # -------------------------------------------------------- spectral filters
    def filterl2(self, target_model, updates, sigma=1, expansion=1, itv=None):
        """helper.py:607-674: per layer, chunks of ITV (the itv argument is
        overwritten, :650); filterl2_ with eps = 0.2."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        chosen = {}
        for l, k in enumerate(st.keys):
            out = engine.filter_l2(st.cols(l), eps=0.2, sigma=sigma, expansion=expansion, itv=ITV)
            chosen[k] = out.float().reshape(st.shapes[l])
        self._apply(target_model, chosen)
        return True

    def ex_noregret(self, target_model, updates, eps=1. / 12, sigma=1, expansion=20, itv=ITV):
        """helper.py:466-527: per layer; itv=None becomes int(sqrt(numel)) of the
        first layer and is kept for the rest (:507-508).  fp64 aggregate."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples)
        chosen = {}
        for l, k in enumerate(st.keys):
            if itv is None:
                itv = int(np.sqrt(st.seg[l + 1] - st.seg[l]))
            out = engine.ex_noregret(st.cols(l), eps=eps, sigma=sigma, expansion=expansion, itv=itv)
            chosen[k] = out.reshape(st.shapes[l])
        self._apply(target_model, chosen)
        return True

    # ------------------------------------------------------ history / bucketing
    def _clip_round(self, st, samples, write_back):
        if self.history_prev_average_grad is None:
            prev = torch.zeros(st.seg[-1], dtype=torch.float64, device=st.X.device)
        else:
            prev = torch.cat([self.history_prev_average_grad[k].reshape(-1).to(st.X.device).double()
                              for k in st.keys])
        scale = engine.clip_scales(st.X, prev, st.seg, self.history_tau, running=True)
        clipped = torch.empty((st.n, st.seg[-1]), dtype=torch.float64, device=st.X.device) if write_back else None
        mean = engine.clipped_mean(st.X, prev, scale, clipped=clipped).float()
        if write_back:   # helper.py:759: the clipped updates replace the caller's tensors
            c32 = clipped.float()
            for c, s in enumerate(samples):
                for l, k in enumerate(st.keys):
                    s[k] = c32[c, st.seg[l]:st.seg[l + 1]].reshape(st.shapes[l])
        chosen = st.split(mean)
        self.history_prev_average_grad = {k: v.clone() for k, v in chosen.items()}
        return chosen

    def history(self, target_model, updates):
        """helper.py:722-777."""
        _, _, samples = self._collect(updates)
        shard = self.params["sharding"]
        st = self._staged(samples)
        self._apply(target_model, self._clip_round(st, samples, write_back=not shard))
        return True

    def bucketing(self, target_model, updates):
        """helper.py:779-831: sharding always, then history's clipping."""
        _, _, samples = self._collect(updates)
        st = self._staged(samples, shard=True)
        self._apply(target_model, self._clip_round(st, samples, write_back=False))
        return True

    # --------------------------------------------------------- geometric median
    def geometric_median_update(self, target_model, updates, maxiter=4, eps=1e-5, verbose=False, ftol=1e-6,
                                max_update_norm=None):
        """helper.py:327-410 (RFA, Weiszfeld).  Returns (num_oracle_calls,
        is_updated, names, weights, distances) like the reference."""
        names, alphas, samples = self._collect(updates)
        st = _Staged(samples)
        dev = st.X.device
        alphas = torch.from_numpy(np.asarray(alphas, dtype=np.float64) / sum(alphas)).float()
        a64 = alphas.double().numpy()

        def oracle(w):                     # weighted_average_oracle (:1199-1221)
            w = w.to(dev)
            return engine.weighted_sum(st.X, w / torch.sum(w))

        def dists(m):                      # l2dist of every point (:1176-1181)
            _, nrm = engine.clip_scales(st.X, m.double(), st.seg, 1.0, norms=True)
            return nrm.cpu().numpy()

        median = oracle(alphas)
        num_oracle_calls = 1
        d = dists(median)
        obj_val = float(np.sum(a64 * d))
        wv = None
        for _ in range(maxiter):
            prev_obj_val = obj_val
            weights = torch.tensor([float(a) / max(eps, float(x)) for a, x in zip(alphas, d)], dtype=alphas.dtype)
            weights = weights / weights.sum()
            median = oracle(weights)
            num_oracle_calls += 1
            d = dists(median)
            obj_val = float(np.sum(a64 * d))
            if abs(prev_obj_val - obj_val) < ftol * obj_val:
                break
            wv = copy.deepcopy(weights)
        dist_out = [float(x) for x in d]
        update_norm = math.sqrt(float(torch.sum(median.double() ** 2)))
        if max_update_norm is None or update_norm < max_update_norm:
            chosen = st.split(median)
            for name, data in target_model.state_dict().items():
                upd = chosen[name].to(data.device) * self.params["eta"]
                if self.params["diff_privacy"]:
                    upd.add_(self.dp_noise(data, self.params["sigma"]))
                data.add_(upd)
            is_updated = True
        else:
            is_updated = False
        return num_oracle_calls, is_updated, names, wv.cpu().numpy().tolist(), dist_out


def _foolsgold_update(self, target_model, updates):
    """helper.py:291-325: updates carry per-layer gradient lists; FoolsGold
    weighs the clients by the second-to-last layer (accumulated per client
    name when fg.use_memory), helper.py:1328-1345.  The reference's weighting
    returns through ``alpha(base)`` (:1417) and raises NameError, so this does
    too, after the same side effects (model in train mode, grads cleared,
    memory accumulated); the computed (wv, alpha) stay on ``self.fg.last``."""
    names, _, client_grads = self._collect(updates)
    if hasattr(target_model, "train"):
        target_model.train()
    if hasattr(target_model, "parameters"):
        for p in target_model.parameters():
            p.grad = None
    dev = _device()
    F = torch.stack([torch.as_tensor(g[-2]).reshape(-1).to(dev, torch.float64) for g in client_grads])
    mem = []
    for i, nm in enumerate(names):
        if nm in self.fg.memory_dict:
            self.fg.memory_dict[nm] += F[i]
        else:
            self.fg.memory_dict[nm] = F[i].clone()
        mem.append(self.fg.memory_dict[nm])
    self.fg.memory = torch.stack(mem)
    self.fg.last = foolsgold_weights(self.fg.memory if self.fg.use_memory else F)
    raise NameError("name 'base' is not defined")


HelperAggregation.foolsgold_update = _foolsgold_update


# DBA/main.py:184-240 -- config.AGGR_* name -> call
def aggregate(helper, method, target_model, updates):
    """Mirror of the if/elif chain of src/DBA/main.py:184-240 (config names of
    src/DBA/config.py).  Returns what the Helper method returns."""
    p = helper.params
    if method == "mean":
        return helper.fed_avg(target_model, updates)
    if method == "geom_median":
        return helper.geometric_median_update(target_model, updates, maxiter=p["geom_median_maxiter"])
    if method == "krum":
        return helper.krum(target_model, updates, f=p["krum_f"])
    if method == "trimmedmean":
        return helper.trimmed_mean(target_model, updates, beta=p["trim_beta"])
    if method == "bulyan_krum":
        return helper.bulyan_krum(target_model, updates, f=p["krum_f"])
    if method == "bulyan_trimmed_mean":
        return helper.bulyan_trimmed_mean(target_model, updates, f=p["krum_f"])
    if method == "filterl2":
        return helper.filterl2(target_model, updates, sigma=p["fliter_l2_sigma"], expansion=20, itv=None)
    if method == "ex_noregret":
        return helper.ex_noregret(target_model, updates, eps=1. / 5, sigma=p["fliter_l2_sigma"], expansion=20,
                                  itv=1000)
    if method == "median":
        return helper.median(target_model, updates)
    if method == "bulyan_median":
        return helper.bulyan_median(target_model, updates)
    if method == "clustering":
        return helper.mom_krum(target_model, updates, f=p["krum_f"])
    if method == "history":
        return helper.history(target_model, updates)
    if method == "bucketing":
        return helper.bucketing(target_model, updates)
    if method == "foolsgold":
        return helper.foolsgold_update(target_model, updates)
    raise ValueError("unknown aggregation method %r" % (method,))
