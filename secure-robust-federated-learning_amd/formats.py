"""The on-disk formats either side of the aggregation path,
so the reference's surrounding tooling reads what this engine writes.

* per-round result rows (simulate.py:134-135, 450-458; simulate_gan.py:126-127,
  359, 376): ``'%d, \\t%f, \\t%f\\n'`` (round, test loss, accuracy) or the
  five-column form with the malicious-set loss and attack success rate, in
  ``./results/<attack>_<agg>_<dataset>[_<malnum>].txt``;
* the GAN hand-off (simulate_gan.py:306-326, gan.py:305-372): per layer the
  chosen clients' updates as one ``(N, *layer_shape)`` array
  ``gan_<round>_<layer>.npy``, the global parameters before the update
  ``gan_Global_<round>_<layer>.npy``, and the GAN aggregator's result
  ``ganAgg_<round>.npy`` (a ragged object array of the per-layer parameters).

Client updates that live on the device (``store.ClientStore``) are gathered on
the device and copied to the host once per file.
"""
from __future__ import annotations

import io
import os

import numpy as np


# ---------------------------------------------------------------------------
# results/*.txt
# ---------------------------------------------------------------------------
def results_file_name(attack, agg, dataset, malnum=None, results_dir="./results"):
    """simulate.py:134 (with malnum) / simulate_gan.py:126 (without)."""
    name = "%s_%s_%s" % (attack, agg, dataset)
    if malnum is not None:
        name += "_%s" % malnum
    return os.path.join(results_dir, name + ".txt")


def _num(v):
    """Scalars as the reference formats them: a torch tensor (the accuracy is
    ``100. * correct / len(dataset)``, a float32 tensor) through ``float()``."""
    return float(v.item()) if hasattr(v, "item") else float(v)


def format_result_row(round_number, test_loss, accuracy, mal_loss=None, mal_accuracy=None):
    """One line of the results file; ``round_number`` is ``round_idx + 1``
    (simulate.py:458, and :435 / :450 for the malicious-set columns)."""
    if (mal_loss is None) != (mal_accuracy is None):
        raise ValueError("mal_loss and mal_accuracy go together (the five-column row)")
    if mal_loss is None:
        return "%d, \t%f, \t%f\n" % (int(round_number), _num(test_loss), _num(accuracy))
    return "%d, \t%f, \t%f, \t%f, \t%f\n" % (int(round_number), _num(test_loss), _num(accuracy), _num(mal_loss),
                                             _num(mal_accuracy))


def parse_results(source):
    """Rows of a results file (path, text or file object) as a float64 array of
    shape (rounds, 3 or 5); an empty file gives shape (0, 3)."""
    if hasattr(source, "read"):
        text = source.read()
    elif isinstance(source, str) and "\n" not in source and os.path.exists(source):
        with open(source) as fh:
            text = fh.read()
    else:
        text = source
    rows = []
    for line in text.splitlines():
        line = line.strip()
        if not line:
            continue
        rows.append([float(x) for x in line.split(",")])
    if not rows:
        return np.zeros((0, 3))
    width = {len(r) for r in rows}
    if len(width) != 1 or width.pop() not in (3, 5):
        raise ValueError("results rows must all have 3 or 5 columns")
    return np.array(rows, dtype=np.float64)


class ResultsWriter:
    """``txt_file`` of simulate.py:135: opened once, one row per checkpoint."""

    def __init__(self, path):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        self._fh = open(path, "w")
        self.path = path

    def write(self, round_idx, test_loss, accuracy, mal_loss=None, mal_accuracy=None):
        self._fh.write(format_result_row(round_idx + 1, test_loss, accuracy, mal_loss, mal_accuracy))
        self._fh.flush()

    def close(self):
        self._fh.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---------------------------------------------------------------------------
# GAN hand-off
# ---------------------------------------------------------------------------
def _layer_stack(local_grads, choices, idx):
    """``np.array([local_grads[c][idx] for c in choices])`` with device tensors
    stacked on the device and copied once."""
    first = local_grads[int(choices[0])][idx]
    if hasattr(first, "is_cuda") and first.is_cuda:
        import torch
        store = getattr(local_grads, "store", None)
        rows = [int(c) for c in choices]
        if store is not None and store.intact(rows):
            lo, hi = store.seg[idx], store.seg[idx + 1]
            blk = store.U[:, lo:hi].index_select(0, store.rows(rows))
            return blk.cpu().numpy().reshape((len(rows),) + tuple(store.shapes[idx]))
        return torch.stack([local_grads[c][idx] for c in rows]).cpu().numpy()
    return np.array([np.asarray(local_grads[int(c)][idx]) for c in choices])


def gan_layer_path(round_idx, idx, results_dir="./results"):
    return os.path.join(results_dir, "gan_%d_%d.npy" % (round_idx, idx))


def gan_global_path(round_idx, idx, results_dir="./results"):
    return os.path.join(results_dir, "gan_Global_%d_%d.npy" % (round_idx, idx))


def gan_agg_path(round_idx, results_dir="./results"):
    return os.path.join(results_dir, "ganAgg_%d.npy" % round_idx)


def save_gan_layers(local_grads, choices, round_idx, results_dir="./results"):
    """simulate_gan.py:306-313: ``np.save(f, gan_local)`` per layer."""
    nlayer = len(local_grads[int(choices[0])])
    paths = []
    for idx in range(nlayer):
        p = gan_layer_path(round_idx, idx, results_dir)
        with open(p, "wb") as f:
            np.save(f, _layer_stack(local_grads, choices, idx))
        paths.append(p)
    return paths


def save_gan_global(params, round_idx, results_dir="./results"):
    """simulate_gan.py:321-326: the parameters before the round's update."""
    paths = []
    for idx, p in enumerate(params):
        path = gan_global_path(round_idx, idx, results_dir)
        with open(path, "wb") as f:
            np.save(f, p.detach().cpu().numpy() if hasattr(p, "detach") else np.asarray(p))
        paths.append(path)
    return paths


def load_gan_layer(round_idx, idx, results_dir="./results"):
    """gan.py:307-309 (plain numeric array; no pickle)."""
    with open(gan_layer_path(round_idx, idx, results_dir), "rb") as f:
        return np.load(f, allow_pickle=False)


def save_gan_agg(layers, round_idx, results_dir="./results"):
    """gan.py:364-372: ``np.save(f, gan_results)``; the per-layer arrays are
    ragged, so the file holds an object array (as numpy 1.21 produced it)."""
    arr = np.empty(len(layers), dtype=object)
    for i, a in enumerate(layers):
        arr[i] = a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)
    path = gan_agg_path(round_idx, results_dir)
    with open(path, "wb") as f:
        np.save(f, arr, allow_pickle=True)
    return path


def load_gan_agg(round_idx, results_dir="./results"):
    """simulate_gan.py:133-137 reads ``ganAgg_<round>.npy`` with
    ``allow_pickle=True``.  Only for files this engine (or the reference's
    gan.py) wrote in the caller's own results directory."""
    with open(gan_agg_path(round_idx, results_dir), "rb") as f:
        data = f.read()
    return list(np.load(io.BytesIO(data), allow_pickle=True))
