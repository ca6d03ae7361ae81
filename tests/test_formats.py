"""The on-disk formats around the path (srfl_amd.formats):
results rows reproduce the reference's own results files line for line
(tests/golden/results/ are copies of /root/reference/results/*.txt), and the
GAN hand-off files are byte-identical to what the reference's ``np.save``
calls write (simulate_gan.py:306-326, gan.py:364-372)."""
from __future__ import annotations

import io
import os

import numpy as np
import pytest
import torch

from srfl_amd import formats

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "results")
FILES = sorted(os.listdir(GOLDEN))
CONVNET = [(30, 1, 5, 5), (30,), (30, 30, 5, 5), (30,), (200, 1470), (200,), (10, 200), (10,)]


@pytest.mark.parametrize("name", FILES)
def test_results_rows_roundtrip_reference_files(name):
    path = os.path.join(GOLDEN, name)
    with open(path) as fh:
        lines = fh.readlines()
    rows = formats.parse_results(path)
    assert rows.shape[0] == len(lines)
    for line, row in zip(lines, rows):
        assert formats.format_result_row(int(row[0]), *row[1:]) == line


def test_accuracy_is_formatted_as_the_float32_tensor():
    # simulate.py:419: accuracy = 100. * correct / len(test_loader.dataset), correct a torch integer sum
    acc = 100. * torch.tensor(2655) / 10000
    assert formats.format_result_row(1, 2.244289, acc) == "1, \t2.244289, \t26.549999\n"
    five = formats.format_result_row(3, 0.5, 90.0, 1.25, torch.tensor(12.5))
    assert five == "3, \t0.500000, \t90.000000, \t1.250000, \t12.500000\n"
    assert formats.parse_results(five).shape == (1, 5)
    with pytest.raises(ValueError):
        formats.format_result_row(1, 0.5, 90.0, 1.25)


def test_results_file_names_and_writer(tmp_path):
    assert formats.results_file_name("noattack", "clustering", "MNIST", 20) == \
        "./results/noattack_clustering_MNIST_20.txt"                       # simulate.py:134
    assert formats.results_file_name("krum", "gan", "MNIST") == "./results/krum_gan_MNIST.txt"  # simulate_gan.py:126
    p = formats.results_file_name("noattack", "median", "MNIST", 20, results_dir=str(tmp_path))
    with formats.ResultsWriter(p) as w:
        w.write(0, 2.5, 10.0)
        w.write(1, 2.25, 20.0)
    np.testing.assert_array_equal(formats.parse_results(p), [[1, 2.5, 10.0], [2, 2.25, 20.0]])
    assert formats.parse_results("").shape == (0, 3)


def _ref_save(obj):
    buf = io.BytesIO()
    np.save(buf, obj)
    return buf.getvalue()


def test_gan_files_byte_identical(tmp_path):
    rng = np.random.default_rng(0)
    n = 12
    local_grads = [[rng.standard_normal(s).astype(np.float32) for s in CONVNET] for _ in range(n)]
    choices = rng.permutation(n)[:10]
    paths = formats.save_gan_layers(local_grads, choices, 4, str(tmp_path))
    for idx, p in enumerate(paths):
        assert os.path.basename(p) == "gan_4_%d.npy" % idx
        gan_local = [local_grads[c][idx] for c in choices]                  # simulate_gan.py:308-310
        with open(p, "rb") as f:
            assert f.read() == _ref_save(gan_local)
        np.testing.assert_array_equal(formats.load_gan_layer(4, idx, str(tmp_path)), np.array(gan_local))
    params = [torch.from_numpy(a) for a in local_grads[0]]
    for idx, p in enumerate(formats.save_gan_global(params, 4, str(tmp_path))):
        with open(p, "rb") as f:
            assert f.read() == _ref_save(local_grads[0][idx])
    formats.save_gan_agg(params, 5, str(tmp_path))
    back = formats.load_gan_agg(5, str(tmp_path))
    assert len(back) == len(CONVNET)
    for a, b in zip(back, local_grads[0]):
        np.testing.assert_array_equal(a, b)
