"""The multi-GPU sharding layer (srfl_amd/shard.py) on the GPU through RCCL:
a 1-rank "nccl" process group in this process, so every collective the
N-GPU path issues (the in-place all-gathers of the pipelined coordinate-wise
path on a second stream, the Gram all-reduce of Krum, the per-round distance
all-reduce of Bulyan) runs through RCCL, and each result must equal the
unsharded engine call bit for bit."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from conftest import gpu_available
from synth import make_rows

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch
    import torch.distributed as dist
    from srfl_amd import engine, shard


@pytest.fixture(scope="module")
def nccl_group():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("agg,block", [("trimmedmean", 4096), ("median", 1000), ("average", 333)])
def test_pipelined_coordinatewise_bit_exact(nccl_group, agg, block):
    x = make_rows(128, 20_000, seed=31, byz=20)
    X = torch.from_numpy(x).cuda()
    into = shard.engine_ops()[agg + "_into"]
    got = shard.pipelined_coordinatewise(into, X, 20_000, block)
    want = {"trimmedmean": lambda: engine.trimmed_mean(X, 0.1), "median": lambda: engine.median(X),
            "average": lambda: engine.average(X)}[agg]()
    torch.cuda.synchronize()
    assert torch.equal(got, want)


def test_sharded_krum_bit_exact(nccl_group):
    x = make_rows(100, 30_000, seed=32, byz=20)
    X = torch.from_numpy(x).cuda()
    ops = shard.engine_ops()
    row, idx = shard.krum(ops["gram"], ops["krum_select"], X, 30_000, 20)
    want_row, order = engine.krum(X, 20)
    assert idx == int(order.cpu()[0])
    assert torch.equal(row, want_row)


@pytest.mark.parametrize("mode", ["krum", "median", "trimmedmean"])
def test_sharded_bulyan_bit_exact(nccl_group, mode):
    x = make_rows(64, 12_000, seed=33, byz=10)
    X = torch.from_numpy(x).cuda()
    got = shard.bulyan(shard.engine_ops(), X, 12_000, 10, mode)
    want = engine.bulyan(X, 10, mode)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
