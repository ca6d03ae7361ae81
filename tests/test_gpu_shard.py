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
    row, idx = shard.krum(ops["gram"], ops["krum_select"], X, 30_000, 20, exact=ops)
    want_row, order = engine.krum(X, 20)
    assert idx == int(order.cpu()[0])
    assert torch.equal(row, want_row)


def test_sharded_mom_krum_bit_exact(nccl_group):
    """bench.py's N > 1 mom_krum path: the bucket Gram all-reduced through RCCL,
    the chosen bucket's mean all-gathered; equal to the unsharded fused op."""
    x = make_rows(512, 20_000, seed=34, byz=60)
    X = torch.from_numpy(x).cuda()
    row, idx = shard.mom_krum(shard.engine_ops(), X, 20_000, 20)
    want_row, order = engine.mom_krum(X, 20)
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


def test_pipelined_mom_filter_l2_c5_path(nccl_group):
    """bench.py's N > 1 path for config C5 (mom_filterL2, N = 512): itv-aligned
    block-cyclic blocks, each filtered straight into its slot of the all-gather
    buffer, the in-place all-gathers through RCCL on a second stream -- equal
    bit for bit to the unsharded call (chunks of itv columns are independent,
    robust_estimator.py:192-201)."""
    import bench
    d = 12_000
    x = make_rows(512, d, seed=34, byz=100)
    X = torch.from_numpy(x).cuda()
    block = bench.filter_block(d, 4, bench.FILTER_ARGS["itv"])
    assert block == 3000
    got = shard.pipelined_coordinatewise(bench.filter_into("mom_filterl2"), X, d, block)
    want = engine.mom_filter_l2(X, delta=bench.MOM_DELTA, check=False, **bench.FILTER_ARGS)
    torch.cuda.synchronize()
    assert got.dtype == torch.float64
    assert torch.equal(got, want)


@pytest.mark.parametrize("mode", ["median", "trimmedmean"])
def test_column_split_bulyan_rounds(mode):
    """What an N-GPU Bulyan round computes, on one GPU: each of three column
    slices (unequal, not tile-aligned) runs sra_bulyan_round_f32 on its own,
    the three fp64 distance vectors are added (the all-reduce), and the pick
    is made from the sum.  The summed distances equal the unsharded round's to
    fp32 rounding (each 64-coordinate tile is summed in fp32, and the shard
    bounds regroup the tiles: measured 1.7e-8 relative; the reference's own
    fp32 norms carry ~1e-7), so a near-tie pick may differ between GPU counts
    (INTEGRATION.md); on data without near ties the selection and the final
    stage are identical to the unsharded engine.bulyan."""
    n, d, f = 48, 10_000, 8
    theta = n - 2 * f
    x = make_rows(n, d, seed=35, byz=8)
    X = torch.from_numpy(x).cuda()
    cuts = [(0, 3_001), (3_001, 7_777), (7_777, d)]
    rows = torch.arange(n, dtype=torch.int32, device="cuda")
    nxt = torch.empty_like(rows)
    rows1 = rows.clone()
    nxt1 = torch.empty_like(rows)
    S = torch.empty((theta, d), dtype=torch.float32, device="cuda")
    agg1 = torch.empty(d, dtype=torch.float32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    for t in range(theta):
        nr = n - t
        tot = torch.zeros(nr, dtype=torch.float64, device="cuda")
        for lo, hi in cuts:
            dv = torch.empty(nr, dtype=torch.float64, device="cuda")
            engine.bulyan_round(X[:, lo:hi], rows, nr, mode, S[t, lo:hi], dv)
            tot += dv
        one = torch.empty(nr, dtype=torch.float64, device="cuda")
        engine.bulyan_round(X, rows1, nr, mode, agg1, one)
        torch.testing.assert_close(tot, one, rtol=1e-6, atol=0)
        assert torch.equal(agg1, S[t])
        engine.bulyan_pick(tot, rows, nr, nxt, status)
        engine.bulyan_pick(one, rows1, nr, nxt1)
        rows, nxt = nxt, rows
        rows1, nxt1 = nxt1, rows1
        assert torch.equal(rows[:nr - 1], rows1[:nr - 1]), t
    assert int(status.item()) == 0
    got = engine.bulyan_stage(S, theta - 2 * f)
    want = engine.bulyan(X, f, mode)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
