"""Two ranks EXECUTING the HIP shard path (srfl_amd/shard.py with
shard.engine_ops()) on the one GPU of the box.

test_gpu_shard.py runs every collective through RCCL in a 1-rank group (each
collective is then the identity) and test_shard_gloo.py runs the sharding logic
with world sizes 2 and 3 on CPU with the oracle as the per-shard ops.  Here two
fresh ranks (spawn context: new interpreters, each initialising the GPU
itself) run the real kernels on their own column shards of the same GPU over
a gloo group (RCCL refuses two ranks on one device; shard.py stages device
tensors through host memory for gloo), and the parent requires the assembled
results to equal the unsharded engine call bit for bit:

  * trimmed mean on block-cyclic shards, pipelined in-place all-gather;
  * Krum (partial centred Grams reduced to rank 0, which scores and
    broadcasts), mom_krum (the bucket-mean Gram, never written);
  * Bulyan in all three modes (per-round all-reduce of the distance partials,
    shards 256-column aligned like the round kernel's blocks);
  * config C5's bench path: mom_filterL2 on itv-aligned block-cyclic shards.

Column independence (robust_estimator.py:116-125, 192-201, 223-232) makes the
coordinate-wise and chunked results exact; the Krum / Bulyan picks come from
sums of per-shard fp64 partials (a different association than the unsharded
kernel's, so the data keep the picks away from ties) and the returned rows /
stage outputs are then exact."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
WORLD = 2
SH = dict(n=128, d=40_960, f=20, seed=41, byz=20)     # Krum / Bulyan layers (d % (2 x 256) == 0)
C5 = dict(n=512, d_rank=8_000, itv=1000, seed=42, byz=100)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data():
    from synth import make_rows
    x = make_rows(SH["n"], SH["d"], seed=SH["seed"], byz=SH["byz"])
    xc5 = make_rows(C5["n"], C5["d_rank"] * WORLD, seed=C5["seed"], byz=C5["byz"])
    return x, xc5


EXACT_FIXTURES = ["krum_nan_client_n12_f2", "krum_inf_clients_n12_f2", "krum_nan_two_n12_f2",
                  "krum_nan_client_n128_f20", "krum_nan_client_n300_f30", "mom_krum_nan_client_n30_f3",
                  "bulyan_krum_nan_client_n24_f5"]


def exact_fixtures():
    from conftest import load_fixture
    return {nm: load_fixture(os.path.join(HERE, "golden", nm + ".npz")) for nm in EXACT_FIXTURES}


def wide_nonfinite():
    """SH-sized layers (d = 40,960: not narrow) with a NaN client / +-inf
    entries: the summed Gram's non-finite diagonal switches the route."""
    x, _ = _data()
    nan = x.copy()
    nan[37, 20_000] = np.nan
    inf = x.copy()
    inf[5, 100] = np.inf
    inf[90, 30_000] = -np.inf
    return {"nan": nan, "inf": inf}


def _rank(rank, port, results):
    for p in (ROOT, HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import srfl_loader
    srfl_loader.load()
    import torch
    import torch.distributed as dist
    import bench
    from srfl_amd import engine, shard
    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        ops = shard.engine_ops()
        x, xc5 = _data()
        out = {}
        n, d, f = SH["n"], SH["d"], SH["f"]
        # trimmed mean: block-cyclic shards, pipelined all-gather (device
        # aggregation into the full vector, the collective on a second stream)
        block = 4096
        cols = shard.cyclic_blocks(d, WORLD, rank, block)
        Xc = torch.from_numpy(np.ascontiguousarray(np.concatenate([x[:, lo:hi] for lo, hi in cols], axis=1))).cuda()
        out["trimmedmean"] = shard.pipelined_coordinatewise(ops["trimmedmean_into"], Xc, d, block).cpu().numpy()
        # an explicit communication stream and small blocks (40 rounds): each
        # round's all-gather is ordered after its block's k-select by an event
        # on comm, while the next block's k-select runs on the compute stream
        comm = torch.cuda.Stream()
        block = 512
        cols = shard.cyclic_blocks(d, WORLD, rank, block)
        Xc = torch.from_numpy(np.ascontiguousarray(np.concatenate([x[:, lo:hi] for lo, hi in cols], axis=1))).cuda()
        out["trimmedmean_comm"] = shard.pipelined_coordinatewise(ops["trimmedmean_into"], Xc, d, block,
                                                                comm_stream=comm).cpu().numpy()
        # contiguous 256-aligned shards for the Gram / Bulyan layers
        lo, hi = shard.shard_bounds(d, WORLD, rank, align=256)
        Xs = torch.from_numpy(np.ascontiguousarray(x[:, lo:hi])).cuda()
        row, idx = shard.krum(ops["gram"], ops["krum_select"], Xs, d, f, align=256, exact=ops)
        out["krum_row"], out["krum_idx"] = row.cpu().numpy(), idx
        row, idx = shard.mom_krum(ops, Xs, d, f, align=256)
        out["mom_krum_row"], out["mom_krum_idx"] = row.cpu().numpy(), idx
        for mode in ("krum", "median", "trimmedmean"):
            out["bulyan_" + mode] = shard.bulyan(ops, Xs, d, f, mode, align=256).cpu().numpy()
        # config C5: mom_filterL2 (N = 512, 128 buckets of 4) on itv-aligned
        # block-cyclic shards, the bench's pipeline
        dt = C5["d_rank"] * WORLD
        fblock = bench.filter_block(C5["d_rank"], 4, C5["itv"])
        cols = shard.cyclic_blocks(dt, WORLD, rank, fblock)
        Xf = torch.from_numpy(np.ascontiguousarray(np.concatenate([xc5[:, lo:hi] for lo, hi in cols], axis=1))).cuda()
        out["c5_block"] = fblock
        out["c5"] = shard.pipelined_coordinatewise(bench.filter_into("mom_filterl2"), Xf, dt, fblock,
                                                   comm_stream=comm).cpu().numpy()
        # the exact per-pair route over shards: the live-reference NaN / inf
        # fixtures (narrow layers) and full-width layers with a NaN / inf client
        for name, rec in exact_fixtures().items():
            xe, fe = rec["x"], int(rec["params"]["f"])
            de = xe.shape[1]
            lo, hi = shard.shard_bounds(de, WORLD, rank)
            Xe = torch.from_numpy(np.ascontiguousarray(xe[:, lo:hi])).cuda()
            if rec["func"] == "krum":
                row, idx = shard.krum(ops["gram"], ops["krum_select"], Xe, de, fe, exact=ops)
                out["exact_" + name] = (row.cpu().numpy(), idx)
            elif rec["func"] == "mom_krum":
                row, idx = shard.mom_krum(ops, Xe, de, fe)
                out["exact_" + name] = (row.cpu().numpy(), idx)
            else:
                out["exact_" + name] = (shard.bulyan(ops, Xe, de, fe, "krum").cpu().numpy(), -1)
        for name, xe in wide_nonfinite().items():
            lo, hi = shard.shard_bounds(d, WORLD, rank, align=256)
            Xe = torch.from_numpy(np.ascontiguousarray(xe[:, lo:hi])).cuda()
            _, idx = shard.krum(ops["gram"], ops["krum_select"], Xe, d, f, align=256, exact=ops)
            _, midx = shard.mom_krum(ops, Xe, d, f, align=256)
            out["wide_" + name] = (idx, midx, shard.bulyan(ops, Xe, d, f, "krum", align=256).cpu().numpy())
        torch.cuda.synchronize()
        results[rank] = out
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_rank_hip():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    results = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, results)) for r in range(WORLD)]
    try:
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
    finally:
        # a rank that failed leaves its peer blocked in a gloo collective:
        # end every rank still alive before judging the exit codes
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=30)
    codes = [p.exitcode for p in procs]
    assert all(c == 0 for c in codes), "HIP shard rank failed (exit codes %s)" % codes
    return dict(results)


@pytest.fixture(scope="module")
def unsharded():
    import torch
    import bench
    from srfl_amd import engine
    x, xc5 = _data()
    X = torch.from_numpy(x).cuda()
    f = SH["f"]
    want = {"trimmedmean": engine.trimmed_mean(X, 0.1).cpu().numpy()}
    want["trimmedmean_comm"] = want["trimmedmean"]
    row, order = engine.krum(X, f)
    want["krum_row"], want["krum_idx"] = row.cpu().numpy(), int(order.cpu()[0])
    row, order = engine.mom_krum(X, f)
    want["mom_krum_row"], want["mom_krum_idx"] = row.cpu().numpy(), int(order.cpu()[0])
    for mode in ("krum", "median", "trimmedmean"):
        want["bulyan_" + mode] = engine.bulyan(X, f, mode).cpu().numpy()
    for name, rec in exact_fixtures().items():
        Xe = torch.from_numpy(rec["x"]).cuda()
        fe = int(rec["params"]["f"])
        if rec["func"] == "krum":
            row, order = engine.krum(Xe, fe)
            want["exact_" + name] = (row.cpu().numpy(), int(order.cpu()[0]))
        elif rec["func"] == "mom_krum":
            row, order = engine.mom_krum(Xe, fe)
            want["exact_" + name] = (row.cpu().numpy(), int(order.cpu()[0]))
        else:
            want["exact_" + name] = (engine.bulyan(Xe, fe, "krum").cpu().numpy(), -1)
    for name, xe in wide_nonfinite().items():
        Xe = torch.from_numpy(xe).cuda()
        want["wide_" + name] = (int(engine.krum(Xe, f)[1].cpu()[0]), int(engine.mom_krum(Xe, f)[1].cpu()[0]),
                                engine.bulyan(Xe, f, "krum").cpu().numpy())
    fa = bench.FILTER_ARGS
    Xf = torch.from_numpy(xc5).cuda()
    want["c5"] = engine.mom_filter_l2(Xf, fa["eps"], fa["sigma"], fa["expansion"], fa["itv"],
                                      bench.MOM_DELTA).cpu().numpy()
    return want


@pytest.mark.parametrize("key", ["trimmedmean", "trimmedmean_comm", "krum_idx", "krum_row", "mom_krum_idx", "mom_krum_row",
                                 "bulyan_krum", "bulyan_median", "bulyan_trimmedmean", "c5"])
def test_two_ranks_equal_unsharded(two_rank_hip, unsharded, key):
    assert two_rank_hip[0]["c5_block"] > 0
    for r in range(WORLD):
        got = two_rank_hip[r][key]
        want = unsharded[key]
        if isinstance(want, int):
            assert got == want, "rank %d %s" % (r, key)
        else:
            np.testing.assert_array_equal(got, want, err_msg="rank %d %s" % (r, key))


@pytest.mark.parametrize("name", EXACT_FIXTURES)
def test_two_ranks_exact_route_fixtures(two_rank_hip, unsharded, name):
    """Krum / mom_krum / Bulyan-Krum on the live-reference NaN / inf fixtures,
    column-sharded over two ranks: the exact per-pair route over shards picks
    the reference's client (fixture `index` / `out`) and the unsharded
    engine's."""
    from conftest import load_fixture
    rec = load_fixture(os.path.join(HERE, "golden", name + ".npz"))
    want_out, want_idx = unsharded["exact_" + name]
    for r in range(WORLD):
        got_out, got_idx = two_rank_hip[r]["exact_" + name]
        assert got_idx == want_idx
        if "index" in rec:
            assert got_idx == int(rec["index"])
        np.testing.assert_array_equal(got_out, want_out)
        np.testing.assert_array_equal(got_out, rec["out"])


@pytest.mark.parametrize("name", ["nan", "inf"])
def test_two_ranks_exact_route_wide(two_rank_hip, unsharded, name):
    want = unsharded["wide_" + name]
    for r in range(WORLD):
        got = two_rank_hip[r]["wide_" + name]
        assert got[0] == want[0] and got[1] == want[1]
        np.testing.assert_array_equal(got[2], want[2])
