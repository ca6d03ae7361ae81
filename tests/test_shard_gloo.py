"""world_size-2 gloo tests of the d-sharding layer (srfl_amd/shard.py) on CPU.

The per-shard operations are the oracle's numpy restatements (the GPU ranks
pass the HIP entry points instead, shard.engine_ops()); what is tested here is
the sharding itself: balanced chunk-aligned bounds, the all-gather assembly,
filters restarting their chunking exactly where the unsharded path does, and
Krum from an all-reduced partial centred Gram."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _setup_paths():
    for p in (ROOT, HERE, os.path.join(HERE, "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import srfl_loader
    srfl_loader.load()


def _centred_gram(x):
    z = x.astype(np.float64) - x.astype(np.float64).mean(axis=0)
    return z @ z.T


def cpu_bulyan_ops():
    """The Bulyan per-shard operations restated on CPU tensors with the oracle
    (the GPU ranks use shard.engine_ops())."""
    import warnings
    from oracle import robust_np as orc

    def bulyan_round(X, rows, nr, aggsubfunc, agg):
        sub = X.numpy()[rows[:nr].numpy()]
        a = orc.trimmed_mean(list(sub)) if aggsubfunc == "trimmedmean" else orc.median(list(sub))
        a = np.asarray(a, dtype=np.float32)
        agg.copy_(torch.from_numpy(a))
        return torch.from_numpy(((sub.astype(np.float64) - a.astype(np.float64)) ** 2).sum(axis=1))

    def bulyan_pick(dvec, rows, nr, nxt, status=None):
        dv = dvec.numpy()
        best, bv = -1, np.inf
        for r in range(nr):
            if dv[r] < bv:
                best, bv = r, dv[r]
        if best < 0 and status is not None:
            status[0] = 1
        keep = [rows[r].item() for r in range(nr) if r != max(best, 0)]
        nxt[:nr - 1] = torch.tensor(keep, dtype=torch.int32)

    def bulyan_stage(S, beta):
        A = S.numpy().astype(np.float64)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            return torch.from_numpy(np.array([orc.bulyan_one_coordinate_leftfirst(A[:, j], beta)
                                              for j in range(A.shape[1])]))

    def krum_rounds(G, f, rounds):
        g = G.numpy()
        sq = np.diag(g)[:, None] + np.diag(g)[None, :] - 2 * g
        dd = np.sqrt(np.maximum(sq, 0)).astype(np.float32)
        alive, order = list(range(g.shape[0])), []
        for _ in range(rounds):
            sc = orc.krum_scores_from_dist(dd[np.ix_(alive, alive)], f)
            i = int(np.argmin(sc))
            order.append(alive.pop(i))
        return torch.tensor(order, dtype=torch.int32)

    return {"bulyan_round": bulyan_round, "bulyan_pick": bulyan_pick, "bulyan_stage": bulyan_stage,
            "gram": lambda X: torch.from_numpy(_centred_gram(X.numpy())), "krum_rounds": krum_rounds}


BULYAN_CASE = dict(n=30, d=257, f=5, seed=14, byz=5)


def cpu_exact_ops():
    """sra_krum_pair_sq_f32 / sra_krum_from_pairs restated with numpy: the
    class-coded fp64 sums of squared fp32 differences, and Krum scored from
    sqrt(fp32(sum)) (np.sort puts NaN last, np.argmin takes the first NaN)."""
    from oracle import robust_np as orc

    def pair_sq(X, bs=1):
        x = X.numpy()
        if bs > 1:
            nb = -(-x.shape[0] // bs)
            x = np.array(orc.bucket_means(list(x), bs, nb), dtype=np.float32)
        with np.errstate(all="ignore"):
            diff = (x[:, None, :] - x[None, :, :]).astype(np.float64)
            a = (diff * diff).sum(axis=-1)
        return torch.from_numpy(np.triu(a, 1))

    def krum_from_pairs(A, f, rounds):
        a = A.numpy()
        a = a + a.T
        with np.errstate(all="ignore"):
            dd = np.sqrt(a.astype(np.float32))
        alive, order = list(range(a.shape[0])), []
        for _ in range(rounds):
            sc = orc.krum_scores_from_dist(dd[np.ix_(alive, alive)], f)
            order.append(alive.pop(int(np.argmin(sc))))
        return torch.tensor(order, dtype=torch.int32)

    return {"pair_sq": pair_sq, "krum_from_pairs": krum_from_pairs}


def exact_cases():
    """(x, d, f) inputs for which the unsharded engine takes the exact route."""
    _setup_paths()
    from synth import make_rows
    nan = make_rows(24, 2000, seed=21, byz=4)
    nan[7, 1500] = np.nan
    inf = make_rows(24, 2000, seed=22, byz=4)
    inf[3, 10] = np.inf
    inf[9, 1900] = -np.inf
    narrow = make_rows(24, 777, seed=23, byz=4)
    narrow[12] = narrow[5] + np.float32(1e-7)      # a near tie the Gram cannot resolve
    return {"nan": (nan, 2000, 4), "inf": (inf, 2000, 4), "narrow": (narrow, 777, 4)}


def _worker(rank, world, port, results):
    _setup_paths()
    from srfl_amd import shard
    from oracle import robust_np as orc
    from synth import make_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        # coordinate-wise: trimmed mean / median over a ragged d
        n, d = 37, 1001
        x = make_rows(n, d, seed=11, byz=5)
        lo, hi = shard.shard_bounds(d, world, rank)
        Xs = torch.from_numpy(np.ascontiguousarray(x[:, lo:hi]))
        tm = shard.coordinatewise(lambda X: torch.from_numpy(np.asarray(orc.trimmed_mean(list(X.numpy())))),
                                  Xs, d)
        md = shard.coordinatewise(lambda X: torch.from_numpy(np.asarray(orc.median(list(X.numpy())))), Xs, d)
        out["trimmed"] = tm.numpy()
        out["median"] = md.numpy()
        # chunked filter: shards aligned to itv
        itv = 40
        xf = make_rows(24, 230, seed=12, byz=4)
        lo, hi = shard.shard_bounds(230, world, rank, align=shard.filter_align(itv))
        Xf = torch.from_numpy(np.ascontiguousarray(xf[:, lo:hi]))
        fl = shard.coordinatewise(lambda X: torch.from_numpy(orc.filterL2(list(X.numpy()), 0.2, 0.02, 20, itv)),
                                  Xf, 230, align=itv)
        out["filter"] = fl.numpy()
        # Krum from the all-reduced partial Gram
        xk = make_rows(30, 777, seed=13, byz=6)
        lo, hi = shard.shard_bounds(777, world, rank)
        Xk = torch.from_numpy(np.ascontiguousarray(xk[:, lo:hi]))

        def select(G, f):
            g = G.numpy()
            sq = np.diag(g)[:, None] + np.diag(g)[None, :] - 2 * g
            dd = np.sqrt(np.maximum(sq, 0)).astype(np.float32)
            return int(np.argmin(orc.krum_scores_from_dist(dd, f)))

        row, idx = shard.krum(lambda X: torch.from_numpy(_centred_gram(X.numpy())), select, Xk, 777, 6)
        out["krum_row"] = row.numpy()
        out["krum_idx"] = idx
        # mom_krum: all-reduced partial Gram of the bucket means, the chosen
        # bucket's mean formed per shard and all-gathered
        xm = make_rows(31, 777, seed=15, byz=9)
        Xm = torch.from_numpy(np.ascontiguousarray(xm[:, lo:hi]))

        def gram_buckets(X, bs):
            x = X.numpy()
            nb = -(-x.shape[0] // bs)
            return torch.from_numpy(_centred_gram(np.array(orc.bucket_means(list(x), bs, nb))))

        mops = {"gram_buckets": gram_buckets, "krum_select": select,
                "bucket_mean": lambda R: torch.from_numpy(np.asarray(orc.bucket_means(list(R.numpy()),
                                                                                     R.shape[0], 1)[0]))}
        row, idx = shard.mom_krum(mops, Xm, 777, 2)
        out["mom_krum_row"] = row.numpy()
        out["mom_krum_idx"] = idx
        # block-cyclic shard + pipelined in-place all-gather, ragged last round
        for block in (64, 96, 1001):
            cols = shard.cyclic_blocks(d, world, rank, block)
            Xc = torch.from_numpy(np.ascontiguousarray(np.concatenate([x[:, lo:hi] for lo, hi in cols], axis=1)
                                                       if cols else x[:, :0]))

            def tm_into(X, o):
                o.copy_(torch.from_numpy(np.asarray(orc.trimmed_mean(list(X.numpy())))))
            out["cyclic_%d" % block] = shard.pipelined_coordinatewise(tm_into, Xc, d, block).numpy().copy()
        # config C5's bench path: mom_filterL2 on a block-cyclic shard whose
        # blocks are whole itv-chunks (bench.filter_block), pipelined all-gather
        import bench
        itv, dl = 40, 160
        dt = dl * world
        xc5 = make_rows(24, dt, seed=14, byz=4)
        block = bench.filter_block(dl, 4, itv)
        cols = shard.cyclic_blocks(dt, world, rank, block)
        Xc5 = torch.from_numpy(np.ascontiguousarray(np.concatenate([xc5[:, lo:hi] for lo, hi in cols], axis=1)))

        def mom_into(X, o):
            o.copy_(torch.from_numpy(np.asarray(orc.mom_filterL2(list(X.numpy()), 0.2, 0.02, 20, itv,
                                                                 float(np.exp(-2.0)))).ravel()))
        mom_into.out_dtype = torch.float64
        out["c5_block"] = block
        out["c5"] = shard.pipelined_coordinatewise(mom_into, Xc5, dt, block).numpy().copy()
        # Bulyan: per-round all-reduce of the distance partials (median /
        # trimmed mean), all-reduced Gram (krum), local per-coordinate stage
        c = BULYAN_CASE
        xb = make_rows(c["n"], c["d"], seed=c["seed"], byz=c["byz"])
        lo, hi = shard.shard_bounds(c["d"], world, rank)
        Xb = torch.from_numpy(np.ascontiguousarray(xb[:, lo:hi]))
        for mode in ("krum", "median", "trimmedmean"):
            out["bulyan_" + mode] = shard.bulyan(cpu_bulyan_ops(), Xb, c["d"], c["f"], mode).numpy()
        # Krum's exact per-pair route over shards (NaN / inf clients, a narrow
        # layer): class-coded pair sums per shard, one reduce, scored once
        xops = cpu_exact_ops()
        for name, (xe, de, fe) in exact_cases().items():
            lo, hi = shard.shard_bounds(de, world, rank)
            Xe = torch.from_numpy(np.ascontiguousarray(xe[:, lo:hi]))
            _, idx = shard.krum(lambda X: torch.from_numpy(_centred_gram(X.numpy())), select, Xe, de, fe,
                                exact=xops)
            out["exact_" + name] = idx
        results[rank] = out
    finally:
        dist.destroy_process_group()


def _run(world):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    results = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, results)) for r in range(world)]
    try:
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=180)
    finally:
        for p in procs:          # a failed rank leaves its peers in a collective
            if p.is_alive():
                p.kill()
                p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs), "gloo worker failed: %s" % [p.exitcode for p in procs]
    return dict(results)


@pytest.fixture(scope="module")
def two_rank_results():
    return _run(2)


@pytest.fixture(scope="module")
def three_rank_results():
    return _run(3)


def test_cyclic_blocks_partition():
    _setup_paths()
    from srfl_amd import shard
    for d in (1, 7, 1000, 1001, 12345):
        for world in (1, 2, 3, 8):
            for block in (1, 64, 1000):
                cols = sorted(c for r in range(world) for c in shard.cyclic_blocks(d, world, r, block))
                assert cols[0][0] == 0 and cols[-1][1] == d
                assert all(a[1] == b[0] for a, b in zip(cols, cols[1:]))
                assert shard.cyclic_rounds(d, world, block) * world * block >= d


@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_cyclic_equals_unsharded(world, two_rank_results, three_rank_results):
    _setup_paths()
    from oracle import robust_np as orc
    from synth import make_rows
    res = two_rank_results if world == 2 else three_rank_results
    want = orc.trimmed_mean(list(make_rows(37, 1001, seed=11, byz=5)))
    for r in range(world):
        for block in (64, 96, 1001):
            np.testing.assert_array_equal(res[r]["cyclic_%d" % block], want)


@pytest.mark.parametrize("world", [2, 3])
def test_c5_pipelined_mom_filter_equals_unsharded(world, two_rank_results, three_rank_results):
    """bench.py's N > 1 path for config C5 (mom_filterl2): itv-aligned
    block-cyclic shards, the per-block filter, the overlapped all-gather --
    equal to the unsharded oracle over the whole matrix."""
    _setup_paths()
    from oracle import robust_np as orc
    from synth import make_rows
    res = two_rank_results if world == 2 else three_rank_results
    xc5 = make_rows(24, 160 * world, seed=14, byz=4)
    want = np.asarray(orc.mom_filterL2(list(xc5), 0.2, 0.02, 20, 40, float(np.exp(-2.0)))).ravel()
    for r in range(world):
        assert res[r]["c5_block"] == 40
        np.testing.assert_allclose(res[r]["c5"], want, rtol=1e-12, atol=1e-15)


def test_filter_block_is_itv_aligned():
    _setup_paths()
    import bench
    for d, chunks, itv in ((12_500_000, 16, 1000), (10_000_000, 16, 1000), (160, 4, 40), (1000, 16, 1000),
                           (999, 16, 1000)):
        b = bench.filter_block(d, chunks, itv)
        if b:
            assert d % b == 0 and b % itv == 0 and d // b <= chunks
        else:
            assert d % itv != 0


def test_shard_bounds_cover_and_align():
    _setup_paths()
    from srfl_amd import shard
    for d in (1, 7, 1000, 1001, 12345):
        for world in (1, 2, 3, 8):
            for align in (1, 64, 1000):
                b = shard.all_bounds(d, world, align)
                assert b[0][0] == 0 and b[-1][1] == d
                for (l0, h0), (l1, h1) in zip(b, b[1:]):
                    assert h0 == l1
                for lo, hi in b:
                    assert lo % align == 0 or lo == d
                widths = [hi - lo for lo, hi in b]
                assert max(widths) - min(widths) <= align


def test_sharded_coordinatewise_equals_unsharded(two_rank_results):
    _setup_paths()
    from oracle import robust_np as orc
    from synth import make_rows
    x = make_rows(37, 1001, seed=11, byz=5)
    for r in (0, 1):
        np.testing.assert_array_equal(two_rank_results[r]["trimmed"], orc.trimmed_mean(list(x)))
        np.testing.assert_array_equal(two_rank_results[r]["median"], orc.median(list(x)))


def test_sharded_filter_equals_unsharded(two_rank_results):
    _setup_paths()
    from oracle import robust_np as orc
    from synth import make_rows
    xf = make_rows(24, 230, seed=12, byz=4)
    want = orc.filterL2(list(xf), 0.2, 0.02, 20, 40)
    for r in (0, 1):
        np.testing.assert_allclose(two_rank_results[r]["filter"], want, rtol=1e-12, atol=1e-15)


def test_sharded_krum_equals_unsharded(two_rank_results):
    _setup_paths()
    from oracle import robust_np as orc
    from synth import make_rows
    xk = make_rows(30, 777, seed=13, byz=6)
    row, idx = orc.krum(list(xk), 6)
    for r in (0, 1):
        assert two_rank_results[r]["krum_idx"] == idx
        np.testing.assert_array_equal(two_rank_results[r]["krum_row"], row)


@pytest.mark.parametrize("case", ["nan", "inf", "narrow"])
def test_sharded_krum_exact_route(case, two_rank_results, three_rank_results):
    """A NaN client, +-inf clients and a narrow layer: the sharded Krum takes
    the exact per-pair route (shard.needs_exact on the summed Gram) and picks
    the reference's client with 2 and 3 column shards."""
    _setup_paths()
    from oracle import robust_np as orc
    x, d, f = exact_cases()[case]
    with np.errstate(all="ignore"):
        _, idx = orc.krum(list(x), f)
    for res in (two_rank_results, three_rank_results):
        for r in res:
            assert res[r]["exact_" + case] == idx


def test_needs_exact_triggers():
    _setup_paths()
    from srfl_amd import shard
    g = torch.eye(4, dtype=torch.float64)
    assert shard.needs_exact(g, 1024) and not shard.needs_exact(g, 1025)
    g[2, 2] = float("nan")
    assert shard.needs_exact(g, 5000)
    g = torch.eye(4, dtype=torch.float64) * 2e38
    assert shard.needs_exact(g, 5000)


def test_sharded_mom_krum_equals_unsharded(two_rank_results):
    _setup_paths()
    from oracle import robust_np as orc
    from synth import make_rows
    xm = make_rows(31, 777, seed=15, byz=9)
    want = orc.mom_krum(list(xm), 2)
    bm = orc.bucket_means(list(xm), 3, 11)
    for r in (0, 1):
        np.testing.assert_array_equal(two_rank_results[r]["mom_krum_row"], want)
        np.testing.assert_array_equal(bm[two_rank_results[r]["mom_krum_idx"]], want)


@pytest.mark.parametrize("mode", ["krum", "median", "trimmedmean"])
def test_sharded_bulyan_equals_unsharded(mode, two_rank_results, three_rank_results):
    """Same selection and the same per-coordinate results with 2 and 3 column
    shards as unsharded (world 1, no process group), and the reference-equivalent
    oracle within fp64 rounding."""
    _setup_paths()
    import warnings
    from srfl_amd import shard
    from oracle import robust_np as orc
    from synth import make_rows
    c = BULYAN_CASE
    xb = make_rows(c["n"], c["d"], seed=c["seed"], byz=c["byz"])
    want = shard.bulyan(cpu_bulyan_ops(), torch.from_numpy(xb), c["d"], c["f"], mode).numpy()
    for res in (two_rank_results, three_rank_results):
        for r in res:
            np.testing.assert_array_equal(res[r]["bulyan_" + mode], want)
    rows = [r for r in xb]
    sel, _ = orc.bulyan_select(rows, c["f"], mode)
    S = np.array([np.asarray(g, dtype=np.float64).ravel() for g in sel])
    beta = S.shape[0] - 2 * c["f"]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref = np.array([orc.bulyan_one_coordinate_leftfirst(S[:, j], beta) for j in range(S.shape[1])])
    np.testing.assert_allclose(want, ref, rtol=1e-12, atol=1e-15)


def test_sharded_bulyan_theta_error():
    _setup_paths()
    from srfl_amd import shard
    with pytest.raises(IndexError):
        shard.bulyan(cpu_bulyan_ops(), torch.zeros(10, 4), 4, 5, "median")


def test_sharded_bulyan_nonfinite_raises():
    """A NaN coordinate makes the median-mode round's aggregate NaN in that
    column, so every distance is NaN and the reference's `assert min_index !=
    None` (robust_estimator.py:308/321) fires: the sharded path raises the
    same AssertionError from the pick's status flag."""
    _setup_paths()
    import warnings
    from srfl_amd import shard
    x = torch.randn(12, 9)
    x[3, 4] = float("nan")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        with pytest.raises(AssertionError):
            shard.bulyan(cpu_bulyan_ops(), x, 9, 2, "median")
