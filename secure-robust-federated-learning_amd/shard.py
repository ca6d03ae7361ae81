"""Multi-GPU sharding of the aggregation path.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
The gradient dimension d of a layer is split into contiguous column blocks;
each rank reads only its N x d_r block:

* coordinate-wise aggregators (average / median / trimmed mean, the Bulyan
  per-coordinate stage, bucket means) and the chunked spectral filters are
  independent per column (per itv-chunk for the filters, so filter shards are
  aligned to itv and restart chunking exactly where the single-GPU path
  does): every rank aggregates its block and one all-gather assembles the
  d-vector — no other data-path collective;
* Krum (and the Krum rounds of Bulyan-Krum) needs the N x N client Gram: the
  centred Gram decomposes over columns (each column is centred by its own
  mean), so each rank computes the Gram of its block and one reduce of N*N
  fp64 (128 KiB at N=128) sums them on rank 0, which alone scores the N x N
  matrix (the score matrix stays on one GPU) and broadcasts the chosen
  index(es); the chosen client's row is assembled with the same all-gather.
  Where the unsharded engine takes its exact per-pair route (a NaN / inf
  client, a squared distance beyond fp32's range, or d <= 1024), so does the
  sharded one: ||a - b||^2 is a sum over column shards, so every rank forms
  its class-coded pair sums and a second reduce sums them for the scoring
  rank (``_krum_order``);
* Bulyan's median / trimmed-mean selection rounds: one all-reduce of the
  <= N fp64 distance partials per round (the only per-round exchange), the
  pick made identically on every rank, then the local per-coordinate stage.

The helpers take the per-shard operations as arguments so that the sharding
logic is exercised by world_size-2 gloo tests on CPU; the GPU path passes the
engine's HIP entry points (see ``engine_ops``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(d, world, rank, align=1):
    """[lo, hi) columns of ``rank``: balanced over ceil(d/align) units of
    ``align`` columns (the last unit may be partial)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank %d/%d" % (world, rank))
    align = max(1, int(align))
    units = -(-int(d) // align)
    lo_u = rank * units // world
    hi_u = (rank + 1) * units // world
    return min(d, lo_u * align), min(d, hi_u * align)


def all_bounds(d, world, align=1):
    return [shard_bounds(d, world, r, align) for r in range(world)]


def _world(group):
    if not dist.is_initialized():   # a single process: the unsharded layer
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


# Collectives.  A gloo group over GPU ranks (several ranks sharing one GPU, as
# the two-rank execution test of tests/test_gpu_shard2.py runs them; RCCL
# refuses two ranks on one device) stages device tensors through host memory;
# an RCCL group takes the device tensors directly.
def _staged(t, group):
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _all_gather_into(out, inp, group=None):
    if _staged(inp, group):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _all_reduce(t, group=None):
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


def _reduce(t, dst, group=None):
    if _staged(t, group):
        h = t.cpu()
        dist.reduce(h, dst=dst, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.reduce(t, dst=dst, op=dist.ReduceOp.SUM, group=group)


def _broadcast(t, src, group=None):
    if _staged(t, group):
        h = t.cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src=src, group=group)


def gather_columns(local, d, align=1, group=None):
    """All-gather per-rank column blocks (1-D ``local`` of length hi-lo, or
    2-D with columns last) into the full d-vector on every rank."""
    world, rank = _world(group)
    bounds = all_bounds(d, world, align)
    width = max(hi - lo for lo, hi in bounds)
    lo, hi = bounds[rank]
    if local.shape[-1] != hi - lo:
        raise ValueError("rank %d holds %d columns, expected %d" % (rank, local.shape[-1], hi - lo))
    lead = local.shape[:-1]
    padded = torch.zeros(lead + (width,), dtype=local.dtype, device=local.device)
    padded[..., :hi - lo] = local
    if not dist.is_initialized():
        return padded[..., :d].clone()
    gathered = torch.empty((world,) + lead + (width,), dtype=local.dtype, device=local.device)
    _all_gather_into(gathered, padded.unsqueeze(0).contiguous(), group)
    parts = [gathered[r][..., :bh - bl] for r, (bl, bh) in enumerate(bounds)]
    return torch.cat(parts, dim=-1)


def coordinatewise(local_fn, X_shard, d, align=1, group=None):
    """Coordinate-wise (or per-chunk) aggregation of a column-sharded layer:
    ``local_fn(X_shard) -> (hi-lo,)`` on this rank, then one all-gather."""
    return gather_columns(local_fn(X_shard), d, align, group)


# krum.hip kExactMaxD: layers this narrow always take the exact per-pair route
EXACT_MAX_D = 1024


def needs_exact(G, d):
    """sra_krum_select_f32's switch to the exact per-pair route, evaluated on
    the (summed) centred Gram: a narrow layer (d <= 1024), a non-finite
    diagonal entry (a NaN / inf client; the centring spreads it over every
    entry) or a squared distance G_ii + G_jj - 2 G_ij beyond fp32's range
    (krum.hip krum_dist_kernel)."""
    if d <= EXACT_MAX_D:
        return True
    dg = G.diagonal()
    if not bool(torch.isfinite(dg).all()):
        return True
    sq = dg[:, None] + dg[None, :] - 2.0 * G
    return bool((sq > 3.0e38).any())


def _krum_order(G, X_shard, d, f, rounds, group=None, exact=None, bucket_size=1):
    """The Krum selection order (``rounds`` picks) of a column-sharded layer,
    on every rank.

    The ranks' partial centred Grams ``G`` are summed on the group's first
    rank, which decides the route as the unsharded engine does
    (``needs_exact``) and broadcasts it.  Gram route: that rank scores the
    summed Gram (``exact["krum_rounds"]``).  Exact route (robust_estimator.py:
    242 computes every distance from the rows): every rank forms the class-
    coded pair sums of its own columns (``exact["pair_sq"](X_shard,
    bucket_size)``, sra_krum_pair_sq_f32 -- NaN / inf coded in place, so the
    fp64 sum of the ranks' partials keeps the reference's NaN / inf classes),
    a second reduce sums them on the first rank, which scores them
    (``exact["krum_from_pairs"]``).  Either way the N x N scoring stays on one
    GPU and one broadcast hands the order to every rank.  Without ``exact``
    ops the Gram route is always taken."""
    on = dist.is_initialized()
    _, rank = _world(group)
    root = (dist.get_global_rank(group, 0) if group is not None else 0) if on else 0
    if on:
        _reduce(G, root, group)
    flag = torch.zeros(1, dtype=torch.int32, device=G.device)
    if rank == 0 and exact is not None and "pair_sq" in exact:
        flag.fill_(1 if needs_exact(G, d) else 0)
    if on:
        _broadcast(flag, root, group)
    idx = torch.zeros(rounds, dtype=torch.int64, device=G.device)
    if int(flag.item()):
        A = exact["pair_sq"](X_shard, bucket_size).to(torch.float64).contiguous()
        if on:
            _reduce(A, root, group)
        if rank == 0:
            idx.copy_(torch.as_tensor(exact["krum_from_pairs"](A, f, rounds), device=G.device)
                      .reshape(rounds).to(torch.int64))
    elif rank == 0:
        idx.copy_(torch.as_tensor(exact["krum_rounds"](G, f, rounds), device=G.device).reshape(rounds).to(torch.int64))
    if on:
        _broadcast(idx, root, group)
    return idx


def krum(gram_fn, select_fn, X_shard, d, f, group=None, align=1, exact=None):
    """Krum over a column-sharded layer.

    gram_fn(X_shard) -> (N, N) float64 partial centred Gram;
    select_fn(G, f) -> index of the chosen client (from the full Gram).
    exact (optional): {"pair_sq", "krum_from_pairs"} -- the exact per-pair
    route of ``_krum_order``, taken where sra_krum_select_f32 takes it
    unsharded (NaN / inf clients, fp32-overflowing or d <= 1024), so the pick
    equals the single-GPU engine's and the reference's there too.
    Returns (full row of the chosen client, index)."""
    G = gram_fn(X_shard).to(torch.float64).contiguous()
    ops = dict(exact or {})
    ops["krum_rounds"] = lambda g, ff, rounds: torch.tensor([int(select_fn(g, ff))])
    # (a 1-rank group still goes through the collectives)
    idx = int(_krum_order(G, X_shard, d, f, 1, group, ops)[0])
    row = gather_columns(X_shard[idx], d, align, group)
    return row, idx


def mom_krum(ops, X_shard, d, f, bucket_size=3, group=None, align=1):
    """mom_krum (robust_estimator.py:250-256) over a column-sharded layer.

    The centred Gram of the bucket means decomposes over columns like Krum's:
    each rank forms its partial from its own columns without writing the means
    (``ops["gram_buckets"]``), one reduce of B x B doubles sums them on the
    first rank, which picks the bucket (``ops["krum_select"]``) and broadcasts
    it, and the bucket's mean
    over each rank's columns (``ops["bucket_mean"]``, np.mean order) is
    all-gathered.  Returns (full mean row of the chosen bucket, bucket index)."""
    n = int(X_shard.shape[0])
    G = ops["gram_buckets"](X_shard, bucket_size).to(torch.float64).contiguous()
    kops = {k: ops[k] for k in ("pair_sq", "krum_from_pairs") if k in ops}
    kops["krum_rounds"] = lambda g, ff, rounds: torch.tensor([int(ops["krum_select"](g, ff))])
    idx = int(_krum_order(G, X_shard, d, f, 1, group, kops, bucket_size)[0])
    lo = idx * bucket_size
    part = ops["bucket_mean"](X_shard[lo:min(lo + bucket_size, n)])
    return gather_columns(part, d, align, group), idx


def bulyan(ops, X_shard, d, f, aggsubfunc="trimmedmean", group=None, align=1):
    """Bulyan (robust_estimator.py:277-332) over a column-sharded layer.

    The theta selection rounds need the distance of every remaining client to
    the round's aggregate over ALL columns: each rank computes the aggregate
    and the distances over its own columns (``ops["bulyan_round"]``), one
    all-reduce of <= N fp64 partials per round sums them, and every rank
    makes the same pick (``ops["bulyan_pick"]``) from the identical sums.
    Krum mode: one reduce of the partial centred Gram to the first rank, which
    runs the theta Krum rounds (``ops["krum_rounds"]``) and broadcasts the
    order.  The
    per-coordinate stage is local (``ops["bulyan_stage"]``) and one all-gather
    assembles the (d,) float64 result.

    ops: bulyan_round(X, rows, nr, aggsubfunc, agg_out) -> dist (nr,) float64;
         bulyan_pick(dist, rows, nr, rows_next, status) (status[0] = 1 when no
         distance is finite); bulyan_stage(S, beta) -> (w,);
         gram(X) -> (N, N) float64; krum_rounds(G, f, rounds) -> (rounds,) indices."""
    n = int(X_shard.shape[0])
    theta = n - 2 * int(f)
    if theta <= 0:
        # the reference indexes the empty selection (np_grads[0]): IndexError
        raise IndexError("bulyan needs theta = N - 2f > 0 (N=%d, f=%d)" % (n, f))
    beta = theta - 2 * int(f)
    on = dist.is_initialized()   # (a 1-rank group still goes through the collectives)
    if aggsubfunc == "krum":
        G = ops["gram"](X_shard).to(torch.float64).contiguous()
        order = _krum_order(G, X_shard, d, int(f), theta, group, ops)
        S = X_shard.index_select(0, order.to(torch.long)).contiguous()
    else:
        if aggsubfunc not in ("median", "trimmedmean"):
            raise ValueError("aggsubfunc must be krum, median or trimmedmean")
        S = torch.empty((theta, X_shard.shape[1]), dtype=torch.float32, device=X_shard.device)
        rows = torch.arange(n, dtype=torch.int32, device=X_shard.device)
        nxt = torch.empty_like(rows)
        # set to 1 by a pick that finds no finite minimum (every distance NaN /
        # inf); checked once after the rounds (one host sync)
        status = torch.zeros(1, dtype=torch.int32, device=X_shard.device)
        for t in range(theta):
            nr = n - t
            dvec = ops["bulyan_round"](X_shard, rows, nr, aggsubfunc, S[t])
            if on:
                _all_reduce(dvec, group)
            ops["bulyan_pick"](dvec, rows, nr, nxt, status)
            rows, nxt = nxt, rows
        if int(status.item()) != 0:
            # robust_estimator.py:318: `assert selected_idx >= 0` when no
            # distance is finite (a NaN / inf client in every round's reach)
            raise AssertionError("bulyan: no finite distance in a selection round (non-finite client update)")
    return gather_columns(ops["bulyan_stage"](S, beta), d, align, group)


# ---------------------------------------------------------------------------
# block-cyclic sharding with a pipelined, overlapped all-gather
# ---------------------------------------------------------------------------
def cyclic_blocks(d, world, rank, block):
    """Global column ranges owned by ``rank`` under block-cyclic sharding:
    global block g = [g*block, min((g+1)*block, d)) belongs to rank g % world.
    Returned in the rank's local order (local block k = global block
    k*world + rank)."""
    if world < 1 or not 0 <= rank < world or block < 1:
        raise ValueError("bad world/rank/block %d/%d/%d" % (world, rank, block))
    nb = -(-int(d) // int(block))
    return [(g * block, min((g + 1) * block, d)) for g in range(rank, nb, world)]


def cyclic_rounds(d, world, block):
    """Number of all-gather rounds (one global block per rank per round)."""
    nb = -(-int(d) // int(block))
    return -(-nb // world)


def pipelined_coordinatewise(local_fn, X_local, d, block, group=None, out=None, comm_stream=None):
    """Coordinate-wise (or per-chunk) aggregation of a block-cyclic shard with
    the all-gather of block k overlapped with the aggregation of block k+1.

    ``X_local``: (N, sum of widths) -- this rank's blocks (``cyclic_blocks``)
    side by side.  ``local_fn(X_cols, out_view)`` aggregates one block into
    ``out_view`` (1-D, that block's width).  Round k's results land in
    ``full[k*world*block + rank*block ...]`` -- exactly their global positions,
    so each round is one IN-PLACE all-gather of ``world*block`` elements and no
    reordering copy follows.  On a GPU the collectives run on ``comm_stream``
    (RCCL over xGMI), ordered after the block's aggregation by an event; the
    aggregation of the next block proceeds concurrently on the current stream.
    Returns the (d,) aggregate on every rank."""
    world, rank = _world(group)
    on = dist.is_initialized()
    rounds = cyclic_rounds(d, world, block)
    span = world * block
    full = out
    if full is None or full.numel() < rounds * span:
        full = torch.empty(rounds * span, dtype=_out_dtype(local_fn, X_local), device=X_local.device)
    mine = cyclic_blocks(d, world, rank, block)
    cuda = X_local.is_cuda and on
    compute = torch.cuda.current_stream(X_local.device) if cuda else None
    if cuda and comm_stream is None:
        comm_stream = torch.cuda.Stream(device=X_local.device)
    off = 0
    for k in range(rounds):
        seg = full[k * span + rank * block: k * span + (rank + 1) * block]
        if k < len(mine):
            lo, hi = mine[k]
            local_fn(X_local[:, off:off + hi - lo], seg[:hi - lo])
            off += hi - lo
        if not on:
            continue
        if cuda:
            ev = torch.cuda.Event()
            ev.record(compute)
            with torch.cuda.stream(comm_stream):
                comm_stream.wait_event(ev)
                _all_gather_into(full[k * span:(k + 1) * span], seg, group)
        else:
            _all_gather_into(full[k * span:(k + 1) * span], seg, group)
    if cuda:
        compute.wait_stream(comm_stream)
        full.record_stream(comm_stream)
    return full[:d]


def _out_dtype(local_fn, X):
    return getattr(local_fn, "out_dtype", X.dtype)


def engine_ops():
    """The HIP-backed per-shard operations (GPU ranks)."""
    from . import engine

    def gram_fn(X):
        return engine.gram(X)

    def select_fn(G, f):
        order, _ = engine.krum_from_gram(G, f, 1)
        return int(order[0].item())

    def bulyan_round(X, rows, nr, aggsubfunc, agg):
        dvec = torch.empty(nr, dtype=torch.float64, device=X.device)
        engine.bulyan_round(X, rows, nr, aggsubfunc, agg, dvec)
        return dvec

    def krum_rounds(G, f, rounds):
        order, _ = engine.krum_from_gram(G, f, rounds, scores=False)
        return order

    return {
        "bulyan_round": bulyan_round,
        "bulyan_pick": lambda dvec, rows, nr, nxt, status=None: engine.bulyan_pick(dvec, rows, nr, nxt, status),
        "bulyan_stage": lambda S, beta: engine.bulyan_stage(S, beta),
        "krum_rounds": krum_rounds,
        "average": lambda X: engine.average(X),
        "median": lambda X: engine.median(X),
        "trimmedmean": lambda X: engine.trimmed_mean(X, 0.1),
        "gram": gram_fn,
        "gram_buckets": lambda X, bs: engine.gram_buckets(X, bs),
        "bucket_mean": lambda R: engine.bucket_means(R, int(R.shape[0]), 1)[0],
        "krum_select": select_fn,
        # the exact per-pair route (_krum_order)
        "pair_sq": lambda X, bs=1: engine.krum_pair_sq(X, bs),
        "krum_from_pairs": lambda A, f, rounds: engine.krum_from_pairs(A, f, rounds, scores=False)[0],
        # (X_cols, out_view) forms for pipelined_coordinatewise
        "average_into": lambda X, o: engine.average(X, out=o),
        "median_into": lambda X, o: engine.median(X, out=o),
        "trimmedmean_into": lambda X, o: engine.trimmed_mean(X, 0.1, out=o),
    }


def filter_align(itv):
    """Filter shards must hold whole itv-chunks (robust_estimator.py:116-125)."""
    return int(itv)
