"""Multi-GPU sharding of the aggregation path.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
The gradient dimension d of a layer is split into contiguous column blocks;
each rank reads only its N x d_r block:

* coordinate-wise aggregators (average / median / trimmed mean, the Bulyan
  final stage, bucket means) and the chunked spectral filters are
  independent per column (per itv-chunk for the filters, so filter shards are
  aligned to itv and restart chunking exactly where the single-GPU path
  does): every rank aggregates its block and one all-gather assembles the
  d-vector — no other data-path collective;
* Krum (and the Krum rounds of Bulyan-Krum) needs the N x N client Gram: the
  centred Gram decomposes over columns (each column is centred by its own
  mean), so each rank computes the Gram of its block and one all-reduce of
  N*N fp64 (128 KiB at N=128) sums them; scoring is N-space work done
  redundantly on every rank (identical inputs -> identical index), and the
  chosen client's row is assembled with the same all-gather.

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
    return dist.get_world_size(group), dist.get_rank(group)


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
    if world == 1:
        return padded[..., :d].clone()
    gathered = torch.empty((world,) + lead + (width,), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(gathered, padded.unsqueeze(0).contiguous(), group=group)
    parts = [gathered[r][..., :bh - bl] for r, (bl, bh) in enumerate(bounds)]
    return torch.cat(parts, dim=-1)


def coordinatewise(local_fn, X_shard, d, align=1, group=None):
    """Coordinate-wise (or per-chunk) aggregation of a column-sharded layer:
    ``local_fn(X_shard) -> (hi-lo,)`` on this rank, then one all-gather."""
    return gather_columns(local_fn(X_shard), d, align, group)


def krum(gram_fn, select_fn, X_shard, d, f, group=None, align=1):
    """Krum over a column-sharded layer.

    gram_fn(X_shard) -> (N, N) float64 partial centred Gram;
    select_fn(G, f) -> index of the chosen client (from the full Gram).
    Returns (full row of the chosen client, index)."""
    G = gram_fn(X_shard).to(torch.float64).contiguous()
    world, _ = _world(group)
    if world > 1:
        dist.all_reduce(G, op=dist.ReduceOp.SUM, group=group)
    idx = int(select_fn(G, f))
    row = gather_columns(X_shard[idx], d, align, group)
    return row, idx


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
    world, rank = _world(group) if dist.is_initialized() else (1, 0)
    rounds = cyclic_rounds(d, world, block)
    span = world * block
    full = out
    if full is None or full.numel() < rounds * span:
        full = torch.empty(rounds * span, dtype=_out_dtype(local_fn, X_local), device=X_local.device)
    mine = cyclic_blocks(d, world, rank, block)
    cuda = X_local.is_cuda and world > 1
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
        if world == 1:
            continue
        if cuda:
            ev = torch.cuda.Event()
            ev.record(compute)
            with torch.cuda.stream(comm_stream):
                comm_stream.wait_event(ev)
                dist.all_gather_into_tensor(full[k * span:(k + 1) * span], seg, group=group)
        else:
            dist.all_gather_into_tensor(full[k * span:(k + 1) * span], seg, group=group)
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

    return {
        "average": lambda X: engine.average(X),
        "median": lambda X: engine.median(X),
        "trimmedmean": lambda X: engine.trimmed_mean(X, 0.1),
        "gram": gram_fn,
        "krum_select": select_fn,
        # (X_cols, out_view) forms for pipelined_coordinatewise
        "average_into": lambda X, o: engine.average(X, out=o),
        "median_into": lambda X, o: engine.median(X, out=o),
        "trimmedmean_into": lambda X, o: engine.trimmed_mean(X, 0.1, out=o),
    }


def filter_align(itv):
    """Filter shards must hold whole itv-chunks (robust_estimator.py:116-125)."""
    return int(itv)
