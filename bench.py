#!/usr/bin/env python3
"""Benchmark: aggregated-gradient GB/s (device-resident N x d fp32) on MI355X.

Default workload (BASELINE.json north star): coordinate-wise trimmed mean over
N=128 clients x d=1e8 fp32 per GPU, i.e. 51.2 GB of client updates resident
in HBM per GPU.  One "step" = one aggregation call over the whole N x d
matrix.  With --gpus > 1 (torch.distributed.run, one rank per GPU) the
gradient dimension is sharded: every rank aggregates its own d-shard (fixed
per-GPU work -> weak scaling) and the aggregate is assembled on every rank by
one RCCL all-gather over xGMI, which is part of the timed step.

value = N * d_total * 4 bytes / (max over ranks of the timed region) in GB/s.

Extra fields on the JSON line:
  roofline     — dominant kernel (the k-select) timed with HIP events on the
                 launch stream; achieved = algorithmic bytes per launch
                 (4*N*d + 4*d) / average launch duration; peak = 8000 GB/s.
  cpu_baseline — the numpy restatement of robust_estimator.trimmed_mean
                 (oracle/robust_np.py, kind "port") timed on this host on a
                 bounded sample (rank 0, N=1 only).
  host_inclusive — H2D + kernel + D2H rate from pinned host memory (the
                 simulator hands host arrays over); never `value`.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch  # importing torch does not initialise the GPU; libsra is loaded in main()
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
engine = shard = None   # srfl_amd modules, bound by _load_engine() once this process is a bench rank


def _load_engine():
    global engine, shard
    if engine is not None:
        return
    import srfl_loader
    srfl_loader.load()
    from srfl_amd import engine as _e, shard as _s
    engine, shard = _e, _s

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--agg", default="trimmedmean",
                    choices=["trimmedmean", "median", "average", "krum", "mom_krum", "bulyankrum", "bulyanmedian",
                             "bulyantrimmedmean", "filterl2", "ex_noregret", "mom_filterl2", "mom_ex_noregret",
                             "dba_median", "dba_weighted_sum"])
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--d", type=float, default=1e8, help="coordinates per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--chunks", type=int, default=16,
                    help="N>1: all-gather rounds per step (block-cyclic shard, gather of block k "
                         "overlapped with the aggregation of block k+1)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 PMC (written by tools/pmc_traffic.py)")
    ap.add_argument("--byzantine", type=int, default=20,
                    help="f Byzantine rows of the synthetic input (SURVEY.md §8(d)); 0 = benign only")
    ap.add_argument("--launch-check", action="store_true",
                    help="test hook: every rank joins a gloo group, prints its rank / world size and exits "
                         "(no GPU use); exercises the --gpus launcher on CPU")
    return ap.parse_args()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def ranks_or_launch(a):
    """--gpus N is honoured or the run fails: without WORLD_SIZE in the
    environment and N > 1, start N ranks as ONE child process
    (python -m torch.distributed.run, rendezvous on 127.0.0.1) and return its
    exit code -- this happens before anything touches the GPU, and the parent
    never execs; with WORLD_SIZE set it must equal N.  Returns None when this
    process is a rank that should run the bench."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if a.gpus <= 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.call(cmd)
    if int(env_world) != a.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d: launch one rank per GPU with --gpus equal to the world size"
              % (env_world, a.gpus), file=sys.stderr, flush=True)
        return 2
    return None


def launch_check(a):
    """--launch-check: one gloo collective over the ranks the launcher started."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([1.0])
    if world > 1:
        dist.all_reduce(t)
        world = dist.get_world_size()
    print(json.dumps({"rank": rank, "world_size": world, "ranks_seen": int(t.item()), "gpus": a.gpus}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def synthetic_rows(n, d, byz, seed, device):
    """SURVEY.md §8(d) synthetic updates, generated on the device: 0.01 N(0,1)
    per client plus a shared 0.001 N(0,1) drift; rows < byz Byzantine at -10x
    the benign mean plus 0.001 N(0,1) noise (the generator of the full-size
    filter / Krum / Bulyan parity tests, tests/test_gpu_filters.py)."""
    g = torch.Generator(device=device).manual_seed(seed)
    X = torch.empty((n, d), dtype=torch.float32, device=device)
    cols = max(1, int(1e9 // (8 * max(n, 1))))        # fp64 column-block of <= 1 GB for the benign mean
    drift = torch.empty(min(d, cols), dtype=torch.float32, device=device)
    for j0 in range(0, d, cols):
        j1 = min(d, j0 + cols)
        dv = drift[:j1 - j0].normal_(0.0, 0.001, generator=g)
        blk = X[:, j0:j1]
        blk.normal_(0.0, 0.01, generator=g).add_(dv)
        if byz:
            mean = blk[byz:].double().mean(0)
            blk[:byz] = (-10.0 * mean).float()[None, :] + 0.001 * torch.randn(byz, j1 - j0, device=device,
                                                                                 generator=g)
    return X


def _krum_step(X, out):
    row, order = engine.krum(X, 20)
    out.copy_(row)


def _mom_krum_step(X, out):
    row, order = engine.mom_krum(X, 20)
    out.copy_(row)


def _bulyan_step(mode):
    def step(X, out):
        out.copy_(engine.bulyan(X, 20, mode, check=False))
    return step


# simulate.py defaults (SURVEY.md §8 convention): f=20, eps=0.2, sigma=1e-5,
# expansion=20, itv=1000; for MoM the delta of config C5 (e^-26).
FILTER_ARGS = dict(eps=0.2, sigma=1e-5, expansion=20, itv=1000)
MOM_DELTA = 2.718281828459045 ** -26


def _filter_step(name, mom=False):
    def step(X, out):
        fn = getattr(engine, name)
        if mom:
            out.copy_(fn(X, delta=MOM_DELTA, check=False, **FILTER_ARGS))
        else:
            out.copy_(fn(X, check=False, **FILTER_ARGS))
    return step


_WEIGHTS = {}


def _dba_weighted_step(X, out):
    """DBA Helper.weighted_average_oracle (geometric median's inner step)."""
    n = int(X.shape[0])
    w = _WEIGHTS.get(n)
    if w is None:
        w = _WEIGHTS[n] = torch.full((n,), 1.0 / n, dtype=torch.float32, device=X.device)
    engine.weighted_sum(X, w, out=out)


AGG = {
    "dba_median": lambda X, out: engine.order_stat(X, (int(X.shape[0]) - 1) // 2, out=out),
    "dba_weighted_sum": _dba_weighted_step,
    "trimmedmean": lambda X, out: engine.trimmed_mean(X, 0.1, out=out),
    "median": lambda X, out: engine.median(X, out=out),
    "average": lambda X, out: engine.average(X, out=out),
    "krum": _krum_step,
    "mom_krum": _mom_krum_step,
    "bulyankrum": _bulyan_step("krum"),
    "bulyanmedian": _bulyan_step("median"),
    "bulyantrimmedmean": _bulyan_step("trimmedmean"),
    "filterl2": _filter_step("filter_l2"),
    "ex_noregret": _filter_step("ex_noregret"),
    "mom_filterl2": _filter_step("mom_filter_l2", mom=True),
    "mom_ex_noregret": _filter_step("mom_ex_noregret", mom=True),
}
OUT_DTYPE = {"bulyankrum": torch.float64, "bulyanmedian": torch.float64, "bulyantrimmedmean": torch.float64,
             "filterl2": torch.float64, "ex_noregret": torch.float64, "mom_filterl2": torch.float64,
             "mom_ex_noregret": torch.float64}
KERNEL_NAME = {
    "dba_median": "select_reg_kernel<128, kOrder> (lower median, DBA Helper.median)",
    "dba_weighted_sum": "rows_vec4_kernel<true> (DBA weighted_average_oracle)",
    "trimmedmean": "select_plain_kernel<1, 128, 12>",
    "median": "select_plain_kernel<0, 128, 0>",
    "average": "average_vec4_kernel",
    "krum": "whole krum op (bf16x3 gram_glds_kernel dominant; per-kernel split in profiles/)",
    "mom_krum": "whole mom_krum op (gram_bucket_kernel: bucket means fused into the bf16x3 Gram + scoring)",
    "bulyankrum": "whole bulyan op (bf16x3 Gram + theta Krum rounds + final stage)",
    "bulyanmedian": "whole bulyan op (theta fused select+distance rounds + final stage)",
    "bulyantrimmedmean": "whole bulyan op (theta fused select+distance rounds + final stage)",
    "filterl2": "whole filterL2 op (chunk_gram_kernel fp64 MFMA + wave_solve_kernel<0>, listed chunks on "
                "filter_solve_kernel<0> + chunk_mean_kernel)",
    "ex_noregret": "whole ex_noregret op (chunk Gram + noregret_pre_kernel + wave_solve_kernel<1> + chunk means)",
    "mom_filterl2": "whole op (chunk Gram with the bucket means formed in its loads + wave_solve_kernel<0> / "
                    "filter_solve_kernel<0> fallback + chunk means)",
    "mom_ex_noregret": "whole op (chunk Gram with the bucket means formed in its loads + noregret_pre_kernel + "
                       "wave_solve_kernel<1> + chunk means)",
}


def kernel_label(agg, n):
    """Name of the dominant kernel for the configuration actually launched."""
    if agg in ("trimmedmean", "median") and n > 128:
        mode = 1 if agg == "trimmedmean" else 0
        if n == 512:
            return "select_quad_kernel<4, %d, 512, %d>" % (mode, 51 if mode else -1)
        return "select_quad_kernel<%d, %d>" % (2 if n <= 256 else 4, mode)
    if agg == "trimmedmean" and n == 100:
        return "select_plain_kernel<1, 100, 10>"
    if agg == "median" and n == 100:
        return "select_plain_kernel<0, 100, 0>"
    return KERNEL_NAME[agg]


MFMA_PEAK_TFLOPS = 157.3      # fp32 MFMA (MI355X_MICROARCH.md)
MFMA64_PEAK_TFLOPS = 78.6     # fp64 MFMA


def roofline_model(agg, n, d):
    """(bound, peak, unit, algorithmic amount per launch) — SURVEY.md §8(d)."""
    if agg in ("trimmedmean", "median", "average", "dba_median", "dba_weighted_sum"):
        return "hbm", HBM_PEAK_GBS, "GB/s", 4 * n * d + 4 * d
    # Krum family: the Gram runs on the bf16 MFMA with a three-way split (six
    # bf16 32x32x16 per tile and k-step, ~0.5 ms per 1e7 coordinates at N=128
    # at the 2.5 PF peak) and is bound by streaming X once: bytes, not flops
    if agg == "krum":
        return "hbm", HBM_PEAK_GBS, "GB/s", 4 * n * d
    if agg == "mom_krum":
        # the clients read once (the bucket means are formed inside the Gram's
        # loads, gram_bucket.hip) and the chosen bucket's mean row written
        return "hbm", HBM_PEAK_GBS, "GB/s", 4 * n * d + 4 * d
    if agg == "bulyankrum":
        theta = n - 40
        return "hbm", HBM_PEAK_GBS, "GB/s", 4 * n * d + 4 * theta * d + 8 * d   # Gram, final stage, out
    if agg in ("bulyanmedian", "bulyantrimmedmean"):
        theta = n - 40
        return "hbm", HBM_PEAK_GBS, "GB/s", 4 * d * sum(n - i for i in range(theta)) + 8 * theta * d + 4 * d
    if agg in ("filterl2", "ex_noregret"):
        # chunk Grams (fp64 MFMA) + the client-space solver (fp64), the solver
        # priced from chunk 0's measured Lanczos steps (solver_flops below)
        return "mfma", MFMA64_PEAK_TFLOPS, "TFLOP/s", n * (n + 1) * d
    # MoM filters: the same over the B bucket means (the bucket pass itself,
    # 4Nd + 4Bd bytes, is ~2 % of the call at C5); solver flops added below
    b = engine.mom_bucket_count(n, FILTER_ARGS["eps"], MOM_DELTA)[0]
    return "mfma", MFMA64_PEAK_TFLOPS, "TFLOP/s", b * (b + 1) * d


def solver_flops(agg, X, itv=1000):
    """fp64 flops of the spectral filters' client-space solver for one call,
    priced from chunk 0's per-iteration Lanczos step counts (engine.filter_debug,
    outside the timed region): per iteration M = W^1/2 C W^1/2 is formed
    (~3 n_a^2) and every Lanczos step is one symmetric matvec (2 n_a^2) plus
    O(n_a) vector work, n_a = the clients still active.  Chunks are assumed
    to take chunk 0's step counts (they see statistically identical data)."""
    mode = 0 if agg in ("filterl2", "mom_filterl2") else 1
    fa = FILTER_ARGS
    Xc = X[:, :itv]
    if agg.startswith("mom_"):
        num, size = engine.mom_bucket_count(int(X.shape[0]), fa["eps"], MOM_DELTA)
        Xc = engine.bucket_means(Xc, size, num)
    _, _, recs = engine.filter_debug(Xc, mode, fa["eps"], fa["sigma"], fa["expansion"], fa["itv"])
    recs = recs.numpy()
    per_chunk = 0.0
    iters = 0
    for r in recs:
        if not np.isfinite(r[128]):
            break
        na = float(r[132]) if np.isfinite(r[132]) and r[132] > 0 else float(X.shape[0])
        steps = float(r[129])
        per_chunk += 3 * na * na + steps * (2 * na * na + 10 * na)
        iters += 1
    nchunks = -(-int(X.shape[1]) // itv)
    return per_chunk * nchunks, iters


BF16_PEAK_TFLOPS = 2500.0     # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def secondary_roofline(agg, n, d, kern_ms):
    """The other bound of SURVEY.md §8(d) for the same launch: HBM for the
    MFMA-priced filters (their algorithmic bytes: the chunk Gram pass and the
    chunk-mean pass each read X once, 4Nd, plus the 8d fp64 output), MFMA for
    the HBM-priced Krum family (the bf16x3 Gram issues six bf16 32x32x16
    products per upper 32 x 32 tile and 16-coordinate k-step)."""
    t = kern_ms * 1e-3
    if agg in ("filterl2", "ex_noregret", "mom_filterl2", "mom_ex_noregret"):
        nb = n if not agg.startswith("mom_") else engine.mom_bucket_count(n, FILTER_ARGS["eps"], MOM_DELTA)[0]
        byts = 2 * 4 * nb * d + 8 * d + (4 * n * d + 4 * nb * d if agg.startswith("mom_") else 0)
        return {"bound": "hbm", "achieved": round(byts / t / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(byts / t / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": byts}
    if agg in ("krum", "mom_krum", "bulyankrum"):
        m = n if agg != "mom_krum" else -(-n // 3)
        nbk = -(-m // 32)
        flops = 6 * (nbk * (nbk + 1) // 2) * 2 * 32 * 32 * d
        return {"bound": "mfma", "achieved": round(flops / t / 1e12, 2), "peak": BF16_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(flops / t / 1e12 / BF16_PEAK_TFLOPS, 4),
                "issued_bf16_flops_per_launch": flops,
                "note": "whole op's time; the Gram kernel alone is in profiles/ (kernel stats)"}
    return None


def filter_into(agg):
    """(X_cols, out_view) form of a spectral filter for the pipelined path: the
    block's result is written straight into its slot of the all-gather buffer."""
    _load_engine()
    ffn = {"filterl2": engine.filter_l2, "ex_noregret": engine.ex_noregret,
           "mom_filterl2": engine.mom_filter_l2, "mom_ex_noregret": engine.mom_ex_noregret}[agg]
    kw = dict(FILTER_ARGS, check=False)
    if agg.startswith("mom_"):
        kw["delta"] = MOM_DELTA

    def into(Xc, o):
        ffn(Xc, out=o, **kw)
    into.out_dtype = torch.float64
    return into


def filter_block(d, chunks, itv):
    """Block width for the pipelined filter path: d split into the largest
    number <= chunks of equal blocks that are whole itv-chunks (the filters
    chunk every layer at itv, robust_estimator.py:116-125); 0 if none."""
    nblk = next((c for c in range(int(chunks), 0, -1) if d % (c * itv) == 0), 0)
    return d // nblk if nblk else 0


def cpu_baseline(agg, n, budget_s):
    """Time the oracle's CPU port on a bounded sample until ~budget_s elapsed."""
    from oracle import robust_np as orc
    from oracle import dba_np as odba
    fa = FILTER_ARGS

    def _wsum(xs):
        acc = np.zeros(xs[0].shape[0], np.float32)
        w = np.float32(1.0 / len(xs))
        for r in xs:
            acc = acc + w * r
        return acc
    fn = {"dba_median": lambda xs: odba.median(np.asarray(xs)), "dba_weighted_sum": _wsum,
          "trimmedmean": orc.trimmed_mean, "median": orc.median, "average": orc.average,
          "krum": lambda xs: orc.krum(xs, 20), "mom_krum": lambda xs: orc.mom_krum(xs, 20),
          "bulyankrum": lambda xs: orc.bulyan(xs, 20, "krum"),
          "bulyanmedian": lambda xs: orc.bulyan(xs, 20, "median"),
          "bulyantrimmedmean": lambda xs: orc.bulyan(xs, 20, "trimmedmean"),
          "filterl2": lambda xs: orc.filterL2(xs, fa["eps"], fa["sigma"], fa["expansion"], fa["itv"]),
          "ex_noregret": lambda xs: orc.ex_noregret(xs, fa["eps"], fa["sigma"], fa["expansion"], fa["itv"]),
          "mom_filterl2": lambda xs: orc.mom_filterL2(xs, fa["eps"], fa["sigma"], fa["expansion"], fa["itv"],
                                                      MOM_DELTA),
          "mom_ex_noregret": lambda xs: orc.mom_ex_noregret(xs, fa["eps"], fa["sigma"], fa["expansion"],
                                                            fa["itv"], MOM_DELTA)}[agg]
    d = {"krum": 100_000, "mom_krum": 100_000, "bulyankrum": 2_000, "bulyanmedian": 2_000,
         "bulyantrimmedmean": 2_000, "filterl2": 1000, "ex_noregret": 1000, "mom_filterl2": 1000,
         "mom_ex_noregret": 1000}.get(agg, 1_000_000)
    rng = np.random.default_rng(0)
    x = (0.01 * rng.standard_normal((n, d))).astype(np.float32)
    samples = list(x)
    t0 = time.perf_counter()
    fn(samples)  # warm (also the sample itself when one call is slow)
    first = time.perf_counter() - t0
    reps, el = 1, first
    if first < budget_s / 3:
        t0 = time.perf_counter()
        reps = 0
        while True:
            fn(samples)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget_s or reps >= 200:
                break
    gbs = reps * n * d * 4 / el / 1e9
    return {"value": round(gbs, 6), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "%d x numpy %s over N=%d x d=%d fp32 (oracle/), %.1f s on host cores, "
                      "single thread" % (reps, agg, n, d, el)}


def host_inclusive(agg, n, device):
    """Pinned host N x d -> device, aggregate, result -> host (d = 4e6)."""
    d = 4_000_000
    host = torch.empty((n, d), dtype=torch.float32, pin_memory=True)
    host.normal_(0, 0.01)
    res = torch.empty(d, dtype=OUT_DTYPE.get(agg, torch.float32), pin_memory=True)
    X = torch.empty((n, d), dtype=torch.float32, device=device)
    out = torch.empty(d, dtype=OUT_DTYPE.get(agg, torch.float32), device=device)
    for _ in range(2):
        X.copy_(host, non_blocking=True); AGG[agg](X, out); res.copy_(out, non_blocking=True)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        X.copy_(host, non_blocking=True)
        AGG[agg](X, out)
        res.copy_(out, non_blocking=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": round(reps * n * d * 4 / el / 1e9, 2), "unit": "GB/s", "d": d,
            "note": "pinned H2D + kernel + D2H per call, serial on one stream"}


def main():
    a = parse()
    rc = ranks_or_launch(a)
    if rc is not None:
        return rc
    if a.launch_check:
        return launch_check(a)
    _load_engine()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
        world = dist.get_world_size()
    n = a.clients
    d = int(a.d)
    # synthetic client updates, resident in HBM (fixed seed per rank)
    byz = min(a.byzantine, max(n - 1, 0))
    X = synthetic_rows(n, d, byz, 1234 + rank, device)
    odt = OUT_DTYPE.get(a.agg, torch.float32)
    out = torch.empty(d, dtype=odt, device=device)
    full = torch.empty(d * world, dtype=odt, device=device) if world > 1 else None
    fn = AGG[a.agg]
    # N>1, Krum / Bulyan: the selection is global -- the sharded forms exchange
    # the N x N Gram (one reduce to the scoring rank, the pick broadcast) or,
    # per Bulyan round, the <= N distance partials (one all-reduce each), then
    # assemble the (d*world,) result
    sharded = None
    if world > 1 and a.agg in ("krum", "mom_krum", "bulyankrum", "bulyanmedian", "bulyantrimmedmean"):
        ops = shard.engine_ops()
        dtot = d * world
        if a.agg == "krum":
            sharded = lambda: shard.krum(ops["gram"], ops["krum_select"], X, dtot, 20, exact=ops)[0]
        elif a.agg == "mom_krum":
            sharded = lambda: shard.mom_krum(ops, X, dtot, 20)[0]
        else:
            sharded = lambda: shard.bulyan(ops, X, dtot, 20, a.agg[len("bulyan"):])
    # N>1, coordinate-wise: block-cyclic shard (this rank's X = its blocks side
    # by side) with the in-place all-gather of block k on a second stream,
    # overlapped with the k-select of block k+1 (srfl_amd/shard.py)
    pipelined = world > 1 and a.agg in ("trimmedmean", "median", "average") and d % a.chunks == 0
    block = d // a.chunks if pipelined else None
    into = shard.engine_ops()[a.agg + "_into"] if pipelined else None
    # N>1, spectral filters (config C5: mom_filterl2 at N=512): chunks of itv
    # coordinates are independent (robust_estimator.py:116-125, 192-201), so
    # the same block-cyclic pipeline runs with itv-aligned blocks
    if world > 1 and a.agg in ("filterl2", "ex_noregret", "mom_filterl2", "mom_ex_noregret"):
        block = filter_block(d, a.chunks, FILTER_ARGS["itv"])
        if block:
            pipelined = True
            into = filter_into(a.agg)
    comm = torch.cuda.Stream(device=device) if pipelined else None

    def step(ev=None):
        if pipelined:
            shard.pipelined_coordinatewise(into, X, d * world, block, out=full, comm_stream=comm)
            return
        if ev is not None:
            ev[0].record()
        if sharded is not None:
            full.copy_(sharded())
        else:
            fn(X, out)
        if ev is not None:
            ev[1].record()
        if world > 1 and sharded is None:
            dist.all_gather_into_tensor(full, out)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if pipelined:
        # roofline: this rank's local aggregation alone (no collective), same launch
        for k in range(a.steps):
            evs[k][0].record()
            fn(X, out)
            evs[k][1].record()
        torch.cuda.synchronize()
    kern_ms = sum(s.elapsed_time(e) for s, e in evs) / a.steps
    ms_per_step = elapsed * 1e3 / a.steps
    total_bytes = n * d * world * 4
    value = total_bytes / (elapsed / a.steps) / 1e9

    bound, peak, unit, alg = roofline_model(a.agg, n, d)
    solver_note = None
    n_filter = engine.mom_bucket_count(n, FILTER_ARGS["eps"], MOM_DELTA)[0] if a.agg.startswith("mom_") else n
    if a.agg in ("filterl2", "ex_noregret", "mom_filterl2", "mom_ex_noregret") and n_filter > 128:
        # the debug records (sra_filter_debug_f32) exist for the register solver
        # only (N <= 128): above it the flops are the chunk Grams alone
        solver_note = "chunk Grams n(n+1)d only (N > 128: no per-step records for the solver)"
    elif a.agg in ("filterl2", "ex_noregret", "mom_filterl2", "mom_ex_noregret"):
        sflops, iters = solver_flops(a.agg, X)
        alg = alg + int(sflops)
        solver_note = "chunk Grams n(n+1)d + solver %.3g flop (chunk 0: %d iterations, its Lanczos steps)%s" % (
            sflops, iters, ", n = the bucket means" if a.agg.startswith("mom_") else "")
    scale = 1e9 if unit == "GB/s" else 1e12
    achieved = alg / (kern_ms * 1e-3) / scale
    traffic = None
    try:
        with open(a.traffic_json) as fh:
            tj = json.load(fh)
        rec = tj.get("%s:N=%d:d=%d" % (a.agg, n, d))
        if rec:
            traffic = rec["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        traffic = None
    line = {
        "metric": "aggregated-gradient GB/s (device-resident, N x d fp32)",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "world_size": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (SURVEY.md §8(d)), generated on device: 0.01 N(0,1) per client + shared 0.001 N(0,1) "
                 "drift; rows 0..%d Byzantine at -10x the benign mean + 0.001 N(0,1)" % (byz - 1)
                 if byz else "synthetic, generated on device: 0.01 N(0,1) + shared 0.001 N(0,1) drift, no "
                 "Byzantine rows"),
        "config": {"workload": "%s N=%d clients x d=%d fp32 per GPU%s" % (
                       a.agg, n, d, ", d-sharded + RCCL all-gather" if world > 1 else ""),
                   "aggregator": a.agg, "clients": n, "d_per_gpu": d, "d_total": d * world,
                   "parallelism": ("block-cyclic d-shard x%d, %d overlapped all-gather rounds" % (world, d // block)
                                   if pipelined else
                                   ("d-shard x%d, reduced selection" % world if sharded is not None
                                    else "d-shard x%d" % world))},
        "roofline": {"bound": bound, "kernel": kernel_label(a.agg, n), "achieved": round(achieved, 2),
                     "peak": peak, "unit": unit, "frac": round(achieved / peak, 4),
                     "traffic": traffic,
                     "traffic_source": ("rocprofv3 PMC of a separate run (profiles/traffic.json, tools/pmc.sh)"
                                        if traffic is not None else None),
                     "kernel_ms": round(kern_ms, 4),
                     ("algorithmic_bytes_per_launch" if unit == "GB/s" else "algorithmic_flops_per_launch"): alg},
    }
    if solver_note:
        line["roofline"]["model"] = solver_note
    sec = secondary_roofline(a.agg, n, d, kern_ms)
    if sec:
        line["roofline"]["secondary"] = sec
    if rank == 0 and world == 1 and not a.no_host:
        del X
        torch.cuda.empty_cache()
        line["host_inclusive"] = host_inclusive(a.agg, n, device)
    if rank == 0 and world == 1 and not a.no_cpu:
        line["cpu_baseline"] = cpu_baseline(a.agg, n, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
