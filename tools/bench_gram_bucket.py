"""Time the bucket Gram (gram_bucket.hip) against the current Gram kernels.

  python tools/bench_gram_bucket.py            (on the GPU box)

N = 128 x 1e7 (C3): engine.gram (gram_glds_kernel) vs engine.gram_buckets(X, 1)
(the same kernel family as mom_krum's, bucket size 1); N = 171/200 plain; the
C5 mom_krum shape (512 x 1.25e7, buckets of 3) fused vs bucket means + Gram.
Prints ms per call (HIP events, median of 10) and max |dG| / max|G| between
the two routes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import srfl_loader  # noqa: E402

srfl_loader.load()
from srfl_amd import engine  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    g = torch.Generator(device="cuda").manual_seed(1)
    for n, d in ((128, 10_000_000), (171, 12_500_000), (200, 5_000_000)):
        X = 0.01 * torch.randn(n, d, device="cuda", generator=g)
        t0 = timeit(lambda: engine.gram(X))
        t1 = timeit(lambda: engine.gram_buckets(X, 1))
        G0, G1 = engine.gram(X), engine.gram_buckets(X, 1)
        err = float((G0 - G1).abs().max() / G0.abs().max())
        print("N=%d d=%g  gram %.3f ms (%.2f TB/s)  gram_buckets(1) %.3f ms (%.2f TB/s)  rel diff %.2e"
              % (n, d, t0, 4 * n * d / t0 / 1e9, t1, 4 * n * d / t1 / 1e9, err), flush=True)
        del X
    n, d = 512, 12_500_000
    X = 0.01 * torch.randn(n, d, device="cuda", generator=g)
    t0 = timeit(lambda: engine.gram(engine.bucket_means(X, 3, 171)))
    t1 = timeit(lambda: engine.gram_buckets(X, 3))
    t2 = timeit(lambda: engine.mom_krum(X, 20))
    t3 = timeit(lambda: engine.mom_krum(X, 20, fused=False))
    print("mom N=512 d=1.25e7  means+gram %.3f ms  gram_buckets(3) %.3f ms (%.2f TB/s)  mom_krum fused %.3f ms  "
          "unfused %.3f ms" % (t0, t1, 4 * n * d / t1 / 1e9, t2, t3), flush=True)


if __name__ == "__main__":
    main()
