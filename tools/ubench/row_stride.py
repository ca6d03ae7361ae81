"""Row-stride sensitivity of the north-star kernel (trimmed mean N=128, d=1e8):
the same data in client-major rows padded to ld = d + pad floats, timed with
HIP events over 20 launches after 3 warm-up, pads alternating in rounds.
usage (GPU box): python tools/ubench/row_stride.py [pads...]"""
import sys
import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import srfl_loader  # noqa: E402

srfl_loader.load()
from srfl_amd import engine as eng  # noqa: E402
n, d = 128, 100_000_000
pads = [int(x) for x in sys.argv[1:]] or [0, 64, 1024]
dev = torch.device("cuda", 0)
maxpad = max(pads)
buf = torch.empty(n * (d + maxpad), dtype=torch.float32, device=dev)
out = torch.empty(d, dtype=torch.float32, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(1)
res = {p: [] for p in pads}
for rnd in range(3):
    for p in pads:
        X = buf[: n * (d + p)].view(n, d + p)[:, :d]
        X.normal_(0.0, 0.01, generator=g)
        for _ in range(3):
            eng.trimmed_mean(X, 0.1, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            eng.trimmed_mean(X, 0.1, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[p].append(ms)
        print("round %d pad %5d  %.4f ms  %.1f GB/s" % (rnd, p, ms, 4 * n * d / ms / 1e6), flush=True)
for p in pads:
    print("pad %5d  best %.4f  mean %.4f ms" % (p, min(res[p]), sum(res[p]) / len(res[p])))
