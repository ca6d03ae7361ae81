"""Solver diagnostics on the bench's §8(d) data: per-iteration Lanczos steps,
checks and cycles of chunk 0, and the fallback counters of the whole call."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import srfl_loader
srfl_loader.load()
from srfl_amd import engine
import bench

d = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
bench.engine = engine
X = bench.synthetic_rows(128, d, 20, 1234, torch.device("cuda", 0))
out, G, recs = engine.filter_debug(X, mode, 0.2, 1e-5, 20, 1000)
recs = recs.numpy()
ms, ck, cyc, tck = [], [], [], []
for it in range(recs.shape[0]):
    r = recs[it]
    if np.isnan(r[128]):
        break
    ms.append(int(r[129])); ck.append(int(r[131])); cyc.append(r[136]); tck.append(r[137])
print("iters", len(ms), "steps", sum(ms), ms)
print("checks", sum(ck), ck)
print("cycles/iteration %.0f  cycles per step %.0f  check cycles per check %.0f  check share %.2f" % (
    np.mean(cyc), sum(cyc) / max(1, sum(ms)), sum(tck) / max(1, sum(ck)), sum(tck) / max(1, sum(cyc))))
fb = recs[255, 141:144].view(np.int32)
print("fallback counters [listed, ghost after retry, out of steps, retries, queue, rescued]:", fb.tolist())
