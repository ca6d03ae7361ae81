"""GPU box helper: the plain-Lanczos filter solver -- timing, fallbacks, steps."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import srfl_loader  # noqa: E402

srfl_loader.load()
from srfl_amd import engine  # noqa: E402

for mode in ((0, 1) if len(sys.argv) < 2 else ()):
    g = torch.Generator(device="cuda").manual_seed(1)
    Y = 0.01 * torch.randn(128, 1_000_000, device="cuda", generator=g)
    out, G, recs = engine.filter_debug(Y, mode, 0.2, 1e-5, 20, 1000)
    fbv = recs.view(-1)[-2:].view(torch.int32).tolist()
    fb = "%d (ghost after retry %d, out of steps %d, retries %d)" % tuple(fbv)
    ms = [int(recs[i, 129]) for i in range(250) if not np.isnan(float(recs[i, 128])) and not np.isnan(float(recs[i, 131]))]
    ck = [int(recs[i, 131]) for i in range(len(ms))]
    cyc = [float(recs[i, 136]) for i in range(len(ms))]
    print("mode", mode, "fallback chunks (of 1000)", fb, "iters", len(ms), "steps", sum(ms), ms[:12],
          "checks", sum(ck), "Mcyc/it %.3f cyc/step %.0f" % (np.mean(cyc) / 1e6, sum(cyc) / max(1, sum(ms))),
          "check Mcyc/it %.3f cyc/check %.0f" % (float(recs[:len(ms), 137].sum()) / len(ms) / 1e6, float(recs[:len(ms), 137].sum()) / max(1, sum(ck))),
          "multisection cyc/check %.0f tri_vec cyc/check %.0f rounds/check %.2f" % (float(recs[:len(ms), 138].sum()) / max(1, sum(ck)), float(recs[:len(ms), 139].sum()) / max(1, sum(ck)), float(recs[:len(ms), 140].sum()) / max(1, sum(ck))),
          flush=True)
    lg = recs[250:].reshape(-1)[:240].reshape(60, 4).numpy()
    for r in lg:
        if np.isnan(r[0]):
            break
        print("   first listed chunk: it %d att %d m %d theta %.17g res/theta %.3e" % (
            r[0] // 10000, (r[0] % 10000) // 1000, r[0] % 1000, r[1], r[3] * abs(r[2]) / r[1]))
    for d in (1_000_000, 10_000_000):
        Z = 0.01 * torch.randn(128, d, device="cuda", generator=g)
        fn = engine.filter_l2 if mode == 0 else engine.ex_noregret
        fn(Z, 0.2, 1e-5, 20, 1000, check=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            fn(Z, 0.2, 1e-5, 20, 1000, check=False)
        torch.cuda.synchronize()
        print("   d=%d: %.2f ms" % (d, (time.perf_counter() - t0) / 2 * 1e3), flush=True)
        del Z

if len(sys.argv) > 1 and sys.argv[1] == "log":
    g = torch.Generator(device="cuda").manual_seed(1)
    Y = 0.01 * torch.randn(128, 1000, device="cuda", generator=g)
    out, G, recs = engine.filter_debug(Y, 0, 0.2, 1e-5, 20, 1000)
    lg = recs[250:].reshape(-1)[:240].reshape(60, 4).numpy()
    np.set_printoptions(precision=17, linewidth=200)
    for r in lg:
        if np.isnan(r[0]):
            break
        print("it %d att %d m %d theta %.17g zlast %.3e beta %.3e res/theta %.3e" % (
            r[0] // 10000, (r[0] % 10000) // 1000, r[0] % 1000, r[1], r[2], r[3], r[3] * abs(r[2]) / r[1]))
    z = Y.double().cpu().numpy()
    zc = z - z.mean(0)
    M = zc @ zc.T / 128
    print("true top eig of M(it 0)", np.linalg.eigvalsh(M)[-3:])
