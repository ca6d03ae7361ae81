"""Dump the spectral-filter diagnostics of a golden fixture (GPU box helper)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import srfl_loader  # noqa: E402

srfl_loader.load()
from srfl_amd import engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "filterL2_exit"
z = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
import json
p = json.loads(str(z["params"]))
x = z["x"].reshape(z["x"].shape[0], -1)
mode = 1 if "noregret" in name else 0
itv = p["itv"] or int(np.floor(np.sqrt(x.shape[1])))
out, G, recs = engine.filter_debug(torch.from_numpy(np.ascontiguousarray(x)).cuda(), mode, p["eps"], p["sigma"],
                                   p["expansion"], itv)
np.set_printoptions(precision=6, linewidth=160)
ch = x[:, :itv].astype(np.float64)
zc = ch - ch.mean(0)
print("G err", np.abs(G.numpy() - zc @ zc.T).max(), "G max", np.abs(zc @ zc.T).max())
print("G diag", np.diag(G.numpy())[:8])
n = x.shape[0]
for it in range(recs.shape[0]):
    r = recs[it].numpy()
    if np.isnan(r[128]) and np.isnan(r[0]):
        break
    print("it", it, "lam", r[128], "m", r[129], "resid", r[130], "checks", r[131], "nact", r[132],
          "restarts", r[134], "gs2", r[135], "cycles", r[136], "c", r[:min(n, 8)])
print("out", out.cpu().numpy()[:8])
print("want", z["out"].ravel()[:8] if "out" in z else None)

if len(sys.argv) > 2 and sys.argv[2] == "synthetic":
    import time
    for mode in (0, 1):
        g = torch.Generator(device="cuda").manual_seed(1)
        Y = 0.01 * torch.randn(128, 1000, device="cuda", generator=g)
        out, G, recs = engine.filter_debug(Y, mode, 0.2, 1e-5, 20, 1000)
        ms, ck, p2, cyc = [], [], [], []
        for it in range(recs.shape[0]):
            r = recs[it].numpy()
            if np.isnan(r[128]):
                break
            ms.append(int(r[129]))
            ck.append(int(r[131]))
            p2.append(int(r[135]))
            cyc.append(r[136])
        print("mode", mode, "iters", len(ms), "lanczos steps", sum(ms), ms)
        print("   checks", sum(ck), "second GS passes", sum(p2), "restarts", int(recs[:len(ms), 134].sum()))
        print("   resid", [float("%.1e" % recs[i, 130]) for i in range(len(ms))][:10])
        print("   Mcycles/iteration %.3f, cycles per Lanczos step %.0f" % (np.mean(cyc) / 1e6, sum(cyc) / max(1, sum(ms))))
        cp = recs[:len(ms), [134, 135, 141, 142]].numpy().sum(0)
        print("   per check: Laguerre %.0f  multisection %.0f  chains %.0f  twist+z %.0f cycles" % tuple(cp / max(1, sum(ck))))
        ph = recs[:len(ms), 137:141].numpy().sum(0)
        print("   per step: check %.0f  matvec+alpha %.0f  dots %.0f  update+reduce %.0f cycles" % tuple(ph / max(1, sum(ms))))
        for d in (1000, 10_000_000):
            Z = 0.01 * torch.randn(128, d, device="cuda", generator=g)
            fn = engine.filter_l2 if mode == 0 else engine.ex_noregret
            fn(Z, 0.2, 1e-5, 20, 1000, check=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                fn(Z, 0.2, 1e-5, 20, 1000, check=False)
            torch.cuda.synchronize()
            print("   d=%d: %.3f ms" % (d, (time.perf_counter() - t0) / 3 * 1e3))
            del Z
