"""Replay the golden Bulyan fixtures in test order, synchronising after each;
for the target fixture print the Krum order before the full call (GPU box helper)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import srfl_loader  # noqa: E402

srfl_loader.load()
from srfl_amd import engine, robust_estimator as gre  # noqa: E402
from conftest import fixtures  # noqa: E402

target = sys.argv[1] if len(sys.argv) > 1 else "bulyan_krum_n40_f9"
for rec in fixtures(func="bulyan"):
    x = rec["x"].reshape(rec["x"].shape[0], -1)
    f = rec["params"]["f"]
    if rec["name"] == target:
        xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
        got = gre.bulyan(xs, f, rec["params"]["aggsubfunc"])
        torch.cuda.synchronize()
        print("target ok", float(np.abs(np.asarray(got).ravel() - rec["out"].ravel()).max()), flush=True)
        break
    xs = [rec["x"][i] for i in range(rec["x"].shape[0])]
    got = gre.bulyan(xs, f, rec["params"]["aggsubfunc"])
    torch.cuda.synchronize()
    print(rec["name"], "ok", flush=True)
