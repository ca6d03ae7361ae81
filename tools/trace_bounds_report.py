"""Print device error / bound for every chunk of every trace fixture (no asserts)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import srfl_loader
srfl_loader.load()
import torch
from srfl_amd import engine
from conftest import trace_fixtures
MODE = {"filterL2": 0, "mom_filterL2": 0, "ex_noregret": 1}
for rec in trace_fixtures():
    p, func, x = rec["params"], rec["func"], rec["x"]
    X = torch.from_numpy(np.ascontiguousarray(x.reshape(x.shape[0], -1))).cuda()
    if func == "mom_filterL2":
        num, size = engine.mom_bucket_count(X.shape[0], p["eps"], p["delta"])
        X = engine.bucket_means(X, size, num)
    out, tr = engine.filter_trace(X, MODE[func], p["eps"], p["sigma"], p["expansion"], p["itv"])
    out = out.cpu().numpy()
    want = rec["trace"]
    ratios, dec = [], []
    for c in range(want.shape[0]):
        a = int(rec["agree"][c])
        dec.append(bool(np.array_equal(tr[c][1:1 + a], want[c][1:1 + a])))
        sl = slice(c * p["itv"], (c + 1) * p["itv"])
        err = np.abs(out[sl] - rec["out"][sl]).max() / np.abs(rec["out"][sl]).max()
        ratios.append(err / rec["bound"][c])
    print(rec["name"], "decisions ok" if all(dec) else "DECISIONS DIFFER %s" % dec,
          "err/bound", ["%.3f" % r for r in ratios], flush=True)
