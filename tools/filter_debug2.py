"""One-wave solver diagnostics on the bench's data shape (GPU box helper):
chunk 0 of make_rows(128, itv) (20 Byzantine rows) for filterL2 and
ex_noregret -- per iteration the Lanczos steps, checks and cycle split
(debug records of wave_solve_kernel, filter_wave.hip)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import srfl_loader  # noqa: E402

srfl_loader.load()
from srfl_amd import engine  # noqa: E402
from synth import make_rows  # noqa: E402

itv = 1000
x = make_rows(128, itv, seed=int(sys.argv[1]) if len(sys.argv) > 1 else 1, byz=20)
X = torch.from_numpy(x).cuda()
for mode in (0, 1):
    out, G, recs = engine.filter_debug(X, mode, 0.2, 1e-5, 20, itv)
    r = recs.numpy()
    n_it = 0
    while n_it < r.shape[0] and not np.isnan(r[n_it, 128]) and r[n_it, 136] > 0:
        n_it += 1
    r = r[:n_it]
    ms = r[:, 129].astype(int)
    print("mode %d: %d iterations, %d Lanczos steps, %d checks" % (mode, n_it, ms.sum(), r[:, 131].sum()))
    print("   m per iteration", [int(v) for v in ms])
    print("   full Gram-Schmidt calls per iteration", [int(v) for v in r[:, 143]])
    cyc, tck, tmv, tst = r[:, 136].sum(), r[:, 137].sum(), r[:, 138].sum(), r[:, 139].sum()
    print("   Mcycles: total %.3f  checks %.3f  matvec %.3f  step rest %.3f  other %.3f" %
          (cyc / 1e6, tck / 1e6, tmv / 1e6, tst / 1e6, (cyc - tck - tmv - tst) / 1e6))
    print("   per step: matvec %.0f  rest %.0f cycles; per check %.0f (Laguerre %.0f multisection %.0f chains %.0f twist %.0f)" %
          (tmv / max(1, ms.sum()), tst / max(1, ms.sum()), tck / max(1, r[:, 131].sum()),
           *(r[:, [134, 135, 141, 142]].sum(0) / max(1, r[:, 131].sum()))))
