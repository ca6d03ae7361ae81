"""ex_noregret solver diagnostics on the bench's §8(d) data (chunk 0, debug build of
filter_solve_kernel<1>): per filter iteration the Lanczos steps, restarts, second
Gram-Schmidt passes and cycles, split into check / matvec+alpha / dots / update,
the rest (weights, tau, capped-simplex projection) as 'other'."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import srfl_loader
srfl_loader.load()
from srfl_amd import engine
import bench

d = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
bench.engine = engine
X = bench.synthetic_rows(128, d, 20, 1234, torch.device("cuda", 0))
out, G, recs = engine.filter_debug(X, 1, 0.2, 1e-5, 20, 1000)
recs = recs.numpy()
tot = np.zeros(6)
for it in range(recs.shape[0]):
    r = recs[it]
    if np.isnan(r[128]):
        break
    cyc, ph = r[136], r[137:141]
    other = cyc - ph.sum()
    tot += np.array([cyc, *ph, other])
    print("it %2d  m %3d checks %2d restarts %d passes2 %3d  cycles %8.0f  check %7.0f matvec %7.0f dots %7.0f "
          "update %7.0f other %7.0f" % (it, r[129], r[131], r[134], r[135], cyc, *ph, other))
print("total cycles %.0f: check %.2f matvec %.2f dots %.2f update %.2f other %.2f" % (
    tot[0], *(tot[1:] / tot[0])))
