"""A/B of the N = 128 Gram kernels (GPU box helper): run in a child process per
library (SRA_LIB), time engine.gram at C3 (N = 128, d = 1e7) and require the
Grams to be bit-identical.  usage: python tools/gram_ab.py lib_a.so lib_b.so"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, time, numpy as np, torch
sys.path.insert(0, %r)
import srfl_loader; srfl_loader.load()
from srfl_amd import engine
g = torch.Generator(device="cuda").manual_seed(3)
X = 0.01 * torch.randn(128, 10_000_000, device="cuda", generator=g) + 0.001 * torch.randn(1, 10_000_000, device="cuda", generator=g)
X[:20] = -10.0 * X[20:].mean(0, keepdim=True) + 0.001 * torch.randn(20, 10_000_000, device="cuda", generator=g)
G = engine.gram(X); torch.cuda.synchronize()
ts = []
same = True
for _ in range(20):
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(); G2 = engine.gram(X); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    same = same and bool(torch.equal(G, G2))
print("deterministic over 20 calls:", same)
np.save(%r, G.cpu().numpy())
print("%%s: gram %%.3f ms (median of 20), min %%.3f" %% (%r, float(np.median(ts)), min(ts)))
'''
outs = []
for i, lib in enumerate(sys.argv[1:]):
    out = os.path.join(ROOT, "gpurun_out", "G_ab_%d.npy" % i)
    env = dict(os.environ, SRA_LIB=os.path.abspath(lib))
    subprocess.run([sys.executable, "-c", CHILD % (ROOT, out, os.path.basename(lib))], env=env, check=True)
    outs.append(np.load(out))
for i in range(1, len(outs)):
    print("bit-identical %d vs 0:" % i, np.array_equal(outs[i], outs[0]), "max |diff|", np.abs(outs[i] - outs[0]).max())
