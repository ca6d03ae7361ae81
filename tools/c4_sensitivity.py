"""How far apart two fp64 evaluations of the reference's filterL2_ end on a
C4-shaped chunk (N=128, simulate.py's eps=0.2, sigma=1e-5): the live reference
(outer-product covariance) vs oracle/robust_np.py (one GEMM).  Prints the top
eigenvalue of every iteration from both and the final output gap.  Build
container only (imports the reference).  Usage: python tools/c4_sensitivity.py [0|1]
"""
import numpy as np, sys, types, warnings
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests/golden')
from gen_fixtures import load_reference
ref = load_reference()
from oracle import robust_np as orc
z = np.load('/root/repo/tests/golden/filterL2_n128_c4.npz')
ch = int(sys.argv[1]) if len(sys.argv) > 1 else 1
x = z['x'].reshape(128, -1)[:, [slice(0, 1000), slice(1000, None)][ch]].astype(np.float32)
rec = []
orig = ref.eigh
def spy(a, *args, **kw):
    r = orig(a, *args, **kw); rec.append(float(r[0][0])); return r
ref.eigh = spy
out_ref = ref.filterL2_(x.copy(), 0.2, 1e-5, 20)
lr = rec[:]; rec.clear()
import scipy.linalg
oe = orc.eigh
def spy2(a, *args, **kw):
    r = oe(a, *args, **kw); rec.append(float(r[0][0])); return r
orc.eigh = spy2
out_or = orc.filterL2_(x.copy(), 0.2, 1e-5, 20)
lo = rec[:]
print(len(lr), len(lo))
for i, (a, b) in enumerate(zip(lr, lo)):
    print(i, "%.6e %.6e rel %.1e" % (a, b, abs(a-b)/a), "" if abs(a-b)/a < 1e-10 else "<<<")
print("out rel diff", np.max(np.abs(out_ref - out_or)) / np.max(np.abs(out_ref)))
