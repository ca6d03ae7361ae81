"""Debug: Krum on bucket means with a NaN client (the mom_krum_nan fixture)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import srfl_loader
srfl_loader.load()
import torch
from srfl_amd import engine

z = np.load("tests/golden/mom_krum_nan_client_n30_f3.npz")
x = z["x"]
X = torch.from_numpy(x).cuda()
B = engine.bucket_means(X, 3, 10)
print("B nan rows", torch.isnan(B).any(1).nonzero().flatten().tolist())
G = engine.gram(B)
print("G diag", G.diag().cpu().numpy())
order, sc = engine.krum_select(B, 3, 1, scores=True)
print("order", order.cpu().tolist(), "scores", sc.cpu().numpy())
Bc = B.clone()
order2, sc2 = engine.krum_select(Bc[:, :32].contiguous(), 3, 1, scores=True)
print("d=32: order", order2.cpu().tolist(), sc2.cpu().numpy())
x12 = np.load("tests/golden/krum_nan_client_n12_f2.npz")["x"]
o3, s3 = engine.krum_select(torch.from_numpy(x12).cuda(), 2, 1, scores=True)
print("n12: order", o3.cpu().tolist(), s3.cpu().numpy())
from srfl_amd import robust_estimator as gre
xs = [x[i] for i in range(x.shape[0])]
got = gre.mom_krum(xs, 3)
print("gre.mom_krum nan at", np.where(np.isnan(got))[0].tolist(), got[:3])
row, order = engine.mom_krum(torch.from_numpy(x).cuda(), 3)
print("engine.mom_krum order", order.cpu().tolist())
