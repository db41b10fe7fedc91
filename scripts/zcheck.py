"""Z of tsne_gradient vs tsne_repulsion vs the optimizer on one state (C2, t=300)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, "tsne-flink_amd")
import configs as CF
import oracle_ctypes as O
import tsne_amd as T
from tsne_amd.api import default_params
from test_gpu_configs import pipeline

ctx = T.Context(0)
X = CF.c2()
Xd = torch.from_numpy(X).cuda()
host, Pd = pipeline(ctx, Xd, 90, "sqeuclidean", 30.0)
n = X.shape[0]
params = default_params(iterations=1000, theta=0.5)
Yh, uh, gh = ctx.initWorkingSet(n, 2, seed=0)
Y = torch.from_numpy(Yh).cuda(); u = torch.from_numpy(uh).cuda(); g = torch.from_numpy(gh).cuda()
ctx.dev_opt_setup(params, *Pd, n, Y, u, g)
T0 = int(sys.argv[1]) if len(sys.argv) > 1 else 300
for t in range(1, T0):
    ctx.dev_opt_step(t)
ctx.dev_opt_sync(); ctx.synchronize()
Y0 = Y.cpu().numpy().copy()
ctx.dev_opt_step(T0)
Zopt = ctx.dev_opt_last_z()
P = host["P"]
res = {"Zopt": Zopt}
for k in range(3):
    F, z = ctx.repulsion(Y0, 0.5)
    res[f"Zrep{k}"] = z.sum()
    _, Zg, _ = ctx.gradient(*P, Y0, 0.5, want_loss=False)
    res[f"Zgrad{k}"] = Zg
    _, Zg2, _ = ctx.gradient(*P, Y0, 0.5, want_loss=True)
    res[f"ZgradL{k}"] = Zg2
r = O.gradient(*P, Y0, 0.5, want_loss=False, threads=16)
res["Zoracle"] = r["Z"]
for k, v in res.items():
    print(f"{k:10s} {v:.17g} rel {v / r['Z'] - 1:+.3e}")
