"""C4 probe: 500k x 300 sparse cosine, 3-D embedding (octree extension), the
reference schedule on one GPU; prints each traced iteration's wall time and
stage times, stops after --cap seconds of optimizer time.  Output: JSON lines."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "tsne-flink_amd"), str(ROOT / "tests")]
import configs  # noqa: E402
import tsne_amd as T  # noqa: E402
from tsne_amd.api import default_params  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=500_000)
ap.add_argument("--cap", type=float, default=200.0)
ap.add_argument("--iterations", type=int, default=1000)
ap.add_argument("--trace-range", default="", help="lo:hi:step -- also trace these iterations (e.g. 100:260:5)")
ap.add_argument("--stop", type=int, default=0, help="stop after this iteration (0: the whole schedule)")
ap.add_argument("--dump-y", default="", help="comma-separated iterations t: save Y as <dump-dir>/Y3_t<t>.npy")
ap.add_argument("--dump-dir", default="gpurun_out")
ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE", help="tsne_ctx_set_option")
a = ap.parse_args()
dumps = {int(v) for v in a.dump_y.split(",") if v}
extra = set()
if a.trace_range:
    lo, hi, st = (int(v) for v in a.trace_range.split(":"))
    extra = set(range(lo, hi, st))
dev = torch.device("cuda", 0)
ctx = T.Context(0)
for kv in a.option:
    ctx.set_option(kv.split("=", 1)[0], float(kv.split("=", 1)[1]))
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
X = torch.from_numpy(configs.c4(n=a.n)).to(dev)
n, k = a.n, 90
torch.cuda.synchronize()
t0 = time.perf_counter()
idx = torch.empty((n, k), dtype=torch.int32, device=dev)
dist = torch.empty((n, k), dtype=torch.float64, device=dev)
ctx.dev_knn(X, k, "cosine", 0, n, idx, dist)
torch.cuda.synchronize()
t_knn = time.perf_counter() - t0
t0 = time.perf_counter()
rp = torch.arange(0, n * k + 1, k, dtype=torch.int64, device=dev)
p = torch.empty_like(dist)
ctx.dev_affinities(rp, dist, n, 30.0, p)
cap = 2 * n * k
orp = torch.empty(n + 1, dtype=torch.int64, device=dev)
oc = torch.empty(cap, dtype=torch.int32, device=dev)
ov = torch.empty(cap, dtype=torch.float64, device=dev)
nnz = ctx.dev_joint(rp, idx, p, n, cap, orp, oc, ov)
torch.cuda.synchronize()
t_aff = time.perf_counter() - t0
print(json.dumps({"knn_s": t_knn, "aff_joint_s": t_aff, "nnz": nnz}), flush=True)
Yh, _, _ = ctx.initWorkingSet(n, 3, seed=0)
Y = torch.from_numpy(Yh).to(dev)
upd, gains = torch.zeros_like(Y), torch.ones_like(Y)
ctx.dev_opt_setup(default_params(iterations=a.iterations, theta=0.5, n_components=3, metric="cosine"), orp, oc, ov,
                  n, Y, upd, gains)
torch.cuda.synchronize()
t_start = time.perf_counter()
for t in range(1, a.iterations + 1):
    trace = t in (1, 2, 5, 10, 20, 50, 100, 150, 200, 250, 300, 400, 500, 600, 700, 800, 900, 1000) or t in extra
    if trace:
        ctx.dev_opt_profile(1)
    ts = time.perf_counter()
    ctx.dev_opt_step(t)
    if trace or t in dumps:
        ctx.dev_opt_sync()   # the caller's Y (written at sync)
    torch.cuda.synchronize()
    dt = time.perf_counter() - ts
    if trace:
        ms, _ = ctx.dev_opt_profile(0)
        ext = (Y.max(0).values - Y.min(0).values).max().item()
        print(json.dumps({"t": t, "step_ms": dt * 1e3, "tree_ms": ms[0], "bh_ms": ms[1], "attract_ms": ms[3],
                          "update_ms": ms[4], "extent": ext, "elapsed_s": time.perf_counter() - t_start}), flush=True)
    if t in dumps:
        np.save(Path(a.dump_dir) / f"Y3_t{t}.npy", Y.cpu().numpy())
    if time.perf_counter() - t_start > a.cap or (a.stop and t >= a.stop):
        print(json.dumps({"stopped_at": t, "elapsed_s": time.perf_counter() - t_start}), flush=True)
        break
else:
    print(json.dumps({"done": a.iterations, "loop_s": time.perf_counter() - t_start,
                      "losses": {str(k2): v for k2, v in ctx.dev_opt_losses().items() if k2 % 100 == 0}}), flush=True)
