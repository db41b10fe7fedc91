"""Diagnostic: does torch's HIP init still work after libtsne_hip has run
kernels in the same process?  Prints each step."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tsne-flink_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import tsne_amd as T  # noqa: E402
step = sys.argv[1] if len(sys.argv) > 1 else "gradient"
ctx = T.Context(0)
print("ctx ok", flush=True)
if step in ("gradient", "knn"):
    rng = np.random.default_rng(0)
    n = 500
    if step == "knn":
        X = rng.normal(size=(n, 16))
        ctx.kNearestNeighbors(X, 10)
    else:
        rp = np.arange(0, n * 8 + 1, 8, dtype=np.int64)
        col = rng.integers(0, n, n * 8).astype(np.int32)
        val = np.full(n * 8, 1.0 / (n * 8))
        Y = rng.normal(size=(n, 2)) * 1e-2
        ctx.gradient(rp, col, val, Y, 0.5)
    print(step, "ok", flush=True)
import torch  # noqa: E402
print("torch imported", flush=True)
print("avail", torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
x = torch.zeros(4, device="cuda:0")
print("torch tensor ok", x.sum().item(), flush=True)
