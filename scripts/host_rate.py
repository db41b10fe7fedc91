"""Host enqueue time against GPU time per optimizer step, per phase of the
C3 schedule: set up as bench.py does, then for each 100-iteration block the
wall time of issuing its dev_opt_step calls (host side only, no sync) and the
wall time until the GPU has finished them.  A block whose issue time is close
to its total is bound by the host's launch rate, not by the GPU.

usage: python scripts/host_rate.py [--option KEY=VALUE ...]
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--no-cpu-baseline", "--no-cli-e2e"] + sys.argv[1:]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    ctx = bench.T.Context(0)
    for kv in a.option:
        key, val = kv.split("=", 1)
        ctx.set_option(key, float(val))
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    n = a.n
    orp, oc, ov, *_ = bench.setup_c3(ctx, a, dev, 1, 0, 0, n)
    Y = torch.zeros((n, 2), dtype=torch.float64, device=dev)
    upd, gains = torch.zeros_like(Y), torch.ones_like(Y)
    Yh, _, _ = ctx.initWorkingSet(n, 2, seed=a.y0_seed)
    Y.copy_(torch.from_numpy(Yh))
    params = bench.default_params(iterations=a.iterations, theta=a.theta, n_components=2, metric="sqeuclidean")
    ctx.dev_opt_setup(params, orp, oc, ov, n, Y, upd, gains)
    ctx.synchronize()
    rows = []
    for b in range(a.iterations // 100):
        t0 = time.perf_counter()
        for t in range(100 * b + 1, 100 * b + 101):
            ctx.dev_opt_step(t)
        t1 = time.perf_counter()
        ctx.synchronize()
        t2 = time.perf_counter()
        rows.append({"t": f"{100 * b + 1}-{100 * b + 100}", "issue_ms_per_it": round(1e3 * (t1 - t0) / 100, 4),
                     "total_ms_per_it": round(1e3 * (t2 - t0) / 100, 4)})
    for r in rows:
        print(r, flush=True)


if __name__ == "__main__":
    main()
