"""The same embedding through the optimizer's BH and through a single
repulsion call, in one process: C3 set up as bench.py does, the schedule run
to --t0, then the optimizer's step t0+1, three single tsne_dev_repulsion calls
on the Y it started from, and the optimizer's step t0+2.  Run under
`rocprofv3 --kernel-trace` to compare the kernels' durations; prints the wall
times (synchronised) and the traversal-option state.

usage: python scripts/loop_vs_single.py [--t0 249] [--option KEY=VALUE ...]
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
    t0 = 249
    argv = list(sys.argv[1:])
    if "--t0" in argv:
        i = argv.index("--t0")
        t0 = int(argv[i + 1])
        del argv[i:i + 2]
    sys.argv = [sys.argv[0], "--no-cpu-baseline", "--no-cli-e2e"] + argv
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
    sync_at = {int(v) for v in os.environ.get("SYNC_AT", "").split(",") if v}   # intermediate syncs (bench's trace pass)
    ext = {}
    for t in range(1, t0 + 1):
        ctx.dev_opt_step(t)
        if t in sync_at:
            ctx.dev_opt_sync()
            ext[t] = float((Y.max(0).values - Y.min(0).values).max().item())
    ctx.dev_opt_sync()
    torch.cuda.synchronize()
    Ys = Y.clone()

    def wall(f):
        torch.cuda.synchronize()
        s = time.perf_counter()
        f()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - s)

    out = {"t0": t0, "extents_at_syncs": ext, "extent_t0": float((Ys.max(0).values - Ys.min(0).values).max().item()),
           "opt_step_ms": wall(lambda: ctx.dev_opt_step(t0 + 1))}
    F = torch.empty_like(Ys)
    z = torch.empty(n, dtype=torch.float64, device=dev)
    out["single_ms"] = [wall(lambda: ctx.dev_repulsion(Ys, a.theta, F, z)) for _ in range(3)]
    out["opt_step2_ms"] = wall(lambda: ctx.dev_opt_step(t0 + 2))
    out["options"] = {k: ctx.get_option(k) for k in ("near_tol_early", "near_tol_late", "narrow", "root_tile")}
    ref = os.environ.get("SNAP_REF")   # a bench.py --dump-y snapshot of the same t to compare with
    if ref and os.path.exists(ref):
        Yr = np.load(ref)
        Yl = Ys.cpu().numpy()
        out["vs_dump_max_abs_diff"] = float(np.abs(Yr - Yl).max())
        out["extent_live"] = float(np.ptp(Yl, axis=0).max())
        out["extent_dump"] = float(np.ptp(Yr, axis=0).max())
    dump = os.environ.get("SNAP_OUT")
    if dump:
        np.save(dump, Ys.cpu().numpy())
    print(out, flush=True)


if __name__ == "__main__":
    main()
