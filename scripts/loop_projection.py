"""Multi-GPU projection on ONE GPU: the library's own world > 1 optimizer run
as W loopback ranks that take turns on the device (option loop_serial,
comm.cpp LoopGroup, read with tsne_ctx_loop_profile), against the world = 1
run of the same problem.

Each rank logs the wall time of every stretch of its own work between two
collectives, alone on the device.  The sum over collectives of the slowest
rank's stretch is the compute span W devices would take; the collectives are
priced by a model (below), not measured -- the output is a PROJECTION, not a
multi-GPU measurement.

C3 problem (1M x 128 GMM, k = 90, perplexity 30, theta 0.5, seeded Y0),
through the host API tsne_optimize (the same call for world 1 and W).
Output: one JSON line.
"""
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

# collective model for W MI355X on xGMI (MI355X_MICROARCH.md: 7 links x ~153
# GB/s per GPU, point to point): each ragged all-gather of the updated
# embedding (n x 2 doubles; every rank receives (W-1)/W of it) and each
# ragged reduce-scatter of the tree partition's forces (n x 2 doubles; every
# rank sends (W-1)/W of it) at an assumed 100 GB/s effective per GPU, plus
# ~25 us latency for each small all-reduce (Z every iteration, the loss every
# 10th, the tree partition's W costs); the counts are the run's own (the
# serial summary's per-collective counts)
AG_GBS = 100.0
AR_US = 25.0


def build_p(n, d, k, dev):
    ctx = T.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    X = configs.c3_torch(n, d, 2, dev)
    idx = torch.empty((n, k), dtype=torch.int32, device=dev)
    dist = torch.empty((n, k), dtype=torch.float64, device=dev)
    ctx.dev_knn(X, k, "sqeuclidean", 0, n, idx, dist)
    rp = torch.arange(0, n * k + 1, k, dtype=torch.int64, device=dev)
    p = torch.empty_like(dist)
    ctx.dev_affinities(rp, dist, n, 30.0, p)
    cap = 2 * n * k
    orp = torch.empty(n + 1, dtype=torch.int64, device=dev)
    oc = torch.empty(cap, dtype=torch.int32, device=dev)
    ov = torch.empty(cap, dtype=torch.float64, device=dev)
    nnz = ctx.dev_joint(rp, idx, p, n, cap, orp, oc, ov)
    torch.cuda.synchronize()
    P = (orp.cpu().numpy(), oc[:nnz].cpu().numpy(), ov[:nnz].cpu().numpy())
    Y0, _, _ = ctx.initWorkingSet(n, 2, seed=0)
    ctx.close()
    del X, idx, dist, p, orp, oc, ov
    torch.cuda.empty_cache()
    return P, Y0


def run(h, P, Y0, iterations):
    Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
    t0 = time.perf_counter()
    loss = h.optimize(*P, Y, u, g, default_params(iterations=iterations, theta=0.5))
    return time.perf_counter() - t0, loss


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--iterations", type=int, default=1000)
    ap.add_argument("--skip-single", action="store_true")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="tsne_ctx_set_option on both handles (e.g. narrow=0, recut=1)")
    a = ap.parse_args()
    opts = {kv.split("=", 1)[0]: float(kv.split("=", 1)[1]) for kv in a.option}
    dev = torch.device("cuda", 0)
    P, Y0 = build_p(a.n, 128, 90, dev)
    out = {"n": a.n, "world": a.world, "iterations": a.iterations, "options": opts}
    if not a.skip_single:
        with T.Context(0) as one:
            for k_, v_ in opts.items():
                one.set_option(k_, v_)
            t_setup, _ = run(one, P, Y0, 1)
            t_full, loss1 = run(one, P, Y0, a.iterations)
        out.update({"single_call_s": t_full, "single_setup_s": t_setup, "single_loop_s": t_full - t_setup,
                    "single_final_loss": loss1[max(loss1)]})
    m = T.Context.multi([0] * a.world)
    for k_, v_ in opts.items():
        m.set_option(k_, v_)
    m.set_option("loop_serial", 1)
    try:
        t_w, lossw = run(m, P, Y0, a.iterations)
        ser = m.loop_profile()
    finally:
        m.close()
    span_s = ser["span_ms"] * 1e-3
    cnt = {k_: v_["count"] for k_, v_ in ser["by_collective"].items()}
    big = sum(v_ for k_, v_ in cnt.items() if k_ in ("allgatherv", "reduce_scatterv"))
    small = sum(v_ for k_, v_ in cnt.items() if k_.startswith("allreduce_") and not k_.endswith(f"[{(a.n + 255) // 256}]"))
    ag_s = big * (a.world - 1) / a.world * a.n * 16 / (AG_GBS * 1e9)
    ar_s = small * AR_US * 1e-6
    proj = span_s + ag_s + ar_s
    out.update({"serial_call_s": t_w, "multi_final_loss": lossw[max(lossw)], "serial": ser,
                "span_s": span_s, "collective_counts": cnt, "modelled_allgather_s": ag_s, "modelled_allreduce_s": ar_s,
                "projected_loop_s": proj,
                "model": f"all-gather {AG_GBS} GB/s effective per GPU, {AR_US} us per small all-reduce"})
    if "single_loop_s" in out:
        out["projected_speedup"] = out["single_loop_s"] / proj
        out["projected_efficiency"] = out["single_loop_s"] / (a.world * proj)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
