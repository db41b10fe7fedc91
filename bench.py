"""bench.py -- t-SNE hot path on MI355X (BASELINE.json configs[2]: 1M x 128 GMM,
sqeuclidean, k = 90, perplexity 30, theta 0.5, 1000 Barnes-Hut iterations).

One "step" = one optimizer iteration t of the reference schedule (tree build +
BH repulsion + attraction + fused gains/momentum update + centring) of the
device-resident loop; the embedding, P and all state stay in HBM.  By default
the timed steps are the WHOLE schedule t = 1..T (T = 1000): per-iteration cost
varies by >1000x over a run (near-exact O(N^2) BH while the embedding is tiny,
~2 node visits per point once it has expanded: SURVEY.md section 8a row A15),
so `value` = T / (time of the full loop) is the honest iterations/s.  Warmup
iterations run on a snapshot of the initial state, which is restored before
timing.  Setup (synthetic data, kNN, affinities, symmetrisation, seeded init)
is timed separately; kNN points/s and end-to-end seconds are reported beside.

Multi-GPU: launched by torch.distributed.run, one process per GPU; the
library's own RCCL communicator carries the per-iteration all-gathers;
torch.distributed is used only for the one-time id exchange / kNN graph
gather and for the barriers around the timed region.  Rows of P and BH
queries are sharded, so N GPUs share one problem (strong scaling).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "tsne-flink_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import tsne_amd as T  # noqa: E402
from tsne_amd.api import default_params  # noqa: E402

METRIC = "t-SNE iterations/sec + end-to-end sec at N=1M×128 on 1/2/4/8 MI355X; kNN pts/s"
FP32_MFMA_PEAK_TF = 157.3
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed iterations (0 = the whole schedule T)")
    ap.add_argument("--warmup", type=int, default=3, help="untimed iterations on a restored snapshot")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=90)
    ap.add_argument("--perplexity", type=float, default=30.0)
    ap.add_argument("--theta", type=float, default=0.5)
    ap.add_argument("--iterations", type=int, default=1000, help="schedule length T")
    ap.add_argument("--trace", type=int, default=50, help="profile every N-th timed iteration (0 = off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=64, help="queries in the CPU baseline sample")
    ap.add_argument("--dump-y", default="", help="comma-separated iterations t: save Y as gpurun_out/Y_t<t>.npy")
    ap.add_argument("--locality", action="store_true",
                    help="diagnostic: label-distance histogram of P's edges in the final Morton order (stderr)")
    return ap.parse_args()


def gmm(n, d, seed, device):
    """C3 generator: 10 centres ~ N(0, 5^2 I), within-blob N(0, I), fp32-rounded."""
    g = torch.Generator(device=device).manual_seed(seed)
    centers = torch.randn(10, d, generator=g, device=device, dtype=torch.float64) * 5.0
    lab = torch.randint(0, 10, (n,), generator=g, device=device)
    X = centers[lab] + torch.randn(n, d, generator=g, device=device, dtype=torch.float64)
    return X.float().double().contiguous()


def sync_barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
    ctx = T.Context(local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    if world > 1:
        obj = [T.Context.unique_id() if rank == 0 else None]
        torch.distributed.broadcast_object_list(obj, src=0)
        ctx.init_comm(rank, world, obj[0])
    n, d, k = a.n, a.dim, a.k
    kk = min(k, n - 1)
    r0, r1 = T.shard_rows(n, world, rank)
    steps = a.steps if a.steps > 0 else a.iterations

    # ---------------------------------------------------------- setup stages
    X = gmm(n, d, 2, dev)
    sync_barrier(world)
    t0 = time.perf_counter()
    idx = torch.empty((r1 - r0, kk), dtype=torch.int32, device=dev)
    dist = torch.empty((r1 - r0, kk), dtype=torch.float64, device=dev)
    ctx.dev_knn(X, k, "sqeuclidean", r0, r1, idx, dist)
    sync_barrier(world)
    t_knn = max_over_ranks(time.perf_counter() - t0, world)

    t0 = time.perf_counter()
    rp_local = torch.arange(0, (r1 - r0) * kk + 1, kk, dtype=torch.int64, device=dev)
    p = torch.empty_like(dist)
    ctx.dev_affinities(rp_local, dist, r1 - r0, a.perplexity, p)
    chunk = -(-n // world)
    if world > 1:   # full conditional graph on every rank for the symmetrisation
        pad = chunk - (r1 - r0)
        gi = torch.nn.functional.pad(idx, (0, 0, 0, pad)).contiguous()
        gp = torch.nn.functional.pad(p, (0, 0, 0, pad)).contiguous()
        all_i = torch.empty((world * chunk, kk), dtype=torch.int32, device=dev)
        all_p = torch.empty((world * chunk, kk), dtype=torch.float64, device=dev)
        torch.distributed.all_gather_into_tensor(all_i, gi)
        torch.distributed.all_gather_into_tensor(all_p, gp)
        idx_full, p_full = all_i[:n].contiguous(), all_p[:n].contiguous()
    else:
        idx_full, p_full = idx, p
    rp_full = torch.arange(0, n * kk + 1, kk, dtype=torch.int64, device=dev)
    cap = 2 * n * kk
    orp = torch.empty(n + 1, dtype=torch.int64, device=dev)
    oc = torch.empty(cap, dtype=torch.int32, device=dev)
    ov = torch.empty(cap, dtype=torch.float64, device=dev)
    nnz = ctx.dev_joint(rp_full, idx_full, p_full, n, cap, orp, oc, ov)
    e0, e1 = int(orp[r0].item()), int(orp[r1].item())      # this rank's rows of P
    sync_barrier(world)
    t_aff = max_over_ranks(time.perf_counter() - t0, world)
    del X, dist, p

    Y = torch.zeros((n, 2), dtype=torch.float64, device=dev)
    upd = torch.zeros_like(Y)
    gains = torch.ones_like(Y)
    Yh, _, _ = ctx.initWorkingSet(n, 2, seed=0)
    Y[:n].copy_(torch.from_numpy(Yh))
    snap = (Y.clone(), upd.clone(), gains.clone())
    params = default_params(iterations=a.iterations, theta=a.theta)
    ctx.dev_opt_setup(params, orp, oc, ov, n, Y, upd, gains)

    # ----------------------------------------------- warmup on a snapshot
    for t in range(1, a.warmup + 1):
        ctx.dev_opt_step(t)
    torch.cuda.synchronize()
    Y.copy_(snap[0]); upd.copy_(snap[1]); gains.copy_(snap[2])
    ctx.dev_opt_setup(params, orp, oc, ov, n, Y, upd, gains)   # fresh loss slots

    # ------------------------------------------------------- timed steps
    timeline = []
    snap_at = {1, max(1, steps // 10), max(1, steps // 5), max(1, 2 * steps // 5), steps}
    snaps = {}
    sync_barrier(world)
    t0 = time.perf_counter()
    t_progress = t0
    for t in range(1, steps + 1):
        traced = a.trace and (t % a.trace == 0 or t == 1)
        if traced:
            ctx.dev_opt_profile(1)
        ctx.dev_opt_step(t)
        if traced:
            ms_t, vis_t = ctx.dev_opt_profile(0)
            timeline.append({"t": t, "tree_ms": ms_t[0], "bh_ms": ms_t[1], "exchange_ms": ms_t[2],
                             "attract_ms": ms_t[3], "centre_ms": ms_t[4],
                             "visits_per_point": vis_t[0] / max(1, r1 - r0),
                             "moment_evals_per_point": vis_t[1] / max(1, r1 - r0),
                             "dense_pairs_per_point": vis_t[2] / max(1, r1 - r0),
                             "pops_per_wave": vis_t[3] / max(1, (r1 - r0) / 64),
                             "tile_points_per_wave": vis_t[4] / max(1, (r1 - r0) / 64),
                             "lane_utilisation": vis_t[5] / max(1, 64 * vis_t[6]),
                             "heaviest_wave_vs_mean": vis_t[7] / max(1e-9, (vis_t[3] + vis_t[4] / 16) / max(1, (r1 - r0) / 64)),
                             "max_wave_pops": vis_t[8], "max_wave_dense_points": vis_t[9],
                             "extent": (Y[:n].max(0).values - Y[:n].min(0).values).max().item()})
        if rank == 0 and world == 1 and not a.no_cpu_baseline and t in snap_at and traced:
            snaps[t] = Y[:n].cpu().numpy().copy()
        if rank == 0 and a.dump_y and t in {int(v) for v in a.dump_y.split(",")}:
            os.makedirs("gpurun_out", exist_ok=True)
            np.save(f"gpurun_out/Y_t{t}.npy", Y[:n].cpu().numpy())
        if rank == 0 and time.perf_counter() - t_progress > 20.0:   # keep long runs visibly alive
            t_progress = time.perf_counter()
            print(f"[bench] t={t}/{steps} elapsed {t_progress - t0:.1f}s", file=sys.stderr, flush=True)
    sync_barrier(world)
    t_loop = max_over_ranks(time.perf_counter() - t0, world)
    losses = ctx.dev_opt_losses()

    value = steps / t_loop
    # ---- roofline of the HBM-bound gradient kernel attract_rows (stage [3])
    # bytes per launch = nnz*(4 col + 8 val) + (rows+1)*8 row_ptr
    #   + rows*(16 own Y + 16 attr out) + n*16 (gathered Y_j, counted once)
    rows = r1 - r0
    attr_bytes = (e1 - e0) * 12 + (rows + 1) * 8 + rows * 32 + n * 16
    attr_ms = float(np.median([e["attract_ms"] for e in timeline])) if timeline else None
    attr_gbs = attr_bytes / (attr_ms * 1e-3) / 1e9 if attr_ms else None
    knn_flops = 2.0 * (r1 - r0) * n * d

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * t_loop / steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic 10-blob Gaussian mixture (seed 2, fp32-rounded), seeded Y0 ~ N(0, 1e-4^2)",
        "config": {"workload": f"C3: {n}x{d} GMM, sqeuclidean, k={k}, perplexity {a.perplexity}, "
                               f"theta {a.theta}, schedule T={a.iterations}, timed t=1..{steps}",
                   "n": n, "dim": d, "k": k, "theta": a.theta, "parallelism": f"rows{world}",
                   "nnz_P": int(nnz)},
        "end_to_end_s": t_knn + t_aff + t_loop,
        "loop_s": t_loop,
        "knn_s": t_knn,
        "knn_pts_per_s": n / t_knn,
        "knn_mfma_tflops": knn_flops / t_knn / 1e12,
        "knn_mfma_frac_of_peak": knn_flops / t_knn / 1e12 / FP32_MFMA_PEAK_TF,
        "affinities_joint_s": t_aff,
        "final_loss": losses.get(max(losses)) if losses else None,
        "roofline": {"kernel": "attract_rows<64,4,LOSS=true> (CSR attraction + KL terms, TsneHelpers.scala:269-306), timed alone in loss iterations; the non-loss launches share the CUs with the BH traversal on a side stream",
                     "bound": "hbm", "achieved": attr_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (attr_gbs / HBM_PEAK_GBS) if attr_gbs else None, "traffic": None,
                     "bytes_per_launch": attr_bytes, "avg_ms": attr_ms},
        "timeline": timeline,
    }
    # HBM bytes per launch of attract_rows from the committed PMC passes
    # (profiles/r01_attract_traffic.json, scripts/gpu_pmc_attract.sh), valid for this workload
    tf = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01_attract_traffic.json")
    if os.path.exists(tf) and n == 1_000_000 and d == 128 and world == 1:
        with open(tf) as fh:
            tj = json.load(fh)
        out["roofline"]["traffic"] = tj["traffic_bytes"]
        out["roofline"]["traffic_source"] = tj["source"] + "; " + tj["window"] + "; " + tj["note"]
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(snaps, a, n, steps)
    if rank == 0 and a.locality:
        locality_report(Y[:n], orp, oc, n)
    if rank == 0:
        print(json.dumps(out))
    ctx.close()
    if world > 1:
        torch.distributed.destroy_process_group()


def locality_report(Y, rp, col, n):
    """Diagnostic: how far apart (in Morton rank of the final embedding, i.e.
    the optimizer's relabelled row order) the endpoints of P's edges lie --
    the CSR attraction's Y_j gathers hit L2 only for near edges."""
    q = ((Y - Y.min(0).values) / (Y.max(0).values - Y.min(0).values + 1e-300) * (2 ** 20 - 1)).long()
    key = torch.zeros(n, dtype=torch.int64, device=Y.device)
    for b in range(20):
        key |= ((q[:, 0] >> b) & 1) << (2 * b) | ((q[:, 1] >> b) & 1) << (2 * b + 1)
    rank = torch.empty_like(key)
    rank[torch.argsort(key)] = torch.arange(n, device=Y.device)
    rows = torch.repeat_interleave(torch.arange(n, device=Y.device), rp[1:n + 1] - rp[:n])
    dist = (rank[rows] - rank[col[:rows.numel()].long()]).abs().double()
    qs = torch.tensor([0.5, 0.75, 0.9, 0.99], dtype=torch.float64, device=Y.device)
    sample = dist[torch.randint(0, dist.numel(), (1 << 22,), device=Y.device)]
    for w in (64, 512, 2048, 16384, 131072):
        frac = (dist <= w).double().mean().item()
        print(f"[locality] |rank_i - rank_j| <= {w:6d}: {frac:.3f}", file=sys.stderr)
    print(f"[locality] quantiles 50/75/90/99%: {torch.quantile(sample, qs).tolist()}", file=sys.stderr)


def cpu_baseline(snaps, a, n, steps):
    """The oracle (C fp64 restatement of the reference, OpenMP) timed on a
    bounded sample of the same run: at each embedding snapshot taken from the
    GPU trajectory (t in snaps), the reference quadtree build of all n points
    + BH repulsion of `cpu_sample` random queries, extrapolated to n queries;
    the per-iteration cost is held piecewise constant between snapshots and
    integrated over the timed schedule -> iterations/s."""
    import oracle_ctypes as O
    threads = min(16, os.cpu_count() or 1)
    q = min(a.cpu_sample, n)
    sel = np.random.default_rng(0).choice(n, q, replace=False)
    per_t = {}
    for t, Ys in sorted(snaps.items()):
        print(f"[bench] cpu baseline sample at t={t}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        O.repulsion_queries(Ys, a.theta, Ys[sel], threads=threads)
        t_sample = time.perf_counter() - t0
        t0 = time.perf_counter()
        O.repulsion_queries(Ys, a.theta, Ys[sel[:1]], threads=1)
        t_build = time.perf_counter() - t0
        per_t[t] = t_build + max(t_sample - t_build, 1e-9) / q * n
    ts = sorted(per_t)
    total = 0.0
    for it in range(1, steps + 1):
        nearest = min(ts, key=lambda s: abs(s - it))
        total += per_t[nearest]
    return {"value": steps / total, "unit": "iterations/s", "cores": threads, "kind": "port",
            "per_iteration_s_at": {str(t): per_t[t] for t in ts},
            "sample": f"oracle (C fp64 reference restatement, OpenMP {threads} threads): at GPU-trajectory "
                      f"snapshots t={ts}, reference quadtree build of all {n} points + BH repulsion of {q} "
                      f"random queries extrapolated to {n}; piecewise-constant over t=1..{steps}; "
                      f"attraction/update excluded (so the CPU figure is optimistic)"}


if __name__ == "__main__":
    main()
