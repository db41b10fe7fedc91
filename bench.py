"""bench.py -- t-SNE hot path on MI355X (BASELINE.json configs[2]: 1M x 128 GMM,
sqeuclidean, k = 90, perplexity 30, theta 0.5, 1000 Barnes-Hut iterations).

One "step" = one optimizer iteration t of the reference schedule (tree build +
BH repulsion + attraction + fused gains/momentum update + centring) of the
device-resident loop; the embedding, P and all state stay in HBM.

Timeline of a run:
  setup    synthetic data on the device, kNN, affinities, symmetrisation,
           seeded init, tsne_dev_opt_setup -- each timed;
  warmup   W iterations (t = 1..W) on a snapshot of the initial state, with
           the per-stage profile and BH work counters ON (they describe the
           first W iterations of the timed window); the snapshot is restored;
  window   `value`: EXACTLY K iterations t = 1..K timed between barriers +
           synchronisations (no profiling inside; the attraction kernel's HIP
           events are recorded on its own stream and read afterwards);
  rest     the remaining iterations t = K+1..T of the schedule (per-iteration
           cost varies by >1000x over a run: SURVEY.md 8a row A15), profiled
           every --trace iterations -> `full_schedule_it_s` = T / (window + rest)
           and `end_to_end_s` = setup + whole schedule + D2H of Y and the losses.

Multi-GPU: launched by torch.distributed.run, one process per GPU; the
library's own RCCL communicator carries the per-iteration all-gathers;
torch.distributed is used only for the one-time id exchange / kNN graph
gather and for the barriers around the timed region.  Rows of P and BH
queries are sharded, so N GPUs share one problem (strong scaling).
"""
import argparse
import json
import re
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
BF16_MFMA_PEAK_TF = 2500.0   # dense (MI355X_MICROARCH.md); the kNN filter's bf16x3 passes run 3 bf16 MFMAs per product
HBM_PEAK_GBS = 8000.0
PMC_ATTRACT = "r06_ar_attract_traffic.json"   # committed PMC summaries the line quotes (see main)
PMC_BH = "r06_ar_bh_valu.json"
UPDATE_KERNELS = ("combine_update", "center2")   # update + centre kernels in the PMC summary


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=["c3", "c4", "c5"],
                    help="c3: 1M x 128 GMM (the metric's workload); c4: 500k x 300 sparse rows, cosine kNN, 3-D "
                         "embedding (octree); c5: 50,000-point precomputed distance matrix "
                         "(--inputDistanceMatrix: affinities + joint + optimizer, no kNN)")
    ap.add_argument("--steps", type=int, default=20,
                    help="the timed schedule t=1..T as K steps of T/K iterations (0 = one step per iteration)")
    ap.add_argument("--warmup", type=int, default=5,
                    help="untimed warmup: the first W steps of the schedule on a restored snapshot")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=90)
    ap.add_argument("--perplexity", type=float, default=30.0)
    ap.add_argument("--theta", type=float, default=0.5)
    ap.add_argument("--iterations", type=int, default=1000, help="schedule length T")
    ap.add_argument("--trace", type=int, default=50,
                    help="trace pass after the timed region: profile t=1..5 and every N-th iteration (0 = no pass)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cli-e2e", action="store_true",
                    help="skip the end-to-end leg through the native CLI from the reference's COO input (C3, N=1)")
    ap.add_argument("--cpu-sample", type=int, default=64, help="queries in the CPU baseline sample")
    ap.add_argument("--cpu-knn-sample", type=int, default=32, help="queries in the CPU baseline kNN sample")
    ap.add_argument("--dump-y", default="", help="comma-separated iterations t: save Y as <dump-dir>/Y_t<t>.npy")
    ap.add_argument("--dump-dir", default="gpurun_out")
    ap.add_argument("--y0-perturb", type=float, default=0.0,
                    help="relative N(0, eps^2) perturbation of Y0 (measures the chaotic spread of the final KL)")
    ap.add_argument("--y0-perturb-seed", type=int, default=1)
    ap.add_argument("--y0-seed", type=int, default=0, help="initWorkingSet seed (the reference is unseeded)")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="tsne_ctx_set_option on the bench's context (A/B of a tunable; repeatable)")
    ap.add_argument("--detail-out", default="gpurun_out/bench_detail.json",
                    help="side file for the per-iteration timeline, attraction launch log and PMC blobs "
                         "(the stdout line stays < 8 KB; '' = none)")
    ap.add_argument("--cpu-budget", type=float, default=1.0,
                    help="CPU baseline: seconds of BH queries per snapshot (the build is timed apart)")
    ap.add_argument("--locality", action="store_true",
                    help="diagnostic: label-distance histogram of P's edges in the final Morton order (stderr)")
    return ap.parse_args()


def gmm(n, d, seed, device):
    """C3 generator (tests/configs.py c3_torch): 10 centres ~ N(0, 5^2 I),
    within-blob N(0, I), fp32-rounded -- the same data the full-size parity
    test (tests/test_gpu_configs.py) checks."""
    import configs
    return configs.c3_torch(n, d, seed, device)


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


def trace_entry(ctx, t, rows, Y, n):
    ms_t, vis_t = ctx.dev_opt_profile(0)
    ctx.synchronize()   # Y (dev_opt_sync) is written on the context's stream
    per_wave = max(1, rows / 64)
    return {"t": t, "tree_ms": ms_t[0], "bh_ms": ms_t[1], "exchange_ms": ms_t[2],
            "attract_ms": ms_t[3], "update_ms": ms_t[4],
            "pops": vis_t[3], "child_evals": vis_t[5], "dense_pairs": vis_t[2], "moment_evals": vis_t[1],
            "visits_per_point": vis_t[0] / max(1, rows),
            "moment_evals_per_point": vis_t[1] / max(1, rows),
            "dense_pairs_per_point": vis_t[2] / max(1, rows),
            "pops_per_wave": vis_t[3] / per_wave,
            "tile_points_per_wave": vis_t[4] / per_wave,
            "lane_utilisation": vis_t[5] / max(1, 64 * vis_t[6]),
            "heaviest_wave_vs_mean": vis_t[7] / max(1e-9, (vis_t[3] + vis_t[4] / 16) / per_wave),
            "max_wave_pops": vis_t[8], "max_wave_dense_points": vis_t[9],
            "narrow_groups": ctx.counter("opt.narrow_groups"),
            "wave_mhz": ctx.counter("opt.wave_mhz"),
            "extent": (Y[:n].max(0).values - Y[:n].min(0).values).max().item()}


def setup_c3(ctx, a, dev, world, rank, r0, r1, metric="sqeuclidean"):
    """C3: device-generated GMM -> kNN (query rows of this rank) -> affinities
    -> (all-gather of the conditional graph) -> symmetrised P on every rank.
    C4 (BASELINE configs[3]): the same stages on tests/configs.py c4's 500k x
    300 sparse rows (dense on the device, its nonzeros the COO input) with the
    cosine metric."""
    n, d, k = a.n, a.dim, a.k
    kk = min(k, n - 1)
    if a.config == "c4":
        import configs
        X = torch.from_numpy(configs.c4(n=n, d=d)).to(dev)
    else:
        X = gmm(n, d, 2, dev)
    sync_barrier(world)
    t0 = time.perf_counter()
    idx = torch.empty((r1 - r0, kk), dtype=torch.int32, device=dev)
    dist = torch.empty((r1 - r0, kk), dtype=torch.float64, device=dev)
    ctx.dev_knn(X, k, metric, r0, r1, idx, dist)
    sync_barrier(world)
    t_knn = max_over_ranks(time.perf_counter() - t0, world)
    knn_filter_ms = float(sum(ctx.stage_ms("knn.filter")))

    t0 = time.perf_counter()
    rp_local = torch.arange(0, (r1 - r0) * kk + 1, kk, dtype=torch.int64, device=dev)
    p = torch.empty_like(dist)
    ctx.dev_affinities(rp_local, dist, r1 - r0, a.perplexity, p)
    ctx.synchronize()   # the context's outputs before torch reads them (its stream is its own: api.py _fence)
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
    X_host = X.cpu().numpy() if (rank == 0 and world == 1 and not a.no_cpu_baseline) else None
    del X, dist, p
    return orp, oc, ov, nnz, e0, e1, t_knn, knn_filter_ms, t_aff, X_host


def setup_c5(ctx, a, dev, world):
    """C5 (BASELINE configs[4]): a 50,000-point C3-style GMM in 64-D (seed 4,
    tests/configs.py c5_points) whose full sqeuclidean distance matrix,
    diagonal excluded, is the input (Tsne.readDistanceMatrix: every (i, j, d)
    line is a neighbour, Tsne.scala:69-70,155-159) -- 2.5e9 entries, built on
    the device; affinities (workgroup per 49,999-entry row) + joint (64-bit
    offsets).  Every rank builds the same P."""
    import configs
    n = a.n
    Xd = torch.from_numpy(configs.c5_points(n, a.dim, 4)).to(dev)
    sq = (Xd * Xd).sum(1)
    m = n - 1
    dist = torch.empty((n, m), dtype=torch.float64, device=dev)
    col = torch.empty((n, m), dtype=torch.int32, device=dev)
    ar = torch.arange(n, device=dev, dtype=torch.int32)
    for b0 in range(0, n, 1024):
        b1 = min(n, b0 + 1024)
        D = (sq[b0:b1, None] + sq[None, :] - 2.0 * (Xd[b0:b1] @ Xd.T)).clamp_(min=0.0)
        keep = torch.ones((b1 - b0, n), dtype=torch.bool, device=dev)
        keep[torch.arange(b1 - b0, device=dev), torch.arange(b0, b1, device=dev)] = False
        dist[b0:b1] = D[keep].view(b1 - b0, m)
        col[b0:b1] = ar.expand(b1 - b0, n)[keep].view(b1 - b0, m)
        del D, keep
    rp = torch.arange(0, n * m + 1, m, dtype=torch.int64, device=dev)
    sync_barrier(world)
    t0 = time.perf_counter()
    p = torch.empty_like(dist)
    ctx.dev_affinities(rp, dist, n, a.perplexity, p)
    del dist
    cap = n * m
    orp = torch.empty(n + 1, dtype=torch.int64, device=dev)
    oc = torch.empty(cap, dtype=torch.int32, device=dev)
    ov = torch.empty(cap, dtype=torch.float64, device=dev)
    nnz = ctx.dev_joint(rp, col, p, n, cap, orp, oc, ov)
    sync_barrier(world)
    t_aff = max_over_ranks(time.perf_counter() - t0, world)
    del p, col
    torch.cuda.empty_cache()
    return orp, oc, ov, nnz, t_aff


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
    for kv in a.option:
        key, val = kv.split("=", 1)
        ctx.set_option(key, float(val))
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    if world > 1:
        obj = [T.Context.unique_id() if rank == 0 else None]
        torch.distributed.broadcast_object_list(obj, src=0)
        ctx.init_comm(rank, world, obj[0])
    if a.config == "c5":
        if a.n == 1_000_000:
            a.n = 50_000
        a.dim = 64
    C, metric = 2, "sqeuclidean"
    if a.config == "c4":
        if a.n == 1_000_000:
            a.n = 500_000
        if a.dim == 128:
            a.dim = 300
        C, metric = 3, "cosine"
        a.no_cpu_baseline = True   # the CPU baseline leg restates the 2-D path (oracle_gradient); C3 carries it
    n, d, k = a.n, a.dim, a.k
    kk = min(k, n - 1)
    r0, r1 = T.shard_rows(n, world, rank)
    steps = a.steps if a.steps > 0 else a.iterations
    steps = min(steps, a.iterations)

    # ---------------------------------------------------------- setup stages
    if a.config == "c5":
        orp, oc, ov, nnz, t_aff = setup_c5(ctx, a, dev, world)
        t_knn, knn_filter_ms, X_host = 0.0, 0.0, None
        e0, e1 = 0, nnz
        kk = n - 1
    else:
        orp, oc, ov, nnz, e0, e1, t_knn, knn_filter_ms, t_aff, X_host = setup_c3(ctx, a, dev, world, rank, r0, r1,
                                                                                  metric)
    Y = torch.zeros((n, C), dtype=torch.float64, device=dev)
    upd = torch.zeros_like(Y)
    gains = torch.ones_like(Y)
    Yh, _, _ = ctx.initWorkingSet(n, C, seed=a.y0_seed)
    if a.y0_perturb:
        Yh = Yh * (1.0 + a.y0_perturb * np.random.default_rng(a.y0_perturb_seed).normal(size=Yh.shape))
    Y[:n].copy_(torch.from_numpy(Yh))
    snap = (Y.clone(), upd.clone(), gains.clone())
    params = default_params(iterations=a.iterations, theta=a.theta, n_components=C, metric=metric)
    sync_barrier(world)
    t0 = time.perf_counter()
    ctx.dev_opt_setup(params, orp, oc, ov, n, Y, upd, gains)
    sync_barrier(world)
    t_setup = max_over_ranks(time.perf_counter() - t0, world)

    # ---------- warmup on a snapshot: the first W steps of the schedule, untimed;
    # inside it the pre-expansion window t = 1..20 is timed on its own (window_it_s)
    chunks = [(a.iterations * (k - 1) // steps + 1, a.iterations * k // steps) for k in range(1, steps + 1)]
    w_end = chunks[min(a.warmup, steps) - 1][1] if a.warmup > 0 else 0
    win = min(20, a.iterations)
    t_win = None
    for t in range(1, w_end + 1):
        if t == 1:
            sync_barrier(world)
            t0 = time.perf_counter()
        ctx.dev_opt_step(t)
        if t == win:
            sync_barrier(world)
            t_win = max_over_ranks(time.perf_counter() - t0, world)
    torch.cuda.synchronize()
    Y.copy_(snap[0]); upd.copy_(snap[1]); gains.copy_(snap[2])
    ctx.dev_opt_setup(params, orp, oc, ov, n, Y, upd, gains)   # fresh loss slots, kernel logs, labels

    # ------------- timed region: the whole schedule t = 1..T as K steps of T/K iterations
    sync_barrier(world)
    t0 = time.perf_counter()
    t_progress = t0
    for (c0, c1) in chunks:
        for t in range(c0, c1 + 1):
            ctx.dev_opt_step(t)
        if rank == 0 and time.perf_counter() - t_progress > 20.0:   # keep long runs visibly alive
            t_progress = time.perf_counter()
            print(f"[bench] t={c1}/{a.iterations} elapsed {t_progress - t0:.1f}s", file=sys.stderr, flush=True)
    sync_barrier(world)
    t_loop = max_over_ranks(time.perf_counter() - t0, world)
    t0 = time.perf_counter()
    losses = ctx.dev_opt_losses()
    csort_over = ctx.counter("opt.csort_oversized_total") if C == 2 else None   # the timed run's sorts
    ctx.dev_opt_sync()   # the working set back to the caller's buffers (collective), timed with the D2H
    ctx.synchronize()    # (written on the context's stream)
    Y_final = Y[:n].cpu().numpy() if rank == 0 else None   # noqa: F841 (the D2H of the result, timed)
    t_out = time.perf_counter() - t0
    alog = ctx.dev_opt_attract_log()
    upd_ms = ctx.stage_ms("opt.update")

    # ------- trace pass (untimed): the same schedule again from the same state,
    # profiled every --trace iterations (per-stage times, BH work counters),
    # plus the CPU baseline's trajectory snapshots and --dump-y
    window_profile, timeline, snaps = [], [], {}
    snap_at = sorted({max(1, a.iterations * f // 20) for f in (0, 2, 3, 4, 6, 8, 12)} | {a.iterations})
    want_snaps = rank == 0 and world == 1 and not a.no_cpu_baseline
    dumps = {int(v) for v in a.dump_y.split(",")} if a.dump_y else set()
    if a.trace > 0 or want_snaps or dumps:
        Y.copy_(snap[0]); upd.copy_(snap[1]); gains.copy_(snap[2])
        ctx.dev_opt_setup(params, orp, oc, ov, n, Y, upd, gains)
        for t in range(1, a.iterations + 1):
            traced = a.trace > 0 and (t <= 5 or t % a.trace == 0)
            if traced:
                ctx.dev_opt_profile(1)
            ctx.dev_opt_step(t)
            if traced or t in dumps or (world == 1 and t in snap_at):
                ctx.dev_opt_sync()   # the caller's Y (every rank: a collective with several)
            if traced:
                (window_profile if t <= 5 else timeline).append(trace_entry(ctx, t, r1 - r0, Y, n))
            if want_snaps and t in snap_at:
                torch.cuda.synchronize()
                snaps[t] = Y[:n].cpu().numpy().copy()
            if rank == 0 and t in dumps:
                ctx.synchronize()   # the sync's write-back is on the context's stream (before round 6's fix
                # the dump raced it and held the previous sync point's Y: DESIGN.md 6)
                os.makedirs(a.dump_dir, exist_ok=True)
                np.save(os.path.join(a.dump_dir, f"Y_t{t}.npy"), Y[:n].cpu().numpy())
        torch.cuda.synchronize()

    value = a.iterations / t_loop
    # ---- roofline of the HBM-bound gradient kernel (the attraction, stage [3])
    # bytes per launch = nnz*(4 col + 8 val) + (rows+1)*8 row_ptr
    #   + rows*(16 own Y + 16 attr out) + n*16 (gathered Y_j, counted once)
    rows = r1 - r0
    attr_bytes = (e1 - e0) * 12 + (rows + 1) * 8 + rows * 16 * C + n * 8 * C
    # log flags: 0 = non-loss launch on the side stream (beside the tree build / BH),
    # 1 = launch alone on the context stream, 2 = loss launch on the side stream
    # (Z-free KL terms), 3 = non-loss launch alone on the context stream
    nonloss = [ms for (t, sa, ms) in alog if sa in (0, 3)]
    loss_l = [ms for (t, sa, ms) in alog if sa in (1, 2)]
    win_nl = [ms for (t, sa, ms) in alog if sa in (0, 3) and t <= win]
    attr_ms = float(np.mean(nonloss)) if nonloss else None
    attr_gbs = attr_bytes / (attr_ms * 1e-3) / 1e9 if attr_ms else None
    kinds = sorted({sa for (_, sa, _) in alog if sa in (0, 3)})
    attr_kernel = {0: "attract_rows<64,4,LOSS=false>", 1: "attract_tiles<LOSS=false>",
                   2: "attract3<LOSS=false>", 3: "attract_tiles3<LOSS=false>"}.get(ctx.counter("opt.attract_kernel"), "?")
    knn_flops = 2.0 * (r1 - r0) * n * d
    knn_mode = "bf16x3" if ctx.get_option("knn_bf16") else "f32"
    upd_bytes = 64 * C * rows   # N*C*(5 reads + 3 writes)*8 B
    upd_avg = float(np.mean(upd_ms)) if upd_ms else None
    prof = window_profile + timeline
    bh_ms_sum = sum(e["bh_ms"] for e in prof)

    def bh_rate(key):
        return sum(e[key] for e in prof) / (bh_ms_sum * 1e-3) if bh_ms_sum > 0 else None

    def r4(x):   # compact numbers for the one-line record
        return None if x is None else float(f"{x:.4g}")

    workload = {"c3": f"C3: {n}x{d} GMM, sqeuclidean, k={k}, perplexity {a.perplexity}, theta {a.theta}",
                "c4": f"C4: {n}x{d} sparse rows, cosine, k={k}, perplexity {a.perplexity}, theta {a.theta}, 3-D",
                "c5": f"C5: {n}-point distance matrix, perplexity {a.perplexity}, theta {a.theta}"}[a.config]
    workload += (f"; timed = the whole schedule t=1..{a.iterations} (TsneHelpers.scala:396-430) as {steps} steps; "
                 f"value = T / loop s")
    e2e = t_knn + t_aff + t_setup + t_loop + t_out
    detail_path = a.detail_out

    out = {
        "metric": METRIC,
        "value": r4(value),
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": a.warmup,
        "ms_per_step": r4(1e3 * t_loop / steps),
        "ms_per_iteration": r4(1e3 * t_loop / a.iterations),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": {"c3": "synthetic 10-blob GMM (seed 2), seeded Y0",
                 "c4": "synthetic 20-topic sparse rows (seed 3), seeded Y0",
                 "c5": "distance matrix of a synthetic 64-D GMM (seed 4), seeded Y0"}[a.config],
        "config": {"workload": workload, "n": n, "dim": d, "k": k, "theta": a.theta, "iterations": a.iterations,
                   "parallelism": f"rows{world}", "nnz_P": int(nnz),
                   "options": {kv.split("=", 1)[0]: float(kv.split("=", 1)[1]) for kv in a.option}},
        "loop_full_s": r4(t_loop),
        "window_it_s": r4(win / t_win) if t_win else None,
        "end_to_end_s": r4(e2e),
        "end_to_end_note": "kNN + affinities + joint + setup + schedule + D2H; input in HBM",
        "knn_s": r4(t_knn),
        "knn_pts_per_s": r4(n / t_knn) if t_knn > 0 else None,
        "knn_filter_ms": r4(knn_filter_ms),
        "knn_filter_mode": knn_mode,
        # fraction of the MFMA pipe the filter runs on: f32-input MFMA (157.3 TF),
        # or bf16x3 = 3 bf16 MFMA products per dot-product term (2.5 PF dense)
        "knn_mfma_frac_of_peak": r4((knn_flops / (knn_filter_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TF) if knn_mode == "f32"
                                    else (3 * knn_flops / (knn_filter_ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TF))
        if knn_filter_ms > 0 else None,
        "affinities_joint_s": r4(t_aff),
        "opt_setup_s": r4(t_setup),
        "final_loss": losses.get(max(losses)) if losses else None,
        "roofline": {"kernel": attr_kernel + ", mean HIP-event time of its non-loss launches over the timed "
                               "schedule, on the stream each ran on (" +
                               ", ".join({0: "side, beside BH", 3: "context, alone"}[k_] for k_ in kinds) + ")",
                     "bound": "hbm", "achieved": r4(attr_gbs), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": r4(attr_gbs / HBM_PEAK_GBS) if attr_gbs else None, "traffic": None,
                     "bytes_per_launch": attr_bytes, "avg_ms": r4(attr_ms), "launches": len(nonloss),
                     # the window's launches (root-tile phase: beside the short build kernels
                     # only); over the schedule the launches share the CUs with the BH kernels
                     "frac_window": r4(attr_bytes / (float(np.mean(win_nl)) * 1e-3) / 1e9 / HBM_PEAK_GBS)
                     if win_nl else None,
                     "loss_launch_ms": r4(float(np.mean(loss_l))) if loss_l else None},
        "update_centre": {"avg_ms": r4(upd_avg), "bytes_per_iteration": upd_bytes,
                          "achieved_GBs": r4(upd_bytes / (upd_avg * 1e-3) / 1e9) if upd_avg else None,
                          "frac": r4(upd_bytes / (upd_avg * 1e-3) / 1e9 / HBM_PEAK_GBS) if upd_avg else None},
        "bh": {"kernel_ms_traced": r4(bh_ms_sum),
               "pops_per_s": r4(bh_rate("pops")), "lane_child_evals_per_s": r4(bh_rate("child_evals")),
               "dense_pair_terms_per_s": r4(bh_rate("dense_pairs")),
               "moment_evals_per_s": r4(bh_rate("moment_evals")),
               "csort_oversized_total": csort_over},
        "detail": detail_path,
    }
    detail = {"window_profile": window_profile, "timeline": timeline,
              "attract_log_note": "placement 0 side stream, 3 alone; loss launches apart",
              "attract_ms_by_t": [[t, sa, ms] for (t, sa, ms) in alog],
              "losses": {str(t): losses[t] for t in sorted(losses)}}
    # HBM bytes per non-loss attraction launch and BH VALU utilisation: PMC
    # counters cannot be collected by the process they count (rocprofv3 runs
    # the bench as its child), so these come from committed PMC passes over
    # this same command, each file naming the commit it was measured at
    # (profiles/PMC_ATTRACT, profiles/PMC_BH below)
    here = os.path.dirname(os.path.abspath(__file__))
    if n == 1_000_000 and d == 128 and world == 1 and a.config == "c3":
        tf = os.path.join(here, "profiles", PMC_ATTRACT)
        if os.path.exists(tf):
            with open(tf) as fh:
                tj = json.load(fh)
            out["roofline"]["traffic"] = tj.get("traffic_bytes_per_launch")
            out["roofline"]["traffic_source"] = "profiles/" + PMC_ATTRACT + " @" + str(tj.get("commit"))
            upk = tj.get("kernels", {})
            ub = sum(upk.get(kn, {}).get("traffic_bytes_per_launch", 0.0) for kn in UPDATE_KERNELS)
            if ub:
                out["update_centre"]["traffic"] = r4(ub)
            detail["pmc_attract"] = tj
        pmc = os.path.join(here, "profiles", PMC_BH)
        if os.path.exists(pmc):
            with open(pmc) as fh:
                bj = json.load(fh)
            out["bh"]["valu_issue_pmc"] = {kn: r4(v.get("valu_issue_frac")) for kn, v in bj.get("kernels", {}).items()}
            out["bh"]["valu_source"] = "profiles/" + PMC_BH + " @" + str(bj.get("commit"))
            detail["pmc_bh"] = bj
    if a.config == "c4":
        out["metric"] = "t-SNE iterations/sec at C4 (500k x 300 sparse, cosine, 3-D embedding); end-to-end s"
        for key in ("pops_per_s", "lane_child_evals_per_s", "dense_pair_terms_per_s", "moment_evals_per_s"):
            out["bh"].pop(key, None)
    if a.config == "c5":
        out["metric"] = "t-SNE iterations/sec at the 50k precomputed-distance-matrix config (C5); affinities+joint s"
        for key in ("knn_s", "knn_pts_per_s", "knn_filter_ms", "knn_filter_mode", "knn_mfma_frac_of_peak"):
            out.pop(key, None)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cb, cb_detail = cpu_baseline(snaps, a, n, X_host, (orp, oc, ov))
        out["cpu_baseline"] = cb
        detail["cpu_baseline"] = cb_detail
    if rank == 0 and world == 1 and a.config == "c3" and not a.no_cli_e2e:
        out["end_to_end_cli"] = cli_end_to_end(a, X_host, dev)
    if rank == 0 and a.locality:
        locality_report(Y[:n], orp, oc, n)
    if rank == 0:
        if detail_path:
            os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
            with open(detail_path, "w") as fh:
                json.dump(detail, fh)
        line = json.dumps(out)
        assert len(line) < 8192, f"bench line is {len(line)} bytes; the driver parses lines < 8 KB"
        print(line, flush=True)
    ctx.close()
    if world > 1:
        torch.distributed.destroy_process_group()


def cli_end_to_end(a, X_host, dev):
    """The native CLI (tsne-flink_amd/tsne_hip: Tsne.main's flags and file
    formats, Tsne.scala:54-101) end to end on this workload written as the
    reference's input: one "i,j,v" COO line per entry (Tsne.readInput,
    Tsne.scala:138-153; 3.7 GB at 1M x 128), produced untimed on local disk by
    scripts/coo_write.  The timed child process reads the file, runs kNN,
    affinities + joint and the whole schedule, and writes the embedding CSV and
    the loss file (Tsne.scala:86, 99-101); its own phase times come from its
    log.  Returns the line's block (wall time and phases, seconds)."""
    import shutil
    import subprocess
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    exe, writer = os.path.join(here, "tsne-flink_amd", "tsne_hip"), os.path.join(here, "scripts", "coo_write")
    if not (os.path.exists(exe) and os.path.exists(writer)):
        return {"skipped": "tsne_hip / scripts/coo_write not built (__graft_entry__.build)"}
    n, d = a.n, a.dim
    wd = tempfile.mkdtemp(prefix="tsne_cli_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        X = X_host if X_host is not None else gmm(n, d, 2, dev).cpu().numpy()
        xbin, csv = os.path.join(wd, "x.bin"), os.path.join(wd, "input.csv")
        np.ascontiguousarray(X, dtype="<f8").tofile(xbin)
        del X
        t0 = time.perf_counter()
        subprocess.run([writer, xbin, str(n), str(d), csv], check=True, timeout=900)
        t_gen = time.perf_counter() - t0
        os.remove(xbin)
        in_bytes = os.path.getsize(csv)
        cmd = [exe, "--input", csv, "--output", os.path.join(wd, "y.csv"), "--dimension", str(d),
               "--knnMethod", "bruteforce", "--metric", "sqeuclidean", "--perplexity", str(a.perplexity),
               "--iterations", str(a.iterations), "--theta", str(a.theta), "--loss", os.path.join(wd, "loss.txt")]
        print("[bench] CLI end to end: " + " ".join(os.path.basename(c) for c in cmd[:1]) + f" on {in_bytes} B",
              file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            return {"failed": r.returncode, "log": r.stderr[-400:]}
        ph = {}
        for line in r.stderr.splitlines():
            m = re.search(r"\[tsne_hip\] (read|kNN|affinities \+ joint|\d+ iterations|end-to-end)\D.*?([0-9.]+) s", line)
            if m:
                key = {"read": "read_s", "kNN": "knn_s", "affinities + joint": "affinities_joint_s",
                       "end-to-end": "inside_s"}.get(m.group(1), "loop_s")
                ph[key] = float(m.group(2))
        out = {"wall_s": round(wall, 3), "input_bytes": in_bytes, "input_write_s_untimed": round(t_gen, 1)}
        out.update({k: round(v, 3) for k, v in ph.items()})
        if "inside_s" in ph:
            known = sum(ph.get(k, 0.0) for k in ("read_s", "knn_s", "affinities_joint_s", "loop_s"))
            out["setup_and_write_s"] = round(ph["inside_s"] - known, 3)
            out["process_start_s"] = round(wall - ph["inside_s"], 3)
        out["note"] = ("tsne_hip --knnMethod bruteforce --perplexity %g --iterations %d --theta %g from the "
                       "reference's COO text input on local disk to the embedding CSV + loss file" %
                       (a.perplexity, a.iterations, a.theta))
        return out
    finally:
        shutil.rmtree(wd, ignore_errors=True)


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


def cpu_threads():
    """Host threads for the CPU baseline: the cores this process may run on
    (nproc), capped by OMP_NUM_THREADS where the box sets the CPU share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def cpu_baseline(snaps, a, n, X_host, P_dev):
    """The oracle (C fp64 restatement of the reference, OpenMP) timed on a
    bounded sample of the same run.  Optimizer, at embedding snapshots taken
    from the GPU trajectory (t in snaps): the reference's serial quadtree
    build of all n points (TsneHelpers.scala:234-256, one Flink task) timed
    once, then BH repulsion of random queries against that tree
    (TsneHelpers.scala:258-264) in batches of growing size until --cpu-budget
    seconds are spent (more queries where they are cheap: the late
    snapshots), extrapolated to n queries; plus the attraction + update of a
    sample of rows extrapolated to n.  The per-iteration cost is held
    piecewise constant between snapshots and integrated over the schedule.
    kNN: the reference brute force (oracle_knn, all n candidates) for
    `cpu_knn_sample` queries, extrapolated to n queries.  Returns the line's
    block and the side file's detail."""
    import oracle_ctypes as O
    threads = cpu_threads()
    rng = np.random.default_rng(0)
    per_t, detail = {}, {}
    # attraction + update of ~20000 rows (one thread), extrapolated
    rp, col, val = (x.cpu().numpy() for x in P_dev)
    nr = int(min(n, 20000, max(16, 2e7 / max(1.0, len(val) / n))))   # ~2e7 entries at most
    r0 = int(rng.integers(0, n - nr + 1))
    Ys0 = next(iter(snaps.values())) if snaps else np.zeros((n, 2))
    t0 = time.perf_counter()
    g, _ = O.attraction_rows(rp, col, val, Ys0, np.zeros((n, 2)), 1.0, r0, r0 + nr, want_loss=True)
    O.update(np.ascontiguousarray(g), Ys0[r0:r0 + nr].copy(), np.zeros((nr, 2)), np.ones((nr, 2)), 0.01, 0.8, 1000.0)
    t_attr = (time.perf_counter() - t0) / nr * n
    del rp, col, val
    qmax = min(n, 1 << 16)
    for t, Ys in sorted(snaps.items()):
        print(f"[bench] cpu baseline sample at t={t}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        tree = O.Tree(Ys)
        t_build = time.perf_counter() - t0
        order = rng.permutation(n)
        pos, q, spent, visits, batches = 0, max(threads, 16), 0.0, 0, []
        while pos < qmax and (spent < a.cpu_budget or len(batches) < 2):
            sel = order[pos:min(pos + q, qmax)]
            pos += len(sel)
            t0 = time.perf_counter()
            _, _, v = tree.query(a.theta, Ys[sel], threads=threads)
            dt = time.perf_counter() - t0
            spent += dt
            visits += v
            batches.append(dt / len(sel))
            q = min(2 * q, 1 << 14)
        tree.close()
        per_q = spent / pos     # wall seconds per query on `threads` threads
        per_t[t] = t_build + per_q * n + t_attr
        full = [b for b in batches[1:]] or batches   # the first batch warms the caches
        detail[str(t)] = {"build_s": t_build, "queries": pos, "query_s": spent, "visits_per_query": visits / pos,
                          "per_query_ms_batches": [1e3 * b for b in batches]}
        detail[str(t)]["per_query_spread"] = (max(full) / min(full) - 1.0) if min(full) > 0 else None
    ts = sorted(per_t)

    def total(t_end):
        return sum(per_t[min(ts, key=lambda s: abs(s - it))] for it in range(1, t_end + 1))

    def r4(x):
        return float(f"{x:.4g}")

    out = {"value": r4(a.iterations / total(a.iterations)), "unit": "iterations/s", "cores": threads, "kind": "port",
           "per_iteration_s_at": {str(t): r4(per_t[t]) for t in ts},
           "build_s_at": {str(t): r4(detail[str(t)]["build_s"]) for t in ts},
           "queries_at": {str(t): detail[str(t)]["queries"] for t in ts},
           "per_query_spread_at": {str(t): (r4(detail[str(t)]["per_query_spread"])
                                            if detail[str(t)]["per_query_spread"] is not None else None) for t in ts},
           "sample": f"oracle (C fp64 restatement, OpenMP {threads} threads) at GPU-trajectory snapshots: serial "
                     f"reference quadtree build of all {n} points timed once, then BH queries against it "
                     f"(random points, batches to ~{a.cpu_budget:g} s) extrapolated to {n}, + attraction/update "
                     f"of {nr} rows extrapolated; piecewise-constant over t=1..{a.iterations}"}
    if X_host is not None:
        qk = min(a.cpu_knn_sample, n)
        t0 = time.perf_counter()
        O.knn(X_host, a.k, "sqeuclidean", q0=0, q1=qk, threads=threads)
        t_k = time.perf_counter() - t0
        out["knn_pts_per_s"] = r4(qk / t_k)
        out["knn_sample"] = f"oracle_knn exact fp64 brute force over all {n} points, {qk} queries, {threads} threads"
    detail["attraction_update_s_per_iteration"] = t_attr
    return out, detail


if __name__ == "__main__":
    main()
