"""Time the repulsion (tsne_dev_repulsion: tree build + BH traversal +
tiles + moments; 2-D quadtree or, for n x 3 snapshots, the octree) on
embedding snapshots written by `bench.py --dump-y T1,T2,... --dump-dir DIR`
(C3) or `scripts/c4_probe.py --dump-y ...` (C4), and print per snapshot the
median wall time and checksums of F and z (to compare variants: equal
checksums = equal results up to the printed digits).

usage: python scripts/bh_snap.py DIR/Y_t250.npy [...] [--reps 5] [--theta 0.5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tsne-flink_amd"))
import tsne_amd as T  # noqa: E402


def ctx_has_option(ctx, key):
    """False for a library build without the option (A/B against older builds)."""
    try:
        ctx.get_option(key)
        return True
    except Exception:
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("snaps", nargs="+")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--theta", type=float, default=0.5)
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE", help="tsne_ctx_set_option")
    ap.add_argument("--wavelog", default="", help="with --stats: save each snapshot's BH wave timeline "
                    "(start, end, kind; option wave_log) to <wavelog>_<snapshot>.npz")
    ap.add_argument("--stats", action="store_true",
                    help="after the timed calls, one call of the counting traversal (option rep_stats): "
                         "wave pops, child slots, tile points (2-D)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    with T.Context(0) as ctx:
        ctx.set_option("reuse_costs", 1)   # repeated calls: the narrow selection from the previous call
        for kv in a.option:
            key, val = kv.split("=", 1)
            ctx.set_option(key, float(val))
        for path in a.snaps:
            Y = torch.from_numpy(np.load(path)).to(dev, torch.float64).contiguous()
            n = Y.shape[0]
            F = torch.empty((n, Y.shape[1]), dtype=torch.float64, device=dev)
            z = torch.empty(n, dtype=torch.float64, device=dev)
            times = []
            for _ in range(a.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ctx.dev_repulsion(Y, a.theta, F, z)
                ctx.synchronize()
                times.append(time.perf_counter() - t0)
            narrow = ctx.counter("bh.narrow_groups")
            times = sorted(times[1:] if len(times) > 1 else times)   # --reps 0: the one (cold) call
            rec = {"snapshot": os.path.basename(path), "n": n, "ms_median": 1e3 * times[len(times) // 2],
                   "ms_min": 1e3 * times[0], "narrow_groups": narrow, "sum_abs_F": float(F.abs().sum()),
                   "sum_z": float(z.sum())}
            if ctx_has_option(ctx, "spill"):
                rec["spill_tasks"] = ctx.counter("bh.spill_tasks")
                rec["spill_flags"] = ctx.counter("bh.spill_flags")
            if a.stats and Y.shape[1] == 2 and ctx_has_option(ctx, "rep_stats"):
                ctx.set_option("rep_stats", 1)
                if a.wavelog:
                    ctx.set_option("wave_log", 1)
                ctx.dev_repulsion(Y, a.theta, F, z)
                if a.wavelog:
                    ctx.synchronize()
                    t0w, t1w, kw = ctx.debug_wave_log()
                    np.savez(f"{a.wavelog}_{os.path.basename(path).replace('.npy', '')}.npz", start=t0w, end=t1w,
                             kind=kw)
                    ctx.set_option("wave_log", 0)
                for k in ("pops", "child_slots", "tile_points", "visits", "wave_ticks_max", "wave_ticks_sum",
                          "span_ticks", "dense_pairs", "moment_evals", "tile_ticks_max", "tile_ticks_sum",
                          "tile_span_ticks", "slow_wave_ticks", "slow_wave_pops", "slow_wave_ties",
                          "slow_wave_tile_points", "slow_wave_slots", "wave_mhz") + tuple(f"tile_{w}{j}" for j in range(4)
                                                                              for w in ("steps", "pairs")):
                    rec[k] = ctx.counter("bh." + k)
                ctx.set_option("rep_stats", 0)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
