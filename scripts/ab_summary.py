"""Summarise gpurun_out/ab_<k>.json (scripts/gpu_ab_bench.sh): loop, window,
end to end, and the timeline's BH / attraction ms at a few iterations."""
import json
import os

idx = [l.split(None, 1) for l in open("gpurun_out/ab_index.txt").read().splitlines()]
for k, name in idx:
    d = json.load(open(f"gpurun_out/ab_{k}.json"))
    tl = {r["t"]: r for r in d.get("timeline", [])}
    pts = " ".join(f"t{t}:{tl[t]['tree_ms']:.2f}/{tl[t]['bh_ms']:.2f}/{tl[t]['attract_ms']:.2f}"
                   for t in (250, 500, 700, 900) if t in tl)
    print(f"{k} {name:40s} loop {d['loop_full_s']:.3f} s  window {d['window_it_s']:.0f} it/s  e2e {d['end_to_end_s']:.2f} s  {pts}")
