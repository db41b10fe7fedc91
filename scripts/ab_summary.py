"""Summarise an A/B bench file of scripts/gpu_session.sh (`# <variant>` lines, each
followed by bench.py's JSON line): loop, end to end, and the timeline's
tree / BH / attraction ms at a few iterations.

usage: python scripts/ab_summary.py gpurun_out/r5<TAG>/bench.jsonl
(the timeline from the side files bench_detail_<k>.json next to it, k-th run)"""
import json
import os
import sys

name = None
k = 0
for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("#"):
        name = line[1:].strip()
        continue
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    k += 1
    det = os.path.join(os.path.dirname(sys.argv[1]), f"bench_detail_{k}.json")
    tlist = d.get("timeline", [])
    if not tlist and os.path.exists(det):
        tlist = json.load(open(det)).get("timeline", [])
    tl = {r["t"]: r for r in tlist}
    pts = " ".join(f"t{t}:{tl[t]['tree_ms']:.2f}/{tl[t]['bh_ms']:.2f}/{tl[t]['attract_ms']:.2f}"
                   for t in (250, 500, 700, 900) if t in tl)
    print(f"{name or '-':32s} loop {d.get('loop_full_s', float('nan')):.3f} s  "
          f"e2e {d.get('end_to_end_s', float('nan')):.2f} s  {pts}")
