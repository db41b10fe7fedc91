"""Per-iteration breakdown of a rocprofv3 kernel trace of bench.py: the
optimizer iterations are cut at each bbox_partial launch (the first kernel of
every tree build); for the timed schedule (the last T iterations) prints, per
phase window, the wall span of an iteration and the summed kernel time of the
main groups (tree build, traversal, tiles, spill tasks, attraction, update)."""
import csv
import re
import sys
from collections import defaultdict

GROUPS = [("attract", r"attract_"), ("trav", r"bh_traverse<\d, \d, false>"), ("task", r"bh_traverse<\d, \d, true>"),
          ("tiles", r"tile_apply|moment_apply|chunk_|task_combine|wave_spill|spill_budget|block_cost"),
          ("upd", r"combine_update|update_center|mean2|center_scatter|reduce_")]


def group(name):
    for g, pat in GROUPS:
        if re.search(pat, name):
            return g
    return "tree"


def main(path, T=1000, windows=((1, 150), (150, 200), (200, 300), (300, 450), (450, 650), (650, 800), (800, 1001))):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "bbox_partial" in r["Kernel_Name"]]
    its = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        acc = defaultdict(float)
        for r in rows[a:b]:
            acc[group(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) * 1e-6 if b > a else 0.0
        its.append((span, acc))
    its = its[-T:] if len(its) >= T else its
    print("iterations in trace: %d (timed schedule = last %d)" % (len(its), min(T, len(its))))
    keys = ["tree", "trav", "tiles", "task", "attract", "upd"]
    print("%-11s %8s %8s " % ("t window", "span ms", "sum s") + " ".join("%8s" % k for k in keys))
    for lo, hi in windows:
        sel = its[lo - 1:hi - 1]
        if not sel:
            continue
        span = sum(s for s, _ in sel) / len(sel)
        print("%4d-%-6d %8.3f %8.3f " % (lo, hi - 1, span, sum(s for s, _ in sel) * 1e-3) +
              " ".join("%8.3f" % (sum(a[k] for _, a in sel) / len(sel)) for k in keys))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:3]))
