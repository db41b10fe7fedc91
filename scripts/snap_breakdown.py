"""Per-kernel time of each tsne_dev_repulsion call in a kernel trace of
scripts/bh_snap.py (calls start at bbox_partial; the last call of every
snapshot's group of reps+1 is printed).

usage: python scripts/snap_breakdown.py [trace.csv] [--reps 2] [--snaps 200,250,...]
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace", nargs="?", default="gpurun_out/snapprof/prof_kernel_trace.csv")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--snaps", default="200,250,300,400,500,700")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if "bbox_partial" in name:
        cur = collections.OrderedDict()
        calls.append(cur)
    if cur is None:
        continue
    m = re.search(r"(?:::)?([A-Za-z_][A-Za-z0-9_]*(?:<[^()]*>)?)\(", name)
    k = (m.group(1) if m else name)[:36]
    cur[k] = cur.get(k, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
g = a.reps + 1
for i, s in enumerate(a.snaps.split(",")):
    if g * i + g - 1 >= len(calls):
        break
    c = calls[g * i + g - 1]
    top = sorted(c.items(), key=lambda x: -x[1])[:8]
    print(f"t={s}: {sum(c.values()):.2f} ms  " + ", ".join(f"{k} {v:.2f}" for k, v in top))
