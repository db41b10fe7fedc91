"""Instructions per wave pop of the 64-query BH traversal (bh_traverse<0,.>)
from scripts/gpu_session.sh's `valusnap` step: the PMC passes valu_<k>/ (one
per VALU_LIBS build; bh_snap.py on Y_t250 and Y_t450 with --reps 1, so two
dispatches per snapshot) and the pop counts of valusnap.jsonl (the counting
traversal of the same snapshots; the trees and decisions do not depend on
the build, so one build's counts serve all).

usage: python scripts/valu_summary.py gpurun_out/r5<TAG>
"""
import csv
import glob
import json
import os
import sys


def pmc_rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return []
    rows = list(csv.DictReader(open(files[0])))
    return rows


def main():
    out = sys.argv[1]
    # pops per snapshot, in file order, from any build that reported them
    pops, labels = {}, []
    for line in open(os.path.join(out, "valusnap.jsonl")):
        line = line.strip()
        if line.startswith("#"):
            labels.append(line[1:].strip())
            continue
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        if "pops" in r:
            pops[r["snapshot"]] = r
    snaps = sorted(pops)
    res = {"snapshots": {s: {k: pops[s][k] for k in ("pops", "child_slots", "tile_points", "visits")} for s in snaps},
           "builds": {}}
    for k, lab in enumerate(labels, start=1):
        rows = [r for r in pmc_rows(os.path.join(out, f"valu_{k}")) if "bh_traverse" in r.get("Kernel_Name", "")]
        # dispatch order: snapshot 0 (2 calls), snapshot 1 (2 calls)
        disp = {}
        for r in rows:
            disp.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(disp)
        per = {}
        for si, s in enumerate(snaps):
            mine = ids[2 * si:2 * si + 2]
            if len(mine) < 2:
                continue
            c = {n: sum(disp[i].get(n, 0.0) for i in mine) / 2 for n in disp[mine[0]]}
            p = pops[s]["pops"]
            per[s] = {"valu_per_pop": c.get("SQ_INSTS_VALU", 0) / p, "salu_per_pop": c.get("SQ_INSTS_SALU", 0) / p,
                      "lds_per_pop": c.get("SQ_INSTS_LDS", 0) / p,
                      "valu_per_child_slot": c.get("SQ_INSTS_VALU", 0) / max(1, pops[s]["child_slots"]),
                      "counters_per_call": c}
        res["builds"][lab] = per
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
