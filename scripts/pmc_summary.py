"""Summarise scripts/gpu_pmc.sh: `python scripts/pmc_summary.py <tag> [commit]`.

profiles/<tag>_attract_traffic.json: HBM bytes per non-loss launch of the
gradient kernels over the bench's run (FETCH_SIZE x 2, the calibrated gfx950
correction of scripts/pmc_calib.hip, + WRITE_SIZE, both reported in KiB);
attract_tiles<LOSS=false> is the key bench.py reads for roofline.traffic.
profiles/<tag>_bh_valu.json: VALU issue of the BH kernels:
SQ_INSTS_VALU x 4 cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

OUT = Path("gpurun_out")
PROF = Path("profiles")
tag = sys.argv[1]
commit = sys.argv[2] if len(sys.argv) > 2 else None


def counters(kind):
    d = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(OUT / kind / "pmc_counter_collection.csv")):
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    return d, names


def label(name):
    if "attract_tiles" in name:
        return "attract_tiles<LOSS=false>" if ", false," in name else None
    for k in ("combine_update", "center2"):
        if k in name:
            return k
    return None


def per_kernel(kind, ctr):
    d, names = counters(kind)
    out = defaultdict(list)
    for k in sorted(d):
        lb = label(names[k])
        if lb:
            out[lb].append(d[k][ctr] * 1024.0)
    return out


fetch, write = per_kernel("pmc_fetch", "FETCH_SIZE"), per_kernel("pmc_write", "WRITE_SIZE")
kern = {}
for lb in fetch:
    f, w = fetch[lb], write.get(lb, [])
    if not f or not w:
        continue
    fm, wm = sum(f) / len(f), sum(w) / len(w)
    kern[lb] = {"launches": len(f), "fetch_bytes_raw_mean": fm, "write_bytes_mean": wm,
                "traffic_bytes_per_launch": 2.0 * fm + wm}
at = kern.get("attract_tiles<LOSS=false>", {})
(PROF / f"{tag}_attract_traffic.json").write_text(json.dumps({
    "kernel": "attract_tiles<LOSS=false>",
    "commit": commit,
    "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) -- python bench.py --no-cpu-baseline "
              "--trace 0 (scripts/gpu_pmc.sh): every non-loss launch of the bench run (warmup window + timed schedule)",
    "unit": "bytes per launch",
    "launches": at.get("launches"),
    "fetch_bytes_raw_mean": at.get("fetch_bytes_raw_mean"),
    "write_bytes_mean": at.get("write_bytes_mean"),
    "traffic_bytes_per_launch": at.get("traffic_bytes_per_launch"),
    "kernels": kern,
    "correction": "FETCH_SIZE x 2: every streaming width reports 1/2 of its bytes on gfx950 (scripts/pmc_calib.hip, "
                  "profiles/r02_attract_traffic.json calibration)",
}, indent=1) + "\n")
vd, vn = counters("pmc_valu")
agg = defaultdict(lambda: defaultdict(float))
for k in vd:
    nm = ("bh_traverse_narrow" if "bh_traverse_narrow" in vn[k] else
          "bh_traverse" if "bh_traverse" in vn[k] else "tile_apply")
    for c, v in vd[k].items():
        agg[nm][c] += v
res = {}
for nm, c in agg.items():
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    res[nm] = {"valu_issue_frac": c["SQ_INSTS_VALU"] * 4.0 / (cyc * 1024.0) if cyc else None,
               "valu_insts": c["SQ_INSTS_VALU"], "kernel_cycles_per_xcd": cyc}
(PROF / f"{tag}_bh_valu.json").write_text(json.dumps({
    "commit": commit,
    "note": "BH kernels over the bench's whole run (warmup window + timed schedule): fp64 VALU issue fraction = "
            "SQ_INSTS_VALU x 4 cycles (a wave64 fp64 VALU op) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); "
            "scripts/gpu_pmc.sh. The narrow kernel runs beside the 64-query one (a second stream), so its "
            "GRBM_GUI_ACTIVE overlaps the other's.",
    "kernels": res}, indent=1) + "\n")
print(open(PROF / f"{tag}_attract_traffic.json").read())
print(open(PROF / f"{tag}_bh_valu.json").read())
