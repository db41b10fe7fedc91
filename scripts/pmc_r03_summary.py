"""Summarise scripts/gpu_pmc_r03.sh into profiles/r03_attract_traffic.json
(HBM bytes per non-loss attract_tiles launch over the bench's timed region:
FETCH_SIZE x 2, the calibrated gfx950 correction of scripts/pmc_calib.hip,
+ WRITE_SIZE, both in KiB) and profiles/r03_bh_valu.json (VALU issue of the
BH kernels: SQ_INSTS_VALU x 4 cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs))."""
import csv
import json
from collections import defaultdict
from pathlib import Path

OUT = Path("gpurun_out")
PROF = Path("profiles")


def counters(kind):
    d = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(OUT / kind / "pmc_counter_collection.csv")):
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    return d, names


def plain(name):
    return "attract_tiles" in name and ", false," in name


fd, fn = counters("pmc_fetch")
wd, wn = counters("pmc_write")
fetch = [fd[k]["FETCH_SIZE"] * 1024.0 for k in sorted(fd) if plain(fn[k])]
write = [wd[k]["WRITE_SIZE"] * 1024.0 for k in sorted(wd) if plain(wn[k])]
traffic = 2.0 * sum(fetch) / len(fetch) + sum(write) / len(write)
(PROF / "r03_attract_traffic.json").write_text(json.dumps({
    "kernel": "attract_tiles<LOSS=false>",
    "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) -- python bench.py --no-cpu-baseline "
              "--trace 0 (scripts/gpu_pmc_r03.sh): every non-loss launch of the bench run (warmup window + timed schedule)",
    "unit": "bytes per launch",
    "launches": len(fetch),
    "fetch_bytes_raw_mean": sum(fetch) / len(fetch),
    "write_bytes_mean": sum(write) / len(write),
    "traffic_bytes_per_launch": traffic,
    "correction": "FETCH_SIZE x 2: every streaming width reports 1/2 of its bytes on gfx950 (scripts/pmc_calib.hip, "
                  "profiles/r02_attract_traffic.json calibration)",
}, indent=1) + "\n")
vd, vn = counters("pmc_valu")
agg = defaultdict(lambda: defaultdict(float))
for k in vd:
    nm = "bh_traverse" if "bh_traverse" in vn[k] else "tile_apply"
    for c, v in vd[k].items():
        agg[nm][c] += v
res = {}
for nm, c in agg.items():
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    res[nm] = {"valu_issue_frac": c["SQ_INSTS_VALU"] * 4.0 / (cyc * 1024.0) if cyc else None,
               "valu_insts": c["SQ_INSTS_VALU"], "kernel_cycles_per_xcd": cyc}
(PROF / "r03_bh_valu.json").write_text(json.dumps({
    "note": "BH kernels over the bench's whole run (warmup window + timed schedule): fp64 VALU issue fraction = "
            "SQ_INSTS_VALU x 4 cycles (a wave64 fp64 VALU op) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); "
            "scripts/gpu_pmc_r03.sh",
    "kernels": res}, indent=1) + "\n")
print(open(PROF / "r03_attract_traffic.json").read())
print(open(PROF / "r03_bh_valu.json").read())
