"""Summarise a scripts/gpu_check.sh run (gpurun_out/) into profiles/:

  <tag>_rocprof_kernel_stats.csv     rocprofv3 --stats of `bench.py --steps K --warmup W` (whole schedule)
  <tag>_attract_dispatches.json      attract_tiles / attract_rows dispatch durations from the kernel trace: the
                                     non-loss launches (roofline kernel; the k-th after the warmup's is the k-th
                                     t with t % 10 != 0) and the loss launches (t = 10 k), averaged over the
                                     timed window t <= K and the whole schedule
  r02_attract_traffic.json           FETCH_SIZE / WRITE_SIZE per non-loss launch in the window
                                     (separate PMC passes of `bench.py --no-rest`), corrected by the
                                     calibration run (scripts/pmc_calib.hip)

usage: python scripts/profile_summary.py <tag> [--steps K] [--warmup W]
"""
import argparse
import csv
import json
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "gpurun_out"
PROF = ROOT / "profiles"


def rows(p):
    with open(p) as fh:
        return list(csv.DictReader(fh))


def is_loss_attraction(name):
    """The loss (LOSS=true) attraction kernel: attract_tiles<true, MET> (the
    optimizer's tiled layout) or attract_rows<LPR, U, true, MET> (CSR rows)."""
    return ("attract_tiles<" in name or "attract_rows<" in name) and ", true," in name


def is_plain_attraction(name):
    """The non-loss attraction kernel (the roofline kernel): attract_tiles<false, MET>
    or attract_rows<LPR, U, false, MET>."""
    return ("attract_tiles<" in name or "attract_rows<" in name) and ", false," in name


def kernel_label(name):
    loss = ", true," in name
    base = "attract_tiles<LOSS=%s>" if "attract_tiles<" in name else "attract_rows<64,4,LOSS=%s>"
    return base % ("true" if loss else "false")


def dispatches(trace_rows, pred):
    """Dispatches of the selected attraction kernel, in dispatch order."""
    sel = [r for r in trace_rows if pred(r["Kernel_Name"])]
    return sorted(sel, key=lambda r: int(r["Dispatch_Id"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    K, W = a.steps, a.warmup
    warm_loss = W // 10          # loss iterations inside the warmup (t = 10, 20, ... <= W)
    warm_plain = W - warm_loss   # non-loss iterations inside the warmup

    shutil.copy(OUT / "prof" / "prof_kernel_stats.csv", PROF / f"{a.tag}_rocprof_kernel_stats.csv")
    tr = rows(OUT / "prof" / "prof_kernel_trace.csv")
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    # the roofline kernel: non-loss launches, iteration t = the k-th t with t % 10 != 0
    pd = dispatches(tr, is_plain_attraction)[warm_plain:]
    pits = [t for t in range(1, 100000) if t % 10][:len(pd)]
    pdur = [dur(r) for r in pd]
    pwin = [d for t, d in zip(pits, pdur) if t <= K]
    ld = dispatches(tr, is_loss_attraction)[warm_loss:]
    ldur = [dur(r) for r in ld]
    lits = [10 * (k + 1) for k in range(len(ldur))]
    lwin = [d for t, d in zip(lits, ldur) if t <= K]
    label = kernel_label(pd[0]["Kernel_Name"]) if pd else "attract_rows<64,4,LOSS=false>"
    summary = {
        "source": "rocprofv3 --kernel-trace --stats -- python bench.py --steps %d --warmup %d --no-cpu-baseline "
                  "(scripts/gpu_check.sh); dispatches of %s after the warmup's" % (K, W, label),
        "launches": len(pdur),
        "avg_ms_window": sum(pwin) / len(pwin) if pwin else None,
        "avg_ms_whole_schedule": sum(pdur) / len(pdur) if pdur else None,
        "per_launch_ms_window": dict(zip(map(str, pits), pwin)),
        "loss_launches": {"kernel": kernel_label(ld[0]["Kernel_Name"]) if ld else None,
                          "avg_ms_window": sum(lwin) / len(lwin) if lwin else None,
                          "avg_ms_whole_schedule": sum(ldur) / len(ldur) if ldur else None,
                          "per_launch_ms": dict(zip(map(str, lits), ldur))},
    }
    (PROF / f"{a.tag}_attract_dispatches.json").write_text(json.dumps(summary, indent=1) + "\n")

    # PMC: per non-loss launch in the window (bench.py --no-rest: the window's launches only)
    def per_launch(kind, counter):
        rs = [r for r in rows(OUT / kind / "pmc_counter_collection.csv")
              if is_plain_attraction(r["Kernel_Name"]) and r["Counter_Name"] == counter]
        rs.sort(key=lambda r: int(r["Dispatch_Id"]))
        return [float(r["Counter_Value"]) * 1024.0 for r in rs[warm_plain:]]   # KiB -> bytes
    fetch = per_launch("pmc_fetch", "FETCH_SIZE")
    write = per_launch("pmc_write", "WRITE_SIZE")
    # calibration: FETCH_SIZE of known-byte streams and gathers
    cal = {}
    calp = OUT / "pmc_calib_fetch" / "pmc_counter_collection.csv"
    if calp.exists():
        known = 512 * 2 ** 20
        for r in rows(calp):
            k = r["Kernel_Name"]
            v = float(r["Counter_Value"]) * 1024.0
            if "read_stream<int>" in k:
                cal.setdefault("stream_4B_per_lane", []).append(v / known)
            elif "read_stream<double>" in k:
                cal.setdefault("stream_8B_per_lane", []).append(v / known)
            elif "read_stream<HIP_vector_type" in k:
                cal.setdefault("stream_16B_per_lane", []).append(v / known)
            elif "gather16" in k:
                cal.setdefault("gather_16B_bytes_per_gather", []).append(v / (64 * 2 ** 20))
        cal = {k: sum(v) / len(v) for k, v in cal.items()}
    corr = 2.0   # every streaming width reports 1/2 of its bytes (calibration above)
    tf = PROF / "r02_attract_traffic.json"
    tj = json.loads(tf.read_text()) if tf.exists() else {}
    tj.update({
        "kernel": label,
        "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) -- python bench.py --steps K "
                  "--warmup W --no-rest --no-cpu-baseline --trace 0 (scripts/gpu_check.sh)",
        "unit": "bytes per launch",
        "calibration": {"FETCH_SIZE_reported_over_known": cal,
                        "note": "scripts/pmc_calib.hip: 512 MiB streams of 4/8/16-B-per-lane loads each report "
                                "exactly 1/2 of their bytes (the guide's x2 holds for every width here); a random "
                                "16-B gather from a 16 MiB table reports ~48 B, i.e. ~97 B of fabric traffic per "
                                "gather after the x2 (a line per gather: the table misses the 4 MiB L2)"},
    })
    tj.setdefault("per_window", {})[f"steps{K}"] = {
        "fetch_bytes_raw": fetch, "write_bytes": write,
        "traffic_bytes": (corr * sum(fetch) / len(fetch) + sum(write) / len(write)) if fetch and write else None,
        "note": f"window t=1..{K} ({len(fetch)} non-loss launches), FETCH_SIZE x2 (calibrated) + WRITE_SIZE",
    }
    tf.write_text(json.dumps(tj, indent=1) + "\n")
    print(json.dumps(summary, indent=1))
    print(json.dumps(tj["per_window"], indent=1))


if __name__ == "__main__":
    main()
