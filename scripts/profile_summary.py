"""Summarise a `STEPS=ktrace bash scripts/gpu_session.sh` run (rocprofv3 --kernel-trace
--stats of the default bench) into profiles/:

  <tag>_rocprof_kernel_stats.csv   rocprofv3 --stats of `bench.py` (warmup + whole timed schedule)
  <tag>_attract_dispatches.json    attract_tiles dispatch durations from the kernel trace: the non-loss
                                   launches (the roofline kernel) and the loss launches (t = 10 k) of the
                                   timed schedule, averaged over it and per 100-iteration bucket

usage: python scripts/profile_summary.py <tag> --dir gpurun_out/r4<TAG>/ktrace [--warmup-iters 250]
"""
import argparse
import csv
import json
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PROF = ROOT / "profiles"


def rows(p):
    with open(p) as fh:
        return list(csv.DictReader(fh))


def attract(name, loss):
    return "attract_tiles<" in name and (", true," if loss else ", false,") in name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--dir", required=True)
    ap.add_argument("--warmup-iters", type=int, default=250,
                    help="iterations the bench's warmup runs before the timed schedule (W steps x T/K)")
    ap.add_argument("--iterations", type=int, default=1000)
    a = ap.parse_args()
    d = Path(a.dir)
    stats = next(d.rglob("*kernel_stats.csv"))
    trace = next(d.rglob("*kernel_trace.csv"))
    shutil.copy(stats, PROF / f"{a.tag}_rocprof_kernel_stats.csv")
    tr = sorted(rows(trace), key=lambda r: int(r["Dispatch_Id"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    W = a.warmup_iters
    plain = [r for r in tr if attract(r["Kernel_Name"], False)]
    loss = [r for r in tr if attract(r["Kernel_Name"], True)]
    plain = plain[W - W // 10:]
    loss = loss[W // 10:]
    pits = [t for t in range(1, a.iterations + 1) if t % 10]
    lits = list(range(10, a.iterations + 1, 10))
    pd = dict(zip(pits, map(dur, plain)))
    ld = dict(zip(lits, map(dur, loss)))
    buckets = {}
    for b in range(0, a.iterations, 100):
        v = [x for t, x in pd.items() if b < t <= b + 100]
        if v:
            buckets[f"{b + 1}-{b + 100}"] = sum(v) / len(v)
    out = {
        "source": "rocprofv3 --kernel-trace --stats -- python bench.py --no-cpu-baseline --trace 0 "
                  "(scripts/gpu_session.sh ktrace); attract_tiles dispatches after the warmup's %d iterations" % W,
        "launches": len(pd),
        "avg_ms_schedule": sum(pd.values()) / len(pd) if pd else None,
        "avg_ms_per_100_iterations": buckets,
        "loss_launches": {"launches": len(ld), "avg_ms_schedule": sum(ld.values()) / len(ld) if ld else None},
    }
    (PROF / f"{a.tag}_attract_dispatches.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
