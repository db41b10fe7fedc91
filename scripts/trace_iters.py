"""Per-iteration view of a rocprofv3 kernel trace of bench.py: iterations are
cut at each tree build's first kernel (bbox_partial / bbox3_partial), the
warmup's builds skipped.  For the chosen iterations of the timed schedule:
the kernel sequence (start offset, duration) and the iteration's span; and a
per-100-iteration table of span and of the summed time per kernel family.

usage: python scripts/trace_iters.py <kernel_trace.csv> [--warmup-iters 250] [--show 250,700,900]
"""
import argparse
import csv
from collections import defaultdict


def family(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    base = base.split("::")[-1]
    return base.split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup-iters", type=int, default=250)
    ap.add_argument("--show", default="250,700,900")
    ap.add_argument("--marker", default="bbox_partial,bbox3_partial")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = set(a.marker.split(","))
    starts = [i for i, r in enumerate(rows) if family(r["Kernel_Name"]) in marks]
    starts = starts[a.warmup_iters:]
    iters = []
    for k, i0 in enumerate(starts):
        i1 = starts[k + 1] if k + 1 < len(starts) else len(rows)
        iters.append(rows[i0:i1])
    show = {int(v) for v in a.show.split(",") if v}
    for t, seg in enumerate(iters, start=1):
        if t not in show:
            continue
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in seg)
        print(f"iteration {t}: span {(t1 - t0) / 1e3:.1f} us, {len(seg)} kernels")
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"  {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {family(r['Kernel_Name'])}")
    print("\nper 100 iterations: mean span (us) and mean summed kernel time per family (us)")
    fams = defaultdict(lambda: defaultdict(float))
    spans = defaultdict(list)
    for t, seg in enumerate(iters, start=1):
        b = (t - 1) // 100
        t0 = int(seg[0]["Start_Timestamp"])
        spans[b].append((int(iters[t][0]["Start_Timestamp"]) if t < len(iters) else max(int(r["End_Timestamp"]) for r in seg)) - t0)
        for r in seg:
            fams[b][family(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for b in sorted(spans):
        nit = len(spans[b])
        top = sorted(fams[b].items(), key=lambda kv: -kv[1])[:8]
        print(f"t {100 * b + 1:4d}-{100 * b + 100:4d}: span {sum(spans[b]) / nit / 1e3:8.1f}  " +
              "  ".join(f"{k} {v / nit / 1e3:.0f}" for k, v in top))


if __name__ == "__main__":
    main()
