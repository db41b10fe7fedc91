"""Per-kernel average time per iteration, by phase window, from a rocprofv3
kernel trace of bench.py (iterations cut at bbox_partial, as trace_iters.py).

usage: python scripts/trace_kernels.py trace.csv [T]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    if "rocprim" in name:
        m = re.search(r"wrapped_(\w+?)_config", name)
        return "rocprim:" + (m.group(1) if m else "?")
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")[:24]) if m else name[:40]


def main(path, T=1000, windows=((1, 150), (150, 200), (200, 300), (300, 450), (450, 650), (650, 800), (800, 1001))):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "bbox_partial" in r["Kernel_Name"]]
    its = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        acc = defaultdict(float)
        for r in rows[a:b]:
            acc[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        its.append(acc)
    its = its[-T:]
    for lo, hi in windows:
        sel = its[lo - 1:hi - 1]
        if not sel:
            continue
        tot = defaultdict(float)
        for a in sel:
            for k, v in a.items():
                tot[k] += v / len(sel)
        top = sorted(tot.items(), key=lambda x: -x[1])
        print("t %d-%d: " % (lo, hi - 1) + ", ".join("%s %.1f" % (k, v) for k, v in top if v >= 2.0))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:3]))
