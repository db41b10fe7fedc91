"""Kernel timeline of one optimizer iteration (cut at bbox_partial) from a
rocprofv3 kernel trace: start / end / duration in us and queue.

usage: python scripts/trace_one.py trace.csv ITER [T]"""
import csv
import re
import sys


def short(n):
    if "rocprim" in n:
        m = re.search(r"wrapped_(\w+?)_config", n)
        k = re.search(r"rocprim::ROCPRIM_\w+::detail::(\w+)<", n)
        return "rocprim:" + (m.group(1) if m else (k.group(1) if k else "?"))
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)(<[^()]*>)?\(", n)
    return (m.group(1) + (m.group(2) or "")[:20]) if m else n[:30]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
T = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
starts = [i for i, r in enumerate(rows) if "bbox_partial" in r["Kernel_Name"]]
its = list(zip(starts, starts[1:] + [len(rows)]))[-T:]
a, b = its[int(sys.argv[2]) - 1]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s = int(r["Start_Timestamp"]) - t0
    e = int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']} grid {r['Grid_Size_X']:>8} "
          f"wg {r['Workgroup_Size_X']:>4} lds {r['LDS_Block_Size']:>6} {short(r['Kernel_Name'])}")
