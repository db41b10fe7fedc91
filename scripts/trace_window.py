"""Print the kernel sequence of one timed-window iteration (and one loss
iteration) from a rocprofv3 kernel trace: start offset, duration, kernel.

usage: python scripts/trace_window.py [gpurun_out/prof/prof_kernel_trace.csv] [nth attraction launch]
"""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/prof_kernel_trace.csv"
nth = int(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
att = [i for i, r in enumerate(rows) if "attract_rows" in r["Kernel_Name"]]
loss = [i for i in att if ", true," in rows[i]["Kernel_Name"]]
for label, i0 in (("window iteration", att[nth]), ("loss iteration", loss[min(2, len(loss) - 1)])):
    print(label)
    t0 = int(rows[i0 - 14]["Start_Timestamp"])
    for r in rows[i0 - 14:i0 + 8]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {r['Kernel_Name'][:90]}")
