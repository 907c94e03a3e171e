"""Print a kernel timeline window from a rocprofv3 --kernel-trace CSV (diagnostic).
Usage: python profiles/trace_timeline.py <kernel_trace.csv> [start_index] [count]
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mppi" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
a = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:a + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("mppi::", "").split("(")[0][-40:]
    print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:7.1f} q{r['Queue_Id']} {name}")
