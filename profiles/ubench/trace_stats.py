"""Per-kernel medians and the step period from a rocprofv3 --kernel-trace CSV (diagnostic).
Usage: python profiles/ubench/trace_stats.py <kernel_trace.csv> [main kernel substring]"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mppi" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
main = sys.argv[2] if len(sys.argv) > 2 else "step_fused"
by = {}
for r in rows:
    name = r["Kernel_Name"].replace("mppi::", "").split("(")[0].split("<")[0]
    by.setdefault(name, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for name, v in sorted(by.items()):
    d = np.array([e - s for s, e in v]) / 1000.0
    print(f"  {name:34s} n={len(v):4d} median {np.median(d):7.2f} us  p10 {np.percentile(d, 10):7.2f}  p90 {np.percentile(d, 90):7.2f}")
m = [k for k in by if main in k]
if m:
    v = by[m[0]][len(by[m[0]]) // 4:]  # skip warmup
    st = np.array([s for s, _ in v]) / 1000.0
    en = np.array([e for _, e in v]) / 1000.0
    per = np.diff(st)
    gap = st[1:] - en[:-1]
    print(f"  {m[0]} period median {np.median(per):.2f} us (p10 {np.percentile(per, 10):.2f}, p90 {np.percentile(per, 90):.2f}); "
          f"end -> next start median {np.median(gap):.2f} us")
