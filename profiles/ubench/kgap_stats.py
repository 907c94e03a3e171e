"""Gaps B.start - A.end per mode from the kgap trace (diagnostic)."""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows]
mode, gaps, lastA = 0, {0: [], 1: [], 2: [], 3: []}, None
for i, (n, s, e, q) in enumerate(ev):
    if n.endswith("ka"):
        lastA = e
    elif n.endswith("kb") and lastA is not None:
        gaps[mode].append((s - lastA) / 1000.0)
        lastA = None
    elif n.endswith("kc") and (i + 1 == len(ev) or ev[i + 1][0].endswith("ka")) and q != ev[i - 1][3]:
        pass
    if n.endswith("kc") and i + 1 < len(ev) and ev[i + 1][0].endswith("ka") and len(gaps[mode]) >= 200:
        mode += 1
names = ["A->B", "A->record->B", "A->record(waited by s2)->B", "A stores pinned->B"]
for m in range(4):
    g = np.array(gaps[m][20:])
    if g.size:
        print(f"  {names[m]:30s} n={g.size:4d} gap median {np.median(g):6.2f} us  p10 {np.percentile(g, 10):6.2f}  p90 {np.percentile(g, 90):6.2f}")
