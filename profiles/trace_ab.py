"""Per-step intervals of the pipelined schedule from a rocprofv3 kernel-trace CSV (diagnostic).
Usage: python profiles/trace_ab.py <kernel_trace.csv>
Steps = consecutive role-split rollout launches; prints the median of each interval (us):
period, rollout, rollout end -> finish start, finish, finish end -> next rollout start, and
how far the previous step's tail and the step's noise reach into the rollout.
"""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mppi" in r["Kernel_Name"]]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
roll = [e for e in ev if "rollout_roles" in e[2] or "rollout_pair" in e[2]]
fin = [e for e in ev if "colfin" in e[2]]
tail = [e for e in ev if "tail_kernel" in e[2]]
noise = [e for e in ev if "noise_kernel" in e[2]]
out = {k: [] for k in ("period", "rollout", "roll_to_fin", "finish", "fin_to_next", "tail_over", "noise_over")}
for a, b in zip(roll[len(roll) // 3:], roll[len(roll) // 3 + 1:]):
    f = next((x for x in fin if x[0] >= a[1]), None)
    if f is None or f[1] > b[0]:
        continue
    out["period"].append(b[0] - a[0])
    out["rollout"].append(a[1] - a[0])
    out["roll_to_fin"].append(f[0] - a[1])
    out["finish"].append(f[1] - f[0])
    out["fin_to_next"].append(b[0] - f[1])
    t = [x for x in tail if x[0] < a[0] < x[1]]
    out["tail_over"].append((t[-1][1] - a[0]) if t else 0)
    n = [x for x in noise if x[0] < b[0] < x[1]]
    out["noise_over"].append((n[-1][1] - b[0]) if n else 0)
print(sys.argv[1], len(out["period"]), "steps")
for k, v in out.items():
    if v:
        print(f"  {k:12s} median {statistics.median(v) / 1000:7.1f}  mean {statistics.mean(v) / 1000:7.1f}")
