"""Summarise rocprofv3 --pmc passes (profiles/pmc.sh) into per-kernel per-launch averages.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM for gfx950:
  read bytes  = FETCH_SIZE (KiB) * 1024 * 2   (FETCH_SIZE counts half of a wide streaming read)
  write bytes = WRITE_SIZE (KiB) * 1024
Writes the JSON that bench.py reads for roofline.traffic (profiles/pmc_latest.json), tagged
with the kernel-source hash (bench.source_hash) and the git commit the sources came from
(GIT_HEAD in the environment: the GPU box has no .git); bench.py refuses a summary whose source
hash differs from the sources it runs.

usage: python pmc_summary.py <pmc dir> [K H]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.strip('"')
    for key in ("mppi_rollout_roles_kernel", "mppi_rollout_pair_kernel", "mppi_step_fused_kernel", "mppi_noise_kernel",
                "mppi_tail_kernel", "mppi_gate_kernel", "mppi_colfin_kernel", "mppi_finish_kernel",
                "mppi_bilinear_kernel"):
        if key in name:
            return key
    return name.split("(")[0][:60]


def main(root, K=65536, H=100):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row.get("Kernel_Name", ""))
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, counters in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in counters.items()}
        d = out[k]
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
    roll = (out.get("mppi_rollout_roles_kernel") or out.get("mppi_rollout_pair_kernel") or {})
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    summary = {"K": K, "H": H, "src_sha256": bench.source_hash(), "git_head": os.environ.get("GIT_HEAD"),
               "kernels": out,
               "hbm_bytes_per_launch": roll.get("hbm_bytes_per_launch"),
               "kernel": next((k for k, v in out.items() if v is roll), None)}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:4]))
