#!/bin/bash
# rocprofv3 kernel stats of the pipelined C3 bench for each library build (A/B by kernel trace).
# Usage (on the box): bash profiles/gpu_prof_ab.sh abl/a.so abl/b.so
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  MPPI_LIB_PATH=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profab_$tag -o k --output-format csv -- \
      python3 $R/bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c4 --no-c5 \
      > $O/profab_$tag.json 2> $O/profab_$tag.err || { tail -20 $O/profab_$tag.err; exit 1; }
  python3 - "$O/profab_$tag" "$lib" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/k_kernel_stats.csv", recursive=True)[0]
for x in csv.DictReader(open(f)):
    n = x["Name"]
    if any(k in n for k in ("rollout", "colfin", "tail", "noise")):
        print(sys.argv[2], n.split("(")[0].split("<")[0].split("::")[-1], x["Calls"], round(float(x["AverageNs"]) / 1e3, 2), "us avg",
              round(float(x["MinNs"]) / 1e3, 1), round(float(x["MaxNs"]) / 1e3, 1))
PY
done
