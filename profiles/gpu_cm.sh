#!/bin/bash
# Costmap builder check: GPU costmap tests, the bench's costmap leg, and a kernel trace of it.
# Usage (on the box): bash profiles/gpu_cm.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-cm}
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_costmap.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1 || { tail -30 $O/pt_$TAG.txt; exit 1; }
tail -1 $O/pt_$TAG.txt
timeout -k 10 120 python -c "import sys, json; sys.path[:0]=['$R', '$R/husky-rover-mppi-isaacsim_amd']; import bench; print(json.dumps(bench.costmap_bench(0, cpu=False)))" > $O/cm_$TAG.json 2>&1 || { tail -20 $O/cm_$TAG.json; exit 1; }
cat $O/cm_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o k --output-format csv -- \
    python3 -c "import sys; sys.path[:0]=['$R', '$R/husky-rover-mppi-isaacsim_amd']; import bench; bench.costmap_bench(0, reps=10, cpu=False)" > /dev/null 2> $O/prof_$TAG.err || { tail -5 $O/prof_$TAG.err; exit 1; }
python3 -c "
import csv
rows = list(csv.DictReader(open('$O/prof_$TAG/k_kernel_stats.csv')))
for r in rows: print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
