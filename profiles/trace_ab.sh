#!/bin/bash
# Kernel-trace timelines of the C3 bench under engine env toggles (diagnostic).
# Usage (on the box): bash profiles/trace_ab.sh "MPPI_X=0" "MPPI_X=1" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  export $v
  timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/tr$i -o tr --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 > /dev/null 2>&1 || exit 1
  echo "== $v"
  python3 $R/profiles/trace_timeline.py $(ls $R/gpurun_out/tr$i/*kernel_trace.csv | head -1) 300 14
  unset ${v%%=*}
  i=$((i+1))
done
