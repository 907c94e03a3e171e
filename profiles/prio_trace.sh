#!/bin/bash
# Kernel traces of the C3 bench line (no side legs) at MPPI_WAVE_PRIO=0 and 1 (diagnostic).
# Usage (on the box): bash profiles/prio_trace.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for p in 1 0; do
  MPPI_WAVE_PRIO=$p timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_p$p -o t -- \
      python3 $R/bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 --no-c4 --no-c5 --no-bilinear --no-costmap \
      > $R/gpurun_out/tr_p$p.json 2> $R/gpurun_out/tr_p$p.err || exit 1
  python3 $R/profiles/trace_ab.py $(ls $R/gpurun_out/tr_p$p/*kernel_trace.csv | head -1)
done
