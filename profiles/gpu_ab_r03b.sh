#!/bin/bash
# A/B: the fused step launch with the deferred tail (noise inside the launch / before it) against
# the three-launch schedule, two alternating rounds, plus a kernel-trace window of the fused one.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash profiles/ab_env2.sh "MPPI_X=0" "MPPI_FUSED=2" "MPPI_FUSED=2 MPPI_FUSED_NOISE_GROUPS=0" || exit 1
cd /tmp && export TMPDIR=/tmp
MPPI_FUSED=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_f2 -o t -- python3 $R/bench.py --steps 60 --warmup 10 --cpu-baseline-seconds 0 --no-c4 --no-c5 --no-bilinear --no-costmap > /dev/null 2>&1 || exit 1
cd $R && python3 profiles/trace_timeline.py $(ls $R/gpurun_out/tr_f2/*kernel_trace.csv | head -1) 300 16
