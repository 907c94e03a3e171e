#!/bin/bash
# A/B: three-launch schedule vs the fused launch with the noise gated on its rollout part
# (MPPI_FUSED=2 MPPI_FUSED_NOISE_GROUPS=-2), then a kernel-trace window of the gated one.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash profiles/ab_env2.sh "MPPI_X=0" "MPPI_FUSED=2 MPPI_FUSED_NOISE_GROUPS=-2" || exit 1
cd /tmp && export TMPDIR=/tmp
MPPI_FUSED=2 MPPI_FUSED_NOISE_GROUPS=-2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_g -o t -- python3 $R/bench.py --steps 60 --warmup 10 --cpu-baseline-seconds 0 --no-c4 --no-c5 --no-bilinear --no-costmap > /dev/null 2>&1 || exit 1
cd $R && python3 profiles/trace_timeline.py $(ls $R/gpurun_out/tr_g/*kernel_trace.csv | head -1) 300 18
