#!/bin/bash
# Kernel-trace medians of the C3 pipelined bench per environment setting (diagnostic).
# Usage (GPU box): bash profiles/ubench/trace_env.sh "MPPI_ARM=1" "MPPI_ARM=0" ...
R=$GRAFT_REPO_ROOT
i=0
for v in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && env $v timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/te$i -o tr --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c4 --no-c5 --no-sync-pass > $R/gpurun_out/te$i.json 2> $R/gpurun_out/te$i.err) || { tail -5 $R/gpurun_out/te$i.err; exit 1; }
  echo "=== $v $(python3 -c "import json; d=json.load(open('$R/gpurun_out/te$i.json')); print(d['value'], d['config'].get('arm'))")"
  python3 $R/profiles/ubench/trace_stats.py $(ls $R/gpurun_out/te$i/*kernel_trace.csv | head -1) rollout_roles
done
