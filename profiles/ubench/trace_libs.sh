#!/bin/bash
# Kernel-trace medians of the C3 pipelined bench per library build (diagnostic).
# Usage (GPU box): bash profiles/ubench/trace_libs.sh abl/a.so abl/b.so ...
R=$GRAFT_REPO_ROOT
i=0
for lib in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && MPPI_LIB_PATH=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/tl$i -o tr --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c4 --no-c5 --no-sync-pass > $R/gpurun_out/tl$i.json 2> $R/gpurun_out/tl$i.err) || { tail -5 $R/gpurun_out/tl$i.err; exit 1; }
  echo "=== $lib $(python3 -c "import json; print(json.load(open('$R/gpurun_out/tl$i.json'))['value'])")"
  python3 $R/profiles/ubench/trace_stats.py $(ls $R/gpurun_out/tl$i/*kernel_trace.csv | head -1)
done
