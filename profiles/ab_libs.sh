#!/bin/bash
# A/B of engine builds: bench.py (C3 line, no side legs) once per library, two rounds.
# Usage (on the box): bash profiles/ab_libs.sh ab/libA.so ab/libB.so ...
set -o pipefail
R=$GRAFT_REPO_ROOT
for round in ${ROUNDS:-1 2}; do
  for lib in "$@"; do
    MPPI_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 > $R/gpurun_out/ab.json 2>$R/gpurun_out/ab.err || { tail -5 $R/gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('$R/gpurun_out/ab.json')); c=d['config']; print('$lib', round(d['value']), 'sync', round(c['sync_steps_per_s']), 'fin', c['finish_kernel_avg_ms'], 'roll', d['roofline']['kernel_avg_ms'])"
    [ -n "$MPPI_HOST_TRACE" ] && grep "host trace" $R/gpurun_out/ab.err | head -4
  done
done
