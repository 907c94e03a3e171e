#!/bin/bash
# A/B of bench.py argument sets on the C3 bench line (no side legs), alternating rounds.
# Usage (on the box): ROUNDS="1 2 3" bash profiles/ab_args.sh "" "--no-timed-events" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
for round in ${ROUNDS:-1 2}; do
  for v in "$@"; do
    timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 $v > $R/gpurun_out/ab.json 2>$R/gpurun_out/ab.err || { tail -5 $R/gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('$R/gpurun_out/ab.json')); c=d['config']; print('[$v]', round(d['value']), 'sync', round(c['sync_steps_per_s']), 'fin', c['finish_kernel_avg_ms'], 'roll', d['roofline']['kernel_avg_ms'])"
  done
done
