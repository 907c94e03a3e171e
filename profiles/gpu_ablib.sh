#!/bin/bash
# A/B of library builds in abl/ (C3 line + C4 leg), two rounds.  Usage: bash profiles/gpu_ablib.sh abl/a.so abl/b.so
set -o pipefail
R=$GRAFT_REPO_ROOT
for round in ${ROUNDS:-1 2}; do
  for lib in "$@"; do
    MPPI_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 $BENCH_ARGS > $R/gpurun_out/ab.json 2>$R/gpurun_out/ab.err || { tail -5 $R/gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('$R/gpurun_out/ab.json')); c=d['config']; ch=c['chain']; print('$lib', round(d['value']), 'sync', round(c['sync_steps_per_s']), 'roll', d['roofline']['kernel_avg_ms'], 'c4', d.get('c4',{}).get('steps_per_s'), 'chain_us', ch['chain_us'], 'leaf', ch['wg0_leaf_us'], 'tail', c.get('tail_kernel_avg_ms'), 'span', ch.get('wg_span_us'), 'spread', ch.get('wg_start_spread_us'), ch.get('wg_end_spread_us'), 'info', c['rollout_kernel'].get('ucache_steps'))"
  done
done
