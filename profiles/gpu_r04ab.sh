#!/bin/bash
# A/B of library builds (MPPI_LIB_PATH), alternating, C3 bench lines with the chain clock.
# Usage (on the box): bash profiles/gpu_r04ab.sh <tag> <rounds> <steps> lib1 [lib2 ...]   ("-" = the in-tree library)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; RN=$2; ST=$3; shift 3
O=$R/gpurun_out
cd $R
BA="--warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard"
for r in $(seq 1 $RN); do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset MPPI_LIB_PATH; else export MPPI_LIB_PATH=$R/$lib; fi
    timeout -k 10 300 python bench.py --steps $ST $BA > $O/ab_$TAG.json 2>$O/ab_$TAG.err || { tail -5 $O/ab_$TAG.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_$TAG.json')); c=d['config']; ch=c['chain']; print('$lib', 'value', d['value'], 'sync', c['sync_steps_per_s'], 'roll', d['roofline']['kernel_avg_ms'], 'leaf', ch['wg0_leaf_us'], 'cyc', ch['cycles_per_step'], 'srv_roll', c.get('server_rollout_us'))"
  done
done
