#!/bin/bash
# A/B of library builds (MPPI_LIB_PATH): C3 value, sync, C4 on one GPU and the C4-shard step.
# Usage (on the box): bash profiles/gpu_r04abc.sh <tag> <rounds> lib1 [lib2 ...]   ("-" = the in-tree library)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; RN=$2; shift 2
O=$R/gpurun_out
cd $R
BA="--steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5"
for r in $(seq 1 $RN); do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset MPPI_LIB_PATH; else export MPPI_LIB_PATH=$R/$lib; fi
    timeout -k 10 300 python bench.py $BA > $O/abc_$TAG.json 2>$O/abc_$TAG.err || { tail -5 $O/abc_$TAG.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/abc_$TAG.json')); c=d['config']; s=d['c4_shard']; print('$lib', 'value', d['value'], 'sync', c['sync_steps_per_s'], 'c4', d['c4']['steps_per_s'], 'shard', s['sharded_ms_per_step'], 'plain', s['plain_ms_per_step'])"
  done
done
