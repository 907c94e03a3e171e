#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04g}
O=$R/gpurun_out
cd $R
MPPI_HOST_TRACE=1 timeout -k 10 120 python -u profiles/ubench/server_diag.py 100 > $O/diag_$TAG.txt 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids $O/diag_$TAG.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_variants.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/ptv_$TAG.txt 2>&1
rc=$?; tail -15 $O/ptv_$TAG.txt; [ $rc -eq 0 ] || exit 1
for env in "MPPI_RESIDENT=1" "MPPI_RESIDENT=0"; do
  for st in 20 200; do
  env $env timeout -k 10 300 python bench.py --steps $st --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard > $O/b2.json 2>$O/b2.err || { tail -5 $O/b2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b2.json')); c=d['config']; print('[$env] $st/5 value', d['value'], 'sync', c['sync_steps_per_s'], 'roll', d['roofline']['kernel_avg_ms'], 'sched', c['schedule'][:20])"
  done
done
