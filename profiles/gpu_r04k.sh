#!/bin/bash
# round 4: uniform-pick optimal-rollout chain + server relaunch without memsets: diag, tests that
# cover the tail (golden async/sync, headline C3 vs oracle, variants), benches
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04k}
O=$R/gpurun_out
cd $R
MPPI_HOST_TRACE=1 timeout -k 10 200 python -u profiles/ubench/server_diag.py 100 > $O/diag_$TAG.txt 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids $O/diag_$TAG.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine_variants.py tests/test_gpu_golden.py tests/test_gpu_headline.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/ptv_$TAG.txt 2>&1
rc=$?; tail -4 $O/ptv_$TAG.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/ptv_$TAG.txt | head; exit 1; }
BA="--warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard"
for i in 1 2; do for env in "MPPI_RESIDENT=1" "MPPI_RESIDENT=0"; do for st in 20 200; do
  env $env timeout -k 10 300 python bench.py --steps $st $BA > $O/b2.json 2>$O/b2.err || { tail -5 $O/b2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b2.json')); c=d['config']; print('[$env] $st/5 value', d['value'], 'sync', c['sync_steps_per_s'], 'roll', d['roofline']['kernel_avg_ms'], 'tail', c.get('tail_kernel_avg_ms'), 'fin', c.get('finish_kernel_avg_ms'))"
done; done; done
