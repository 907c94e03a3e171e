#!/bin/bash
# Round 4: the resident step server.  Microbench of a resident loop vs one launch per step, the
# schedule tests, the headline parity tests, then C3 bench lines (server vs separate launches).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04b}
O=$R/gpurun_out
cd $R
timeout -k 10 90 ./profiles/ubench/server_bin 70 2000 > $O/server_$TAG.txt 2>&1; echo "server ubench rc=$?"; cat $O/server_$TAG.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_variants.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/ptv_$TAG.txt 2>&1
rc=$?; tail -25 $O/ptv_$TAG.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1
rc=$?; tail -3 $O/pt_$TAG.txt; grep -E "reference-f32" $O/pt_$TAG.txt; [ $rc -eq 0 ] || exit 1
for env in "MPPI_RESIDENT=1" "MPPI_RESIDENT=0"; do
  for st in 20 200; do
    env $env MPPI_HOST_TRACE=1 timeout -k 10 300 python bench.py --steps $st --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 > $O/b2.json 2>$O/b2.err || { tail -5 $O/b2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b2.json')); c=d['config']; print('[$env] steps $st value', d['value'], 'sync', c['sync_steps_per_s'], 'roll', d['roofline']['kernel_avg_ms'], 'sched', c['schedule'][:20], 'chain', c['chain']['cycles_per_step'], c['chain']['wg_end_spread_us'], c['chain']['wg0_leaf_us'])"
    grep "host trace" $O/b2.err | tail -2
  done
done
