#!/bin/bash
# quick check: parity-bearing GPU tests + bench lines (resident server) + chain clock
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_golden.py tests/test_gpu_engine_variants.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/ptq_$TAG.txt 2>&1
rc=$?; tail -2 $O/ptq_$TAG.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/ptq_$TAG.txt | head; exit 1; }
BA="--warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard"
for st in 20 200 20 200; do
  timeout -k 10 300 python bench.py --steps $st $BA > $O/bq.json 2>$O/bq.err || { tail -5 $O/bq.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bq.json')); c=d['config']; ch=c['chain']; print('$st/5 value', d['value'], 'sync', c['sync_steps_per_s'], 'roll', d['roofline']['kernel_avg_ms'], 'leaf', ch['wg0_leaf_us'], 'cyc', ch['cycles_per_step'], 'spread', ch['wg_end_spread_us'])"
done
