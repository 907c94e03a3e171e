#!/bin/bash
# role-split kernel with blocks in turn (MPPI_ROLES=1) against the pair kernel (0) at C4, C5 and the
# C4 shard; the variant tests first (the role-split kernel at 1024 blocks runs 4 per workgroup)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_variants.py tests/test_gpu_c5.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/ptr.txt 2>&1
rc=$?; tail -2 $O/ptr.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/ptr.txt | head; exit 1; }
for i in 1 2; do for r in 1 0; do
  MPPI_ROLES=$r timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-sync-pass > $O/br.json 2>$O/br.err || { tail -5 $O/br.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/br.json')); print('ROLES=$r c3', d['value'], 'c4', d.get('c4', {}).get('steps_per_s'), 'c4 roll', d.get('c4', {}).get('rollout_kernel_avg_ms'), 'c5', d.get('c5', {}).get('steps_per_s'), 'c5 roll', d.get('c5', {}).get('rollout_kernel_avg_ms'), 'shard', d.get('c4_shard', {}).get('sharded_ms_per_step'), d.get('c4_shard', {}).get('plain_ms_per_step'))"
done; done
