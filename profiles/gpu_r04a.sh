#!/bin/bash
# Round-4 first call: the headline tests (reference-f32 update included), then a C3 bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04a}
O=$R/gpurun_out
cd $R
timeout -k 10 90 ./profiles/ubench/server_bin 70 2000 > $O/server_$TAG.txt 2>&1; echo "server rc=$?"; cat $O/server_$TAG.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1
rc=$?; tail -5 $O/pt_$TAG.txt; grep -E "reference-f32" $O/pt_$TAG.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 > $O/b_$TAG.json 2>$O/b_$TAG.err || { tail -20 $O/b_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$TAG.json')); c=d['config']; print('value', d['value'], 'sync', c['sync_steps_per_s'], 'fin', c['finish_kernel_avg_ms'], 'tail', c['tail_kernel_avg_ms'], 'roll', d['roofline']['kernel_avg_ms'], 'chain', c['chain'], 'c4', d.get('c4', {}).get('steps_per_s'))"
for env in "" "MPPI_FUSED=2 MPPI_FUSED_NOISE_GROUPS=-2"; do
  for st in 20 200; do
    env $env timeout -k 10 300 python bench.py --steps $st --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 > $O/b2.json 2>$O/b2.err || { tail -5 $O/b2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b2.json')); c=d['config']; print('[$env] steps $st value', d['value'], 'sync', c['sync_steps_per_s'])"
  done
done
