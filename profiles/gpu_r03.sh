#!/bin/bash
# Round-3 GPU check: the full -m gpu suite, a C3 bench line without side legs, and the in-process
# group path rehearsed on one GPU (8 members sharing device 0, device-copy exchange).
# Usage (on the box): bash profiles/gpu_r03.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1
rc=$?
echo "pytest exit=$rc" >> $O/pt_$TAG.txt
tail -3 $O/pt_$TAG.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pt_$TAG.txt | head -30; exit 1; }
timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 > $O/b_$TAG.json 2>$O/b_$TAG.err || { tail -20 $O/b_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$TAG.json')); c=d['config']; print('value', d['value'], 'sync', c['sync_steps_per_s'], 'fin', c['finish_kernel_avg_ms'], 'tail', c['tail_kernel_avg_ms'], 'roll', d['roofline']['kernel_avg_ms'], 'c4', d.get('c4', {}).get('steps_per_s'))"
timeout -k 10 300 python bench.py --group-devices 0,0,0,0,0,0,0,0 --steps 100 --warmup 10 --cpu-baseline-seconds 0 > $O/bg_$TAG.json 2>$O/bg_$TAG.err || { tail -20 $O/bg_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bg_$TAG.json')); c=d['config']; print('group value', d['value'], 'n_gpus', d['n_gpus'], 'sync', c['sync_steps_per_s'], 'speedup', c['speedup_vs_1'], 'group', c['group'], 'c4', d.get('c4'))"
