#!/bin/bash
# GPU round trip used while iterating: the full -m gpu suite, then a C3 bench line without the
# side legs.  Usage (on the box): bash profiles/gpu_quick.sh [tag]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/pt_$TAG.txt 2>&1 || { tail -40 $R/gpurun_out/pt_$TAG.txt; exit 1; }
tail -2 $R/gpurun_out/pt_$TAG.txt
timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 > $R/gpurun_out/b_$TAG.json 2>$R/gpurun_out/b_$TAG.err || exit 1
python3 -c "import json; d=json.load(open('$R/gpurun_out/b_$TAG.json')); c=d['config']; print('value', d['value'], 'sync', c['sync_steps_per_s'], 'fin', c['finish_kernel_avg_ms'], 'tail', c['tail_kernel_avg_ms'], 'roll', d['roofline']['kernel_avg_ms'], 'c4', d.get('c4', {}).get('steps_per_s'))"
