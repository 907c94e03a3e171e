#!/bin/bash
# Armed-step check: its tests first, then the full GPU suite and a C3 bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_arm.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pt_arm.txt 2>&1
rc=$?; tail -12 $O/pt_arm.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_all.txt 2>&1
rc=$?; tail -3 $O/pt_all.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pt_all.txt | head; exit 1; }
for a in 1 0 1 0; do
  MPPI_ARM=$a timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 > $O/b_arm$a.json 2>$O/b_arm$a.err || { tail -5 $O/b_arm$a.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_arm$a.json')); c=d['config']; print('arm $a', round(d['value']), 'sync', round(c['sync_steps_per_s']), 'roll', d['roofline']['kernel_avg_ms'], 'c4', d.get('c4',{}).get('steps_per_s'))"
done
