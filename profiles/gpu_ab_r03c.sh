#!/bin/bash
# costmap tests + timing (prefetching chamfer), then the fused-launch A/B (gpu_ab_r03b.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_costmap.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pt_cm.txt 2>&1 || { tail -30 $O/pt_cm.txt; exit 1; }
tail -1 $O/pt_cm.txt
timeout -k 10 120 python -c "
import sys; sys.path[:0]=['.', 'husky-rover-mppi-isaacsim_amd']
import bench, json
print(json.dumps(bench.costmap_bench(0, cpu=False)))
" || exit 1
bash profiles/gpu_ab_r03b.sh
