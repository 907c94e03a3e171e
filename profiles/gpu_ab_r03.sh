#!/bin/bash
# Round-3 A/B: costmap builder GPU tests (parallel chamfer, OpenCV float32 normalise) + its timing,
# then the C3 bench under the fused-launch variants (two alternating rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_costmap.py tests/test_gpu_engine_variants.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pt_ab.txt 2>&1 || { tail -30 $O/pt_ab.txt; exit 1; }
tail -2 $O/pt_ab.txt
timeout -k 10 120 python -c "
import sys; sys.path[:0]=['.', 'husky-rover-mppi-isaacsim_amd']
import bench, json
print(json.dumps(bench.costmap_bench(0, cpu=False)))
" || exit 1
bash profiles/ab_env2.sh "MPPI_X=0" "MPPI_FUSED=2" "MPPI_FUSED=2 MPPI_FUSED_NOISE_GROUPS=-1" || exit 1
