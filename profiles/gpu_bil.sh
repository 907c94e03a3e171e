#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bilinear.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/pt_bil.txt 2>&1 || { tail -30 $R/gpurun_out/pt_bil.txt; exit 1; }
tail -1 $R/gpurun_out/pt_bil.txt
timeout -k 10 120 python -c "
import sys; sys.path[:0]=['.', 'husky-rover-mppi-isaacsim_amd']
import bench, json, torch
print(json.dumps(bench.bilinear_bench(torch, torch.device('cuda', 0))))
" || exit 1
bash profiles/gpu_ab_gate.sh
