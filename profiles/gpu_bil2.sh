#!/bin/bash
# Bilinear leg under a kernel trace (binning kernels vs the tiled lookup).  Usage: bash profiles/gpu_bil2.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-bil}
O=$R/gpurun_out
cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_bilinear.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1 || { tail -30 $O/pt_$TAG.txt; exit 1; }
tail -1 $O/pt_$TAG.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o k --output-format csv -- \
    python3 -c "import sys, json, torch; sys.path[:0]=['$R', '$R/husky-rover-mppi-isaacsim_amd']; import bench; print(json.dumps(bench.bilinear_bench(torch, torch.device('cuda', 0))))" > $O/bil_$TAG.json 2> $O/prof_$TAG.err || { tail -5 $O/prof_$TAG.err; exit 1; }
cat $O/bil_$TAG.json
python3 -c "
import csv
rows = list(csv.DictReader(open('$O/prof_$TAG/k_kernel_stats.csv')))
for r in rows: print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
