#!/bin/bash
# One GPU round: self-tests + parity (pytest -m gpu), bench, rocprofv3 kernel trace of the C3 step
# alone (no C5 / bilinear / costmap legs, so each kernel's average is the bench line's kernel).
# Usage (on the box): bash profiles/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT/prof_$TAG
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_$TAG.log 2>&1
echo "pytest exit=$?" >> $OUT/pytest_$TAG.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-baseline-seconds ${CPU_S:-0} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o r02 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 0 --no-c4 --no-c5 --no-bilinear --no-costmap > /dev/null 2>&1
cd $GRAFT_REPO_ROOT
tail -3 $OUT/pytest_$TAG.log
cut -c1-400 $OUT/bench_$TAG.json
cat $OUT/prof_$TAG/r02_kernel_stats.csv
