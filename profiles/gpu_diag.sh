#!/bin/bash
# Diagnostics: host-side step trace, a kernel-trace timeline of the pipelined C3 bench, and the
# group rehearsal on one GPU with enough hardware queues for 8 members x 3 streams.
# Usage (on the box): bash profiles/gpu_diag.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-diag}
O=$R/gpurun_out
MPPI_HOST_TRACE=1 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 --no-c4 --no-c5 --no-bilinear --no-costmap > $O/ht_$TAG.json 2> $O/ht_$TAG.err || { tail $O/ht_$TAG.err; exit 1; }
grep "host trace" $O/ht_$TAG.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$TAG -o t -- python3 $R/bench.py --steps 100 --warmup 10 --cpu-baseline-seconds 0 --no-c4 --no-c5 --no-bilinear --no-costmap > /dev/null 2>&1 || exit 1
cd $R
python3 profiles/trace_timeline.py $(ls $O/tr_$TAG/*kernel_trace.csv | head -1) 500 24
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py --group-devices 0,0,0,0,0,0,0,0 --steps 100 --warmup 10 --cpu-baseline-seconds 0 > $O/bgq_$TAG.json 2>$O/bgq_$TAG.err || { tail -20 $O/bgq_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bgq_$TAG.json')); c=d['config']; print('group value', d['value'], 'sync', c['sync_steps_per_s'], 'speedup', c['speedup_vs_1'], 'c4', d.get('c4'))"
