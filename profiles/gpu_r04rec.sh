#!/bin/bash
# Round-4 record at one source hash: smoke, the full -m gpu suite, the default bench line (as the
# driver runs it), the rocprofv3 kernel stats of the same bench, and the PMC passes.
# Usage (on the box): bash profiles/gpu_r03h.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04rec}
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.txt 2>&1 || { tail -20 $O/smoke_$TAG.txt; exit 1; }
tail -1 $O/smoke_$TAG.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1
rc=$?
echo "pytest exit=$rc" >> $O/pt_$TAG.txt
tail -3 $O/pt_$TAG.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pt_$TAG.txt | head -30; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_$TAG.json 2>$O/b_$TAG.err || { tail -20 $O/b_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$TAG.json')); c=d['config']; print('value', d['value'], 'sync', c['sync_steps_per_s'], 'fin', c['finish_kernel_avg_ms'], 'tail', c['tail_kernel_avg_ms'], 'roll', d['roofline']['kernel_avg_ms'], 'frac', d['roofline']['frac'], 'c4', d.get('c4', {}).get('steps_per_s'), 'shard', d.get('c4_shard'), 'sched', c.get('schedule'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o k --output-format csv -- \
    python3 $R/bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c4 --no-c5 > $O/bp_$TAG.json 2> $O/bp_$TAG.err || { tail -20 $O/bp_$TAG.err; exit 1; }
cd $R
bash profiles/pmc.sh $TAG > $O/pmc_$TAG.log 2>&1 || { tail -5 $O/pmc_$TAG.log; cat $O/pmc_$TAG/status.txt; exit 1; }
tail -3 $O/pmc_$TAG.log
