#!/bin/bash
# The driver's default bench line, N times back to back on one box (the spread of the 20-step number).
# Usage (GPU box): bash profiles/bench_repeat.sh <tag> <N>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
for i in $(seq 1 ${2:-5}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/rep_$1_$i.json 2> $O/rep_$1_$i.err || { tail -5 $O/rep_$1_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/rep_$1_$i.json')); c=d['config']; print('run $i', 'value', d['value'], 'sync', c['sync_steps_per_s'], 'roll_ms', d['roofline']['kernel_avg_ms'], 'frac', d['roofline']['frac'], 'c4', d.get('c4', {}).get('steps_per_s'), 'shard_ms', (d.get('c4_shard') or {}).get('sharded_ms_per_step'))"
done
