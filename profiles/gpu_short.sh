#!/bin/bash
# The driver's bench invocation (--steps 20 --warmup 5) three times, then the 200-step line; chain clock.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 > $O/s$k.json 2>$O/s$k.err || { tail -5 $O/s$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/s$k.json')); c=d['config']; print('20/5', round(d['value']), 'sync', round(c['sync_steps_per_s']), 'roll', d['roofline']['kernel_avg_ms'], 'chain', c['chain'])"
done
timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 > $O/s200.json 2>$O/s200.err || { tail -5 $O/s200.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/s200.json')); c=d['config']; print('200/20', round(d['value']), 'sync', round(c['sync_steps_per_s']), 'roll', d['roofline']['kernel_avg_ms'], 'chain', c['chain'])"
