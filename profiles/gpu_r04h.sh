#!/bin/bash
# round 4: resident server with deferred tails (diag timeline, variant tests, 20/200-step benches
# against separate launches), then the chain-alone diagnostic builds (ab/side1.so: wheel and cost
# roles idle; ab/side2.so: also a constant producer)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04h}
O=$R/gpurun_out
cd $R
bash profiles/gpu_r04g.sh $TAG || exit 1
for lib in abx/side1.so abx/side2.so; do
  MPPI_LIB_PATH=$R/$lib MPPI_RESIDENT=0 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard --no-sync-pass > $O/side.json 2>$O/side.err || { tail -5 $O/side.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/side.json')); print('[$lib] chain', d['config'].get('chain'), 'roll', d['roofline']['kernel_avg_ms'])"
done
MPPI_RESIDENT=0 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard --no-sync-pass > $O/side.json 2>$O/side.err || { tail -5 $O/side.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/side.json')); print('[product] chain', d['config'].get('chain'), 'roll', d['roofline']['kernel_avg_ms'])"
for i in 1 2; do for lib in abx/d4.so libmppi; do
  if [ $lib = libmppi ]; then unset MPPI_LIB_PATH; else export MPPI_LIB_PATH=$R/$lib; fi
  MPPI_RESIDENT=0 timeout -k 10 200 python bench.py --steps 200 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard --no-sync-pass > $O/d4.json 2>$O/d4.err || { tail -5 $O/d4.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/d4.json')); c=d['config']; print('[$lib] value', d['value'], 'chain', c.get('chain'), 'roll', d['roofline']['kernel_avg_ms'], 'ucache', (c.get('rollout_kernel') or {}).get('ucache_steps'))"
done; done
unset MPPI_LIB_PATH
