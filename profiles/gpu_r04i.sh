#!/bin/bash
# round 4: packed Box-Muller noise (full -m gpu suite), server vs separate launches (alternating),
# chain-alone diagnostics (abx/side1.so, abx/side2.so) and ring depth 4 (abx/d4.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04i}
O=$R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$TAG.txt 2>&1
rc=$?; tail -4 $O/pytest_$TAG.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/pytest_$TAG.txt | head -20; exit 1; }
BA="--warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard"
for i in 1 2; do for env in "MPPI_RESIDENT=1" "MPPI_RESIDENT=0"; do for st in 20 200; do
  env $env timeout -k 10 300 python bench.py --steps $st $BA > $O/b2.json 2>$O/b2.err || { tail -5 $O/b2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b2.json')); c=d['config']; print('[$env] $st/5 value', d['value'], 'sync', c['sync_steps_per_s'], 'roll', d['roofline']['kernel_avg_ms'])"
done; done; done
for lib in abx/side1.so abx/side2.so abx/d4.so; do
  MPPI_LIB_PATH=$R/$lib MPPI_RESIDENT=0 timeout -k 10 200 python bench.py --steps 200 $BA --no-sync-pass > $O/side.json 2>$O/side.err || { tail -5 $O/side.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/side.json')); c=d['config']; print('[$lib] value', d['value'], 'chain', c.get('chain'), 'roll', d['roofline']['kernel_avg_ms'], 'ucache', (c.get('rollout_kernel') or {}).get('ucache_steps'))"
done
