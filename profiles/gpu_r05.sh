#!/bin/bash
# Round-5 GPU runner (on the box).  Usage: bash profiles/gpu_r05.sh <tag> [pytest selection] [bench args]
#   selection "all" = the whole -m gpu suite, "none" = skip the tests; bench args "none" = no bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05}
SEL=${2:-all}
BARGS=${3:---steps 20 --warmup 5}
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.txt 2>&1 || { tail -20 $O/smoke_$TAG.txt; exit 1; }
tail -1 $O/smoke_$TAG.txt
if [ "$SEL" != "none" ]; then
  [ "$SEL" = "all" ] && SEL=tests
  timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1
  rc=$?
  echo "pytest exit=$rc" >> $O/pt_$TAG.txt
  tail -3 $O/pt_$TAG.txt
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pt_$TAG.txt | head -30; exit 1; }
fi
if [ "$BARGS" != "none" ]; then
  timeout -k 10 400 python bench.py $BARGS > $O/b_$TAG.json 2>$O/b_$TAG.err || { tail -20 $O/b_$TAG.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$TAG.json')); c=d['config']; print('value', d['value'], 'sync', c.get('sync_steps_per_s'), 'roll', d['roofline']['kernel_avg_ms'], 'frac', d['roofline']['frac'], 'c4', d.get('c4', {}).get('steps_per_s'), 'shard', d.get('c4_shard'), 'cadence', d.get('cadence'))"
fi
