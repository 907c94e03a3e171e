#!/bin/bash
# Round-5 GPU step runner (on the box): runs the named steps in order, each under its own time limit;
# stops at the first failure.  Usage: bash profiles/gpu_steps.sh <tag> step [step ...]
#   smoke                      __graft_entry__.smoke()
#   tests=<paths|all>          pytest -m gpu over the paths (comma-separated) or the whole suite
#   ab=<rounds>,<steps>,<lib>[,<lib>...]   alternating C3 bench lines per library ("-" = in-tree)
#   bench=<args>               bench.py with these args (comma-separated), line -> b_<tag>.json
#   wcal                       rocprofv3 WRITE_SIZE pass over profiles/ubench/wcal (abx/wcal)
#   diag                       MPPI_HOST_TRACE=1 profiles/ubench/server_diag.py
#   prof=<args>                rocprofv3 --kernel-trace --stats of bench.py <args> -> prof_<tag>/
#   pmc=<git head>             profiles/pmc.sh (the PMC passes) -> pmc_<tag>/, summary stamped with the commit
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out
cd $R
n=0
for st in "$@"; do
  n=$((n+1))
  name=${st%%=*}; arg=${st#*=}
  echo "== $n $name $(date +%T)"
  case $name in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.txt 2>&1 || { tail -20 $O/smoke_$TAG.txt; exit 1; }
      tail -1 $O/smoke_$TAG.txt ;;
    tests)
      sel=${arg//,/ }; [ "$sel" = "all" ] && sel=tests
      timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_$TAG.txt 2>&1
      rc=$?; echo "pytest exit=$rc" >> $O/pt_$TAG.txt; tail -3 $O/pt_$TAG.txt
      [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/pt_$TAG.txt | head -30; exit 1; } ;;
    ab)
      IFS=, read -r rounds steps libs <<< "$arg"
      BA="--warmup 5 --cpu-baseline-seconds 0 --no-bilinear --no-costmap --no-c5 --no-c4 --no-shard --no-cadence"
      for r in $(seq 1 $rounds); do
        for lib in ${libs//,/ }; do
          if [ "$lib" = "-" ]; then unset MPPI_LIB_PATH; else export MPPI_LIB_PATH=$R/$lib; fi
          timeout -k 10 300 python bench.py --steps $steps $BA > $O/ab_$TAG.json 2>$O/ab_$TAG.err || { tail -5 $O/ab_$TAG.err; exit 1; }
          python3 -c "import json; d=json.load(open('$O/ab_$TAG.json')); c=d['config']; ch=c['chain']; print('$lib', 'value', d['value'], 'sync', c['sync_steps_per_s'], 'roll', d['roofline']['kernel_avg_ms'], 'leaf', ch['wg0_leaf_us'], 'cyc', ch['cycles_per_step'], 'srv_roll', c.get('server_rollout_us'), 'srv_step', c.get('server_step_us'), 'spread', ch['wg_end_spread_us'], 'tail', c.get('tail_kernel_avg_ms'), 'fin', c.get('finish_kernel_avg_ms'))"
        done
      done
      unset MPPI_LIB_PATH ;;
    bench)
      timeout -k 10 600 python bench.py ${arg//,/ } > $O/b_$TAG.json 2>$O/b_$TAG.err || { tail -20 $O/b_$TAG.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b_$TAG.json')); c=d['config']; print('value', d['value'], 'sync', c.get('sync_steps_per_s'), 'roll', d['roofline']['kernel_avg_ms'], 'frac', d['roofline']['frac'], 'c4', d.get('c4', {}).get('steps_per_s'), 'shard', (d.get('c4_shard') or {}).get('sharded_ms_per_step'))"
      python3 -c "import json; d=json.load(open('$O/b_$TAG.json')); [print(r) for r in (d.get('cadence') or {}).get('rows', [])]" ;;
    wcal)
      cd /tmp && export TMPDIR=/tmp
      timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/wcal_$TAG -o w --output-format csv -- $R/abx/wcal > $O/wcal_$TAG.txt 2>&1 || { tail -5 $O/wcal_$TAG.txt; exit 1; }
      cd $R; find $O/wcal_$TAG -name "*counter_collection*" | head -1 | xargs -I{} python3 -c "
import csv,collections,sys
d=collections.defaultdict(list)
for r in csv.DictReader(open('{}')): d[r['Kernel_Name']].append(float(r['Counter_Value']))
for k,v in d.items(): print(k[:40], 'WRITE_SIZE per launch (KB):', [round(x) for x in v])" ;;
    diag)
      MPPI_HOST_TRACE=1 timeout -k 10 300 python profiles/ubench/server_diag.py > $O/diag_$TAG.txt 2>&1 || { tail -20 $O/diag_$TAG.txt; exit 1; }
      grep -E "back-to-back|async_tail|relaunch|server launches" $O/diag_$TAG.txt | head -20 ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o k --output-format csv -- python3 $R/bench.py ${arg//,/ } > $O/bp_$TAG.json 2> $O/bp_$TAG.err || { tail -20 $O/bp_$TAG.err; exit 1; }
      cd $R ;;
    pmc)
      GIT_HEAD=$arg bash profiles/pmc.sh $TAG > $O/pmc_$TAG.log 2>&1 || { tail -5 $O/pmc_$TAG.log; cat $O/pmc_$TAG/status.txt; exit 1; }
      tail -3 $O/pmc_$TAG.log ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
