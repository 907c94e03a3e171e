set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for args in "--no-c5" "--no-c4 --no-c5 --no-bilinear --no-costmap" "--no-bilinear --no-costmap"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 $args > $O/sx.json 2>$O/sx.err || { tail -5 $O/sx.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sx.json')); s=d.get('c4_shard',{}); print('$args', d['value'], s.get('sharded_ms_per_step'), s.get('plain_ms_per_step'))"
done
