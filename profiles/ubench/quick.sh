# GPU parity tests + bench (no CPU baseline / bilinear) + a traced async window (diagnostic).
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pt.txt 2>&1 || { tail -30 $R/gpurun_out/pt.txt; exit 1; }
tail -1 $R/gpurun_out/pt.txt
timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --no-bilinear > $R/gpurun_out/b.json 2>$R/gpurun_out/b.err || exit 1
python3 -c "import json; d=json.load(open('$R/gpurun_out/b.json')); c=d['config']; print('value', d['value'], 'sync', c['sync_steps_per_s'], 'fin', c['finish_kernel_avg_ms'], 'tail', c['tail_kernel_avg_ms'], 'roll', d['roofline']['kernel_avg_ms'])"
if [ -n "$TRACE" ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/qtr -o tr --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear > /dev/null 2>&1) || exit 1
  python3 $R/profiles/trace_timeline.py $(ls $R/gpurun_out/qtr/*kernel_trace.csv | head -1) 200 16
fi
