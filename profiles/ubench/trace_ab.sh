# Kernel timelines of bench.py under engine environment toggles (diagnostic).
# Usage (GPU box): bash profiles/ubench/trace_ab.sh "ENV=.." "ENV=.." ...
R=$GRAFT_REPO_ROOT
i=0
for v in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 env MPPI_HOST_TRACE=1 $v rocprofv3 --kernel-trace -d $R/gpurun_out/tab$i -o tr --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-bilinear > $R/gpurun_out/tab$i.json 2> $R/gpurun_out/tab$i.err) || exit 1
  echo "=== $v"; grep "host trace" $R/gpurun_out/tab$i.err
  python3 $R/profiles/trace_timeline.py $(ls $R/gpurun_out/tab$i/*kernel_trace.csv | head -1) 150 14
done
