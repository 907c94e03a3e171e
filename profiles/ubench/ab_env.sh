# A/B of engine environment toggles (bench.py, no CPU baseline / bilinear leg).
run() { timeout -k 10 300 env "$@" python bench.py --cpu-baseline-seconds 0 --no-bilinear > gpurun_out/b.json 2>gpurun_out/b.err || exit 1; python -c "import json; d=json.load(open('gpurun_out/b.json')); c=d['config']; print('$*', d['value'], c['sync_steps_per_s'], c['finish_kernel_avg_ms'], d['roofline']['kernel_avg_ms'])"; }
for v in "$@"; do run $v; done
