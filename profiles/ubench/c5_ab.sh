for v in "$@"; do
  timeout -k 10 300 env $v python bench.py --cpu-baseline-seconds 0 --no-bilinear --no-costmap --steps 100 > gpurun_out/c5b.json 2>gpurun_out/c5b.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c5b.json')); print('$v', d['value'], d['c5'])"
done
