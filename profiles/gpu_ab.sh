set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pt_a.log 2>&1; echo "pytest rc=$?" >> $OUT/pt_a.log; tail -3 $OUT/pt_a.log
grep -q "rc=0" $OUT/pt_a.log || exit 1
timeout -k 10 200 python bench.py --steps 400 --warmup 20 --cpu-baseline-seconds 0 > $OUT/b0.json 2>$OUT/b0.err && cut -c1-200 $OUT/b0.json
MPPI_NOISE_AT=1 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --cpu-baseline-seconds 0 > $OUT/b1.json 2>$OUT/b1.err && cut -c1-200 $OUT/b1.json
