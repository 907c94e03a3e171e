set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python profiles/ubench/fold_ab.py 3 200 > gpurun_out/fold_ab.txt 2>&1 || exit 1
cat gpurun_out/fold_ab.txt | grep round
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fold -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/profiles/ubench/fold_ab.py 1 100 > $GRAFT_REPO_ROOT/gpurun_out/fold_prof.txt 2>&1 || exit 1
