set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u profiles/ubench/eps_after_ab.py 2 > gpurun_out/eps_after_ab3.txt 2>&1 || { tail -20 gpurun_out/eps_after_ab3.txt; exit 1; }
grep -E "bitwise|round" gpurun_out/eps_after_ab3.txt
