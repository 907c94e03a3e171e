set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u profiles/ubench/frame_oneshot.py 2 > gpurun_out/frame_oneshot.txt 2>&1 || { tail -20 gpurun_out/frame_oneshot.txt; exit 1; }
grep -E "round|bitwise" gpurun_out/frame_oneshot.txt
