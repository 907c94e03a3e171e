set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_frame -o k --output-format csv -- python3 $R/profiles/ubench/frame_trace.py > $R/gpurun_out/frame_stamps.txt 2> $R/gpurun_out/frame_trace.err || { tail -20 $R/gpurun_out/frame_trace.err; exit 1; }
tail -2 $R/gpurun_out/frame_stamps.txt
