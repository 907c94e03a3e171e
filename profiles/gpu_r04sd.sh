#!/bin/bash
# server timeline (ubench/server_diag.py) for library builds, alternating
# Usage (on the box): bash profiles/gpu_r04sd.sh <tag> <rounds> lib1 [lib2 ...]   ("-" = the in-tree library)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; RN=$2; shift 2
O=$R/gpurun_out
cd $R
for r in $(seq 1 $RN); do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset MPPI_LIB_PATH; else export MPPI_LIB_PATH=$R/$lib; fi
    n=$(basename $lib .so)
    timeout -k 10 240 python profiles/ubench/server_diag.py > $O/sd_${TAG}_${n}_$r.txt 2>&1 || { tail -5 $O/sd_${TAG}_${n}_$r.txt; exit 1; }
    echo "== $lib round $r"; grep -E "back-to-back" $O/sd_${TAG}_${n}_$r.txt
  done
done
