#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04c}
O=$R/gpurun_out
cd $R
timeout -k 10 120 ./profiles/ubench/server_bin 70 1000 > $O/server_$TAG.txt 2>&1; echo "server ubench rc=$?"; cat $O/server_$TAG.txt
MPPI_HOST_TRACE=1 timeout -k 10 120 python -u profiles/ubench/server_diag.py 100 > $O/diag_$TAG.txt 2>&1; echo "diag rc=$?"; cat $O/diag_$TAG.txt
MPPI_RESIDENT=0 MPPI_HOST_TRACE=1 timeout -k 10 120 python -u profiles/ubench/server_diag.py 100 > $O/diag0_$TAG.txt 2>&1; echo "diag0 rc=$?"; cat $O/diag0_$TAG.txt
