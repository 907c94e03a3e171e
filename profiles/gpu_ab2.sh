#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
ROUNDS="1 2 3" bash profiles/ab_env2.sh "MPPI_X=0" "MPPI_FUSED=1" || exit 1
timeout -k 10 120 python profiles/ubench/stamps_fin.py abl/stamps.so 65536 100 1 || exit 1
MPPI_FUSED=1 timeout -k 10 120 python profiles/ubench/stamps_fin.py abl/stamps.so 65536 100 1
