#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
bash profiles/gpu_ablib.sh abl/lib_base.so abl/lib_sp1.so || exit 1
bash profiles/gpu_ab_gate.sh
