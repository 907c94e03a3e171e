#!/bin/bash
# A/B of finish phase stamps: libs x schedules. Usage (box): bash profiles/ubench/fin_ab.sh lib1.so lib2.so ...
set -o pipefail
for lib in "$@"; do
  for env in "MPPI_FUSED=1 MPPI_FUSED_NOISE_GROUPS=-1" "MPPI_FUSED=0" "MPPI_FUSED=0 MPPI_NOISE_AT=0"; do
    echo "== $lib $env"
    env $env timeout -k 10 90 python profiles/ubench/stamps_fin.py $lib 65536 100 1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
