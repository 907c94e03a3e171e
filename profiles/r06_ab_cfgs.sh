#!/bin/bash
# Round 6: alternating bench lines of other configs (C4, the C4 shard, C5) for the in-tree library
# and the libraries named (abx/...).  Usage (GPU box): bash profiles/r06_ab_cfgs.sh <rounds> <lib> [<lib>...]
set -o pipefail
cd $GRAFT_REPO_ROOT
rounds=$1; shift
A="--steps,20,--warmup,5,--cpu-baseline-seconds,0,--no-bilinear,--no-costmap,--no-c5,--no-shard,--no-cadence,--no-sync-pass,--no-c4"
for r in $(seq 1 $rounds); do
  for lib in - "$@"; do
    for cfg in c4 c4s8 c5; do
      if [ "$lib" = "-" ]; then unset MPPI_LIB_PATH; else export MPPI_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
      echo "lib=$lib cfg=$cfg"
      bash profiles/gpu_steps.sh abc_${cfg} bench=--config,$cfg,$A | grep value || exit 1
    done
  done
done
