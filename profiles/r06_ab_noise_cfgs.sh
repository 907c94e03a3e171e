set -o pipefail
cd $GRAFT_REPO_ROOT
A="--steps,20,--warmup,5,--cpu-baseline-seconds,0,--no-bilinear,--no-costmap,--no-c5,--no-shard,--no-cadence,--no-sync-pass,--no-c4"
for r in 1 2; do
  for lib in - abx/libmppi_noise0.so; do
    for cfg in c4 c4s8 c5; do
      if [ "$lib" = "-" ]; then unset MPPI_LIB_PATH; else export MPPI_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
      echo "lib=$lib cfg=$cfg"
      bash profiles/gpu_steps.sh abc_${cfg} bench=--config,$cfg,$A | grep value || exit 1
    done
  done
done
