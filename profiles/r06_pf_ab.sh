set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for lib in base pf4 pf6; do
    MPPI_LIB_PATH=$GRAFT_REPO_ROOT/abx/lib_$lib.so timeout -k 10 120 python -u profiles/ubench/frame_clock.py > gpurun_out/fc_$lib.txt 2>&1 || { tail -5 gpurun_out/fc_$lib.txt; exit 1; }
    grep rep gpurun_out/fc_$lib.txt | sed "s/^/$lib r$r /"
  done
done
bash profiles/gpu_steps.sh pfab ab=2,20,abx/lib_base.so,abx/lib_pf4.so,abx/lib_pf6.so
