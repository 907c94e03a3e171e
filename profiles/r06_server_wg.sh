cd $GRAFT_REPO_ROOT
O=gpurun_out/server_wg2.txt; : > $O
for seed in 42 7; do
  SEED=$seed timeout -k 10 120 python profiles/ubench/server_wg.py 200 --sync >> $O 2>&1 || exit 1
  SEED=$seed MPPI_LIB_PATH=$GRAFT_REPO_ROOT/abx/libmppi_chainend.so timeout -k 10 120 python profiles/ubench/server_wg.py 200 --sync >> $O 2>&1 || exit 1
done
grep rep $O
