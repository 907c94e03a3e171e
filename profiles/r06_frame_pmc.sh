set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $R/gpurun_out/fpmc/p$i -o p --output-format csv -- python3 $R/profiles/ubench/frame_pmc.py > $R/gpurun_out/fpmc_$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/fpmc_$i.txt; exit 1; }
  i=$((i+1))
done
echo ok
