#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only, no sys/runtime trace), on
# separate launches (MPPI_RESIDENT=0): counter collection serializes dispatches, and the resident
# server needs all of its workgroups on the device at once.
# Usage (on the GPU box): GIT_HEAD=<commit> bash profiles/pmc.sh <tag> [bench args...]
# K / H of the summary: PMC_K / PMC_H (default the C3 headline 65536 / 100).  Only the headline
# config's legs run (no C4 shard / cadence legs: their kernels of other sizes would be averaged in;
# round 4's "83 MB" noise-kernel write was C3 and shard launches averaged, profiles/r05_notes.md).
set -o pipefail
TAG=${1:-pmc}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  MPPI_RESIDENT=0 timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o p --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 0 --no-sync-pass --no-c4 --no-c5 --no-bilinear --no-costmap --no-shard --no-cadence "$@" > /dev/null 2> $OUT/p$i.err || { echo "pass $i ($grp) failed rc=$?" >> $OUT/status.txt; exit 1; }
  i=$((i+1))
done
cd $GRAFT_REPO_ROOT
python3 profiles/pmc_summary.py $OUT ${PMC_K:-65536} ${PMC_H:-100} > $OUT/summary.json && cat $OUT/summary.json
