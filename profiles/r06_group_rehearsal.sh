#!/bin/bash
# Round 6: bench.py's in-process C-ABI group path on the one-GPU box (members share device 0).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u bench.py --group-devices 0,0 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $O/grp2_r06.json 2> $O/grp2_r06.err
rc=$?; echo "rc2=$rc"; tail -5 $O/grp2_r06.err
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --group-devices 0,0,0,0,0,0,0,0 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $O/grp8_r06.json 2> $O/grp8_r06.err
rc=$?; echo "rc8=$rc"; tail -5 $O/grp8_r06.err
exit $rc
