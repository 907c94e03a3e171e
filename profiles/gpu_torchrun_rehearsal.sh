#!/bin/bash
# The driver's multi-GPU launch (torch.distributed.run, one process per rank) rehearsed on a
# one-GPU box: N ranks (default 2) share device 0 and exchange records over gloo (RCCL refuses two
# ranks on one GPU).  Usage (on the box): bash profiles/gpu_torchrun_rehearsal.sh <tag> [N]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-tr}
N=${2:-2}
O=$R/gpurun_out
cd $R
MPPI_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --steps 20 --warmup 5 > $O/tr_$TAG.json 2> $O/tr_$TAG.err \
    || { tail -30 $O/tr_$TAG.err; exit 1; }
cat $O/tr_$TAG.json
