#!/bin/bash
# Round 6: the server soak under both policies, then the driver's torchrun launch rehearsed (gloo, 2 ranks on one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
SOAK_RESIDENT=2 timeout -k 10 300 python profiles/ubench/soak.py 20000 > $O/soak_r06_2.txt 2>&1 || { tail -20 $O/soak_r06_2.txt; exit 1; }
tail -4 $O/soak_r06_2.txt
SOAK_RESIDENT=1 timeout -k 10 300 python profiles/ubench/soak.py 20000 > $O/soak_r06_1.txt 2>&1 || { tail -20 $O/soak_r06_1.txt; exit 1; }
tail -4 $O/soak_r06_1.txt
bash profiles/gpu_torchrun_rehearsal.sh r06 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/tr_r06.json')); c=d['config']; print('torchrun gloo', d['value'], d['n_gpus'], c['launcher'], c['parallelism'], c['speedup_vs_1'], d.get('c4',{}).get('speedup_vs_1'))"
