set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pt_f.txt 2>&1; rc=$?
tail -2 $O/pt_f.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pt_f.txt | head -20; exit 1; }
timeout -k 5 60 python profiles/ubench/stamps_fin.py abl/stamps.so 65536 100 1 2>&1 | grep -v amdgpu.ids
