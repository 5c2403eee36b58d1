#!/bin/bash
# Fused FeedForward: lab (fused vs unfused), parity with ZV_FFN=1, C2 bench A/B ZV_FFN=0/1.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ffnab; mkdir -p $O
timeout -k 10 150 tools/lab/ffn_lab 3 1,2 > $O/lab.txt 2>&1 || { echo "lab rc=$?"; cat $O/lab.txt; exit 1; }
cat $O/lab.txt
ZV_FFN=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/ab_env.sh ffnab ${1:-2} "ZV_FFN=0" "ZV_FFN=1" "ZV_FFN=2"
