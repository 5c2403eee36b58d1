#!/bin/bash
# Fused FeedForward + pipelined depthwise conv: lab, the new GPU tests, parity/fullsize with
# ZV_FFN=2, C2 bench A/B over ZV_FFN (0 / 1 / 2) and ZV_DWCONV_PIPE.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ffnab; mkdir -p $O
timeout -k 10 150 tools/lab/ffn_lab 3 1,2 > $O/lab.txt 2>&1 || { echo "lab rc=$?"; cat $O/lab.txt; exit 1; }
cat $O/lab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest_ffn.log 2>&1 || { echo "ffn tests failed"; tail -40 $O/pytest_ffn.log; exit 1; }
grep -E 'ZV_FFN|PASS|passed|fp16' $O/pytest_ffn.log | tail -12
ZV_FFN=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/ab_env.sh ffnab ${1:-2} "ZV_FFN=0" "ZV_FFN=0 ZV_DWCONV_PIPE=1" "ZV_FFN=1 ZV_DWCONV_PIPE=1" "ZV_FFN=2 ZV_DWCONV_PIPE=1"
