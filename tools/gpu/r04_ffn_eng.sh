#!/bin/bash
# Round 4: persistent + joined fused FeedForward in the engine: lab (bit-for-bit + timing), the FF /
# split-stream GPU tests, then the C2 bench A/B (default = joined + persistent; not joined; neither).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_eng}; mkdir -p $O
timeout -k 10 240 tools/lab/ffn_lab 3 1,2,4,8 "78016x1152;78016x1536;78016x1920;39008x1536" > $O/lab_new.txt 2>&1; rc=$?
cat $O/lab_new.txt; [ $rc = 0 ] || { echo "new lab rc=$rc"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_split_streams.py tests/test_gpu_ffn.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest.log | tail -20
bash tools/gpu/ab_env.sh ${1:-r04_eng}/ab ${2:-2} "-" "ZV_FFN_JOIN=0" "ZV_FFN_JOIN=0 ZV_FFN_PERSIST=0"
