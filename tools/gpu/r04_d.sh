#!/bin/bash
# Round 4 GPU session D: epilogue A/B (b2 in the output tiles' initial value; prefetch depths), phase
# timing, the FF tests on the new default, bench A/B of the decoder stream split with the persistent FF.
#   builds: tools/lab/ffn_lab{,_nb2 -DFFN_B2_ACC=0,_pd20 -DFFN_PD=20 -DFFN_PD_OPRE=12 -DFFN_PD_NORM=12,
#           _pd24 -DFFN_PD=24 -DFFN_PD_OPRE=16 -DFFN_PD_NORM=16,_t -DFFN_TIMING=1,_t_pd20}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_d}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab_nb2 ffn_lab ffn_lab_pd20 ffn_lab_pd24; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 1,2,8 "78016x1536;26005x1536" 0 "classic,pers" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
for v in t t_pd20; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 1,2,8 "78016x1536" 0 "pers" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_split_streams.py -x -v -s --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -3
grep -iE "mean" $O/pytest.log | head -20
bash tools/gpu/ab_env.sh ${1:-r04_d}/ab 2 "-" "ZV_SPLIT_STREAMS=1" "ZV_SPLIT_STREAMS=2"
