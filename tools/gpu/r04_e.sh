#!/bin/bash
# Round 4 GPU session E: FF3 + BiasNorm epilogue with the engine's output set compiled in
# (FFN_NORM_SPEC) vs the run-time-checked one; bench A/B of the fused-FF row threshold and the
# per-stream block cap.
#   builds: tools/lab/ffn_lab{,_spec -DFFN_NORM_SPEC=1,_t -DFFN_TIMING=1,_t_spec}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_e}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab ffn_lab_spec; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 8 "78016x1536;26005x1536;13002x1536" 0 "classic,pers" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
for v in t t_spec; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 8 "78016x1536" 0 "pers" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
timeout -k 10 120 tools/lab/ffn_lab 3 1,2,8 "6501x1536;9752x1536;13002x1536" 0 "unfused,classic" > $O/small.txt 2>&1 || { echo "small rc=$?"; tail -5 $O/small.txt; exit 1; }
cat $O/small.txt
bash tools/gpu/ab_env.sh ${1:-r04_e}/ab 2 "-" "ZV_FFN_MIN_ROWS=0" "ZV_FFN_SPLIT_BLOCKS=170" "ZV_FFN_SPLIT_BLOCKS=128"
