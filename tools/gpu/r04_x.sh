#!/bin/bash
# Chunk-step ablations of the fused FF (lab builds with FFN_TIMING): where a step's cycles go; the
# FFN_OUT_ASM / FFN_BIAS_ACC variants (tools/lab/ffn_lab_{oa,ba,oaba}); then the default build's
# bit-for-bit checks and timing over the model's shapes.
#   builds: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/ffn_lab.hip
#           [-DFFN_TIMING=1] [-DFFN_OUT_ASM=1] [-DFFN_BIAS_ACC=1] [-DFFN_X_NOACT=1 ...] -o tools/lab/ffn_lab_<v>
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04_x}; mkdir -p $O
for v in t t_oa t_oaba x_noact x_now2 x_now12 x_noact_now12; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 1 "78016x1536" 0 "pers,noDMA,noEpi" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
for r in 1 2; do
  for v in ffn_lab ffn_lab_oa ffn_lab_ba ffn_lab_oaba; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 1,8 "78016x1536;39008x1536;26005x1536" 0 "unfused,classic,pers,noEpi" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
timeout -k 10 200 tools/lab/ffn_lab 3 1,2,4,8 "78016x1152;78016x1536;78016x1920;39008x1536;26005x1536" 0 "unfused,classic,pers,seg3,noEpi" > $O/lab.txt 2>&1 || { echo "lab rc=$?"; tail -5 $O/lab.txt; exit 1; }
cat $O/lab.txt
