#!/bin/bash
# Round 4 GPU session M: FF3 + BiasNorm pass 2 through the transposer with its constants from LDS
# (tools/lab/ffn_lab_tn: -DFFN_EPI_TN=1) vs per lane (default), lab + phase timing.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_m}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab ffn_lab_tn; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 8 "78016x1536;26005x1536;13002x1536" 0 "classic,pers,seg3" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
for v in t t_tn; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 8 "78016x1536" 0 "pers" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
