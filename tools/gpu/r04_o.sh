#!/bin/bash
# Round 4 GPU session O: FF3 + BiasNorm epilogue prefetch depth with its constants in LDS
# (tools/lab/ffn_lab_pdn{6,12,16}: -DFFN_PD_NORM=...; default 8).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_o}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab ffn_lab_pdn6 ffn_lab_pdn12 ffn_lab_pdn16; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 8 "78016x1536;26005x1536;13002x1536" 0 "classic,pers" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
