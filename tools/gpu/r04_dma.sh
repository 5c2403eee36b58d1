#!/bin/bash
# Fused FF weight-DMA issue slots on the persistent schedule: lab timing (classic / pers / noEpi) and
# one SQ pass (parked / issue-stalled / MFMA busy) of the no-epilogue arm per build:
# d = 1/17/33/49 (default), e = 1/3/5/7, f = 1/5/9/13, m = 1/9/17/25.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_dma}; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
for r in 1 2; do
  for v in d e f m; do
    b=tools/lab/ffn_lab; [ $v != d ] && b=tools/lab/ffn_lab_$v
    echo "== $v round $r" >> $O/lab.txt
    timeout -k 10 120 $b 3 1,8 "78016x1536;26005x1536" 0 "classic,pers,noEpi" >> $O/lab.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/lab.txt; exit 1; }
  done
done
cat $O/lab.txt
for v in d e f m; do
  b=tools/lab/ffn_lab; [ $v != d ] && b=tools/lab/ffn_lab_$v
  timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-include-regex zv_ffn_kernel -f csv -d $O/sq_$v -o run -- $b 3 1 "78016x1536" 0 noEpi > $O/sq_$v.log 2>&1 || { echo "sq $v failed"; tail -5 $O/sq_$v.log; exit 1; }
  f=$(ls $O/sq_$v/*counter_collection.csv | head -1)
  echo "== $v"; python3 tools/sq_summary.py "$f" zv_ffn_kernel | tee $O/sq_$v.txt
done
