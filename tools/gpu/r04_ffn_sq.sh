#!/bin/bash
# SQ / GRBM counters of the persistent fused FeedForward (ffn_lab, M=78016 H=1536, mode 1) for the
# timed arm (pers) and the no-epilogue ablation, one counter pass per run.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_sq}; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
P3="SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for arm in pers noEpi; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex zv_ffn_kernel -f csv -d $O/${arm}_p$i -o run -- tools/lab/ffn_lab 3 1 "78016x1536" 0 $arm > $O/${arm}_p$i.log 2>&1 || { echo "pass $arm $i failed"; tail -5 $O/${arm}_p$i.log; exit 1; }
    f=$(ls $O/${arm}_p$i/*counter_collection.csv | head -1)
    python3 tools/sq_summary.py "$f" zv_ffn_kernel | tee $O/${arm}_sq$i.txt
  done
done
timeout -k 10 120 tools/lab/ffn_lab 3 1 "78016x1536" 0 "classic,pers,noEpi" > $O/lab.txt 2>&1; cat $O/lab.txt
