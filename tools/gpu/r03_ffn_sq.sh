#!/bin/bash
# SQ counters of the fused FeedForward kernel and its ablations (ffn_lab, one shape), two passes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ffnsq; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex zv_ffn_kernel -f csv -d $O/p$i -o run -- tools/lab/ffn_lab 1 1 "78016x1536" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  f=$(ls $O/p$i/*counter_collection.csv | head -1)
  python3 tools/sq_summary.py "$f" zv_ffn_kernel | tee $O/sq$i.txt
done
