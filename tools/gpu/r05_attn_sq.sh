#!/bin/bash
# Attention lab (tools/lab/attn_lab, built on the CPU side): per-shape timings of the fused attention
# consumers, then SQ counters (one pass each) for the three kernels at the bench's per-stream shape.
#   tools/gpu/r05_attn_sq.sh OUT [SHAPE] [ARMS]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_attn}; mkdir -p $O
SH=${2:-21x1219}
ARMS=${3:-stats,na,sa}
LAB=${LAB:-tools/lab/attn_lab}
timeout -k 10 120 $LAB 5 "" "$ARMS" > $O/lab.txt 2>&1 || { echo "lab failed"; tail -5 $O/lab.txt; exit 1; }
cat $O/lab.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM"
P3="SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "zv_attn" -f csv -d $O/p$i -o run -- $LAB 1 "$SH" "$ARMS" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  f=$(ls $O/p$i/*counter_collection.csv | head -1)
  python3 tools/sq_summary.py "$f" zv_attn | tee $O/sq$i.txt
done
