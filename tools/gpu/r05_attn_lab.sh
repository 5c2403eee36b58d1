#!/bin/bash
# Attention lab (tools/lab/attn_lab built with -DATTN_LAB_V2 on the CPU side): first vs second
# generation consumers per shape, then one SQ counter pass per kernel family at the per-stream shape.
#   tools/gpu/r05_attn_lab.sh OUT [SHAPE] [ARMS] [COUNTER_ARMS]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_attn}; mkdir -p $O
SH=${2:-21x1219}
ARMS=${3:-stats,na,sa,sa2,sa2q1,na2,exact}
CARMS=${4:-stats,na,sa,sa2,na2}
LAB=${LAB:-tools/lab/attn_lab}
timeout -k 10 180 $LAB 5 "" "$ARMS" > $O/lab.txt 2>&1 || { echo "lab failed"; cat $O/lab.txt | tail -20; exit 1; }
cat $O/lab.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "zv_attn" -f csv -d $O/p$i -o run -- $LAB 1 "$SH" "$CARMS" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  f=$(ls $O/p$i/*counter_collection.csv | head -1)
  python3 tools/sq_summary.py "$f" zv_attn | tee $O/sq$i.txt
done
