#!/bin/bash
# round 2 (final tree): SQ counters of the depthwise conv, SelfAttention, NonlinAttention and the
# residual GEMM over one guided forward (one decoder stream) - issue / stall breakdown
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sq
mkdir -p $O
RX='zv_dwconv_win|zv_attn_sa_tp|zv_attn_na|zv_biasnorm'
ZV_SPLIT_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -f csv --kernel-include-regex "$RX" -d $O/p1 -o run -- python3 tools/profile_forward.py --iters 1 > $O/p1.log 2>&1 || { echo "p1 rc=$?"; exit 1; }
ZV_SPLIT_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -f csv --kernel-include-regex "$RX" -d $O/p2 -o run -- python3 tools/profile_forward.py --iters 1 > $O/p2.log 2>&1 || { echo "p2 rc=$?"; exit 1; }
python3 tools/sq_summary.py $(ls $O/p1/*counter_collection.csv | head -1) > $O/sq.txt && python3 tools/sq_summary.py $(ls $O/p2/*counter_collection.csv | head -1) >> $O/sq.txt || { echo "summary rc=$?"; exit 1; }
echo done
