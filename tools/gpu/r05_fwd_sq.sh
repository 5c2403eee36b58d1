#!/bin/bash
# SQ counters of the engine's kernels matching a regex over one guided forward (tools/profile_forward.py),
# one rocprofv3 --pmc pass per counter group.   tools/gpu/r05_fwd_sq.sh OUT REGEX
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_fwd_sq}; mkdir -p $O
RX=${2:-zv_dwconv}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM"
P3="SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" -f csv -d $O/p$i -o run -- python3 tools/profile_forward.py --iters 1 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  f=$(ls $O/p$i/*counter_collection.csv | head -1)
  python3 tools/sq_summary.py "$f" "$RX" | tee $O/sq$i.txt
  rm -rf $O/p$i
done
