#!/bin/bash
# Round 4 GPU session F: what a coalesced FF epilogue could gain (lab ablation FFN_X_COAL: lane-
# contiguous residual loads / output stores, wrong results), and the host issue rate of one C2 step.
#   builds: tools/lab/ffn_lab{,_coal -DFFN_X_COAL=1,_t -DFFN_TIMING=1,_t_coal}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_f}; mkdir -p $O
for r in 1 2; do
  for v in ffn_lab ffn_lab_coal; do
    echo "== $v round $r" >> $O/var.txt
    timeout -k 10 120 tools/lab/$v 3 1 "78016x1536;26005x1536" 0 "classic,pers,noEpi" >> $O/var.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/var.txt; exit 1; }
  done
done
cat $O/var.txt
for v in t t_coal; do
  echo "== $v" >> $O/x.txt
  timeout -k 10 60 tools/lab/ffn_lab_$v 2 1 "78016x1536" 0 "pers" >> $O/x.txt 2>&1 || { echo "$v rc=$?"; tail -3 $O/x.txt; exit 1; }
done
cat $O/x.txt
timeout -k 10 300 python -u tools/host_rate.py --steps 5 > $O/host_rate.txt 2>&1 || { echo "host_rate failed"; tail -5 $O/host_rate.txt; exit 1; }
tail -2 $O/host_rate.txt
