#!/bin/bash
# Round 4: persistent fused FeedForward (zv_ffn.inc line schedule) in the lab: new kernel (classic /
# persistent / three ranges / no epilogue, bit-for-bit checks) and the round-3 kernel (FFN_TAIL 0
# and 1 builds: tools/lab/ffn_lab_old0 / ffn_lab_old) on the same box.  A one-shape probe first.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04_lab}; mkdir -p $O
timeout -k 10 60 tools/lab/ffn_lab 1 1 "26005x1536" > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt; [ $rc = 0 ] || { echo "probe rc=$rc"; exit 1; }
timeout -k 10 240 tools/lab/ffn_lab ${2:-3} ${3:-1,2,4,8} > $O/lab_new.txt 2>&1; rc=$?
cat $O/lab_new.txt; [ $rc = 0 ] || { echo "new lab rc=$rc"; exit 1; }
for v in ffn_lab_old0 ffn_lab_old; do
  timeout -k 10 150 tools/lab/$v 3 1 "78016x1152;78016x1536;78016x1920;39008x1536;19504x1536;26005x1536" > $O/$v.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.txt; exit 1; }
  echo "== $v"; cat $O/$v.txt
done
