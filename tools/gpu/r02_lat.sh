#!/bin/bash
# round 2: single-sentence latency with the CFG pair split over two streams (ZV_SPLIT_MIN_ROWS=1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lat
mkdir -p $O
timeout -k 10 200 python -u tools/latency_c1.py bf16 > $O/base.txt 2>&1 || { echo "base rc=$?"; exit 1; }
ZV_SPLIT_MIN_ROWS=1 timeout -k 10 200 python -u tools/latency_c1.py bf16 > $O/split.txt 2>&1 || { echo "split rc=$?"; exit 1; }
timeout -k 10 200 python -u tools/latency_c1.py bf16 > $O/base2.txt 2>&1 || { echo "base2 rc=$?"; exit 1; }
echo done
