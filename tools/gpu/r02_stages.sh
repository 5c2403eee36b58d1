#!/bin/bash
# round 2: ring depth A/B with the fragment preload (0 = BK64 2-stage, 1 = BK64 3-stage,
# 30 = BK32 4-stage, 31 = BK32 3-stage) on the model's shapes; then the GPU suite on the
# pruned tree
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u tools/bench_gemm.py 0,1,30,31 4,1,2 "78016x512x1536;78016x1024x512;78016x1536x512;78016x512x512" > $O/r02_stages.log 2>&1 || { echo "gemm rc=$?"; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/r02_gputest8.log 2>&1
echo "pytest rc=$?"
