#!/bin/bash
# round 2: ping-pong GEMM first check: bitwise selftest, microbench vs the 128x128 kernel,
# GPU test suite, bench line.  Every GPU step has its own time limit; stop at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/gemm_selftest.py 50 "1000x384x200;78016x1536x512;4096x512x1920;777x1024x48;256x256x64;129x128x600" > $O/r02_pp2_selftest.log 2>&1 || { echo "selftest rc=$?"; exit 1; }
timeout -k 10 400 python -u tools/bench_gemm.py 0,50 1,2,3,4 "78016x1536x512;78016x512x1536;78016x1920x512;78016x512x1920;78016x1024x512;78016x512x512;78016x512x48;19520x512x512" > $O/r02_pp2_bench.log 2>&1 || { echo "bench_gemm rc=$?"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/r02_gputest3.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/r02_bench3.json 2> $O/r02_bench3.err
echo "bench rc=$?"
