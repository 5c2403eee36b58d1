#!/bin/bash
# round 2: deeper-ring arm of the staggered GEMM (no-epilogue mode only), then the GPU suite
# (fp16 mixed mode with split attention-score projections) and the bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/bench_gemm.py 0,50,52,53 4 "78016x1536x512;78016x512x1536;78016x1024x512;78016x512x512" > $O/r02_pp3_bench.log 2>&1 || { echo "bench_gemm rc=$?"; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/r02_gputest5.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit 1
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $O/r02_bench5.json 2> $O/r02_bench5.err
echo "bench rc=$?"
