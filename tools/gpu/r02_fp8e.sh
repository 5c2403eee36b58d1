#!/bin/bash
# round 2: fp8 mode with the NonlinAttention in-projection on the fp8 GEMM - tests, timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fp8e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -x -v -s --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --precision fp8 --no-cpu-baseline --no-fp32-mode --steps 4 > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/config_bench.py C5 3 fp8 > $O/c5.txt 2>&1 || { echo "c5 rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/config_bench.py C5 3 bf16 >> $O/c5.txt 2>&1 || { echo "c5 rc=$?"; exit 1; }
echo done
