#!/bin/bash
# round 2: fp8 mode with fused fp8 copies (BiasNorm, depthwise conv, wave-specialised residual
# epilogue) - tests (fp8 + counted-epilogue bitwise + parity), then C5 / C2 timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fp8c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_res.py tests/test_gpu_fp8.py -x -v -s --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/config_bench.py C5 3 fp8 > $O/c5_fp8.txt 2>&1 || { echo "c5 fp8 rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/config_bench.py C5 3 bf16 > $O/c5_bf16.txt 2>&1 || { echo "c5 bf16 rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --precision fp8 --no-cpu-baseline --no-fp32-mode > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench rc=$?"; exit 1; }
echo done
