# GEMM tile variants after the epilogue register fix (no scratch for TM/TN = 8),
# plus the parity subset for the changed epilogue.
set -o pipefail
mkdir -p gpurun_out/tiles2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decoder_forward or sample_c1" > gpurun_out/tiles2/pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_gemm.py 0,2,3,5,8,9,10 1,2,3 "78016x1536x512;78016x512x1536;78016x1024x512;78016x512x512;78016x1920x512;78016x512x1920;4096x4096x4096" > gpurun_out/tiles2/gemm_variants.txt 2>&1
