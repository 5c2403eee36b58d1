# Epilogue 8-column chunks + BK=32 4-stage variants: GPU tests, GEMM self-check,
# tile-variant microbench with the store ablation (mode 4).
set -o pipefail
mkdir -p gpurun_out/bk32
timeout -k 10 120 python -u tools/gemm_selftest.py 22,30 "1000x300x200;78016x1536x512;4096x512x1920;777x1024x48" > gpurun_out/bk32/selftest.txt 2>&1 && \
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bk32/pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_gemm.py 0,3,30,31 1,2,3,4 "78016x1536x512;78016x512x1536;78016x1024x512;78016x512x512;78016x1152x512;78016x512x48" > gpurun_out/bk32/gemm_variants.txt 2>&1
