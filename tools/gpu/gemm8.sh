# 256x256 phased GEMM: bitwise self-check against the 128x128 kernel, then
# tile-variant microbench on the decoder shapes.
set -o pipefail
mkdir -p gpurun_out/gemm8
timeout -k 10 120 python -u tools/gemm_selftest.py > gpurun_out/gemm8/selftest.txt 2>&1 && \
timeout -k 10 400 python -u tools/bench_gemm.py 0,3,20,21,22,23 1,2,3 "78016x1536x512;78016x512x1536;78016x1024x512;78016x512x512;78016x1920x512;78016x1152x512;4096x4096x4096;8192x8192x8192" > gpurun_out/gemm8/gemm_variants.txt 2>&1
