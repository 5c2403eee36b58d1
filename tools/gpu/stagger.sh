# Stagger A/B: the second half of the persistent grid starts 0/1/2/4 x 8k cycles
# late (co-resident blocks out of phase: one's epilogue beside the other's MFMAs).
set -o pipefail
mkdir -p gpurun_out/stagger
timeout -k 10 400 python -u tools/bench_gemm.py 0,1000,2000,4000,100,3,1003,2003 1,2,3 "78016x1536x512;78016x512x1536;78016x512x512;78016x1152x512" > gpurun_out/stagger/gemm.txt 2>&1
