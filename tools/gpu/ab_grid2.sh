# Same-box A/B after the uniform-activation fix: plain/fused policies.
set -o pipefail
mkdir -p gpurun_out/abgrid2
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abgrid2/fwd_$name.txt 2>&1; }
ZV_LIB_PATH=$PWD/zipvoice_amd/libzipvoice_hip_a.so timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abgrid2/fwd_a.txt 2>&1 && \
run p1g2 ZV_GEMM_OCC_PLAIN=1 ZV_GEMM_GRIDX_PLAIN=2 ZV_GEMM_OCC_RESID=2 ZV_GEMM_GRIDX_RESID=-1 && \
run p1g0 ZV_GEMM_OCC_PLAIN=1 ZV_GEMM_GRIDX_PLAIN=0 ZV_GEMM_OCC_RESID=2 ZV_GEMM_GRIDX_RESID=-1 && \
run p1nt ZV_GEMM_OCC_PLAIN=1 ZV_GEMM_GRIDX_PLAIN=-1 ZV_GEMM_OCC_RESID=2 ZV_GEMM_GRIDX_RESID=-1 && \
run p2g0 ZV_GEMM_OCC_PLAIN=2 ZV_GEMM_GRIDX_PLAIN=0 ZV_GEMM_OCC_RESID=2 ZV_GEMM_GRIDX_RESID=-1 ZV_GEMM_OCC_FUSED=2 && \
run p2nt ZV_GEMM_OCC_PLAIN=2 ZV_GEMM_GRIDX_PLAIN=-1 ZV_GEMM_OCC_RESID=2 ZV_GEMM_GRIDX_RESID=-1 ZV_GEMM_OCC_FUSED=2 ZV_GEMM_GRIDX_FUSED=-1 && \
timeout -k 10 200 python -u tools/latency_c1.py bf16 > gpurun_out/abgrid2/latency.txt 2>&1
