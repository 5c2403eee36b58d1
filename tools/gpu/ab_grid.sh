# Same-box A/B of GEMM occupancy x grid policies (env-selected, one build).
set -o pipefail
mkdir -p gpurun_out/abgrid
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abgrid/fwd_$name.txt 2>&1; }
ZV_LIB_PATH=$PWD/zipvoice_amd/libzipvoice_hip_a.so timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/abgrid/fwd_a.txt 2>&1 && \
run o1g2 ZV_GEMM_OCC_PLAIN=1 ZV_GEMM_GRIDX_PLAIN=2 ZV_GEMM_OCC_FUSED=1 ZV_GEMM_GRIDX_FUSED=2 ZV_GEMM_GRIDX_RESID=4 && \
run o1g4 ZV_GEMM_OCC_PLAIN=1 ZV_GEMM_GRIDX_PLAIN=4 ZV_GEMM_OCC_FUSED=1 ZV_GEMM_GRIDX_FUSED=4 ZV_GEMM_GRIDX_RESID=8 && \
run o1nt ZV_GEMM_OCC_PLAIN=1 ZV_GEMM_GRIDX_PLAIN=-1 ZV_GEMM_OCC_FUSED=1 ZV_GEMM_GRIDX_FUSED=-1 ZV_GEMM_GRIDX_RESID=-1 && \
run o2g4 ZV_GEMM_OCC_PLAIN=2 ZV_GEMM_GRIDX_PLAIN=4 ZV_GEMM_OCC_FUSED=2 ZV_GEMM_GRIDX_FUSED=4 && \
run o2nt ZV_GEMM_OCC_PLAIN=2 ZV_GEMM_GRIDX_PLAIN=-1 ZV_GEMM_OCC_FUSED=2 ZV_GEMM_GRIDX_FUSED=-1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_onnx_compat.py tests/test_gpu_pipeline.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/abgrid/pytest_new.log 2>&1
