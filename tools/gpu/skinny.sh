# Skinny-GEMM tiles (N = 272 on 128x96, V^T N = 48 on 64x64 one tile per block):
# parity, same-box forward profiles on/off.
set -o pipefail
mkdir -p gpurun_out/skinny
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/skinny/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/skinny/fwd_on.txt 2>&1 && \
ZV_GEMM_SKINNY=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/skinny/fwd_off.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/skinny/fwd_on2.txt 2>&1
