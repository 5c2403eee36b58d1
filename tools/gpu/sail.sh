# SelfAttention interleaved query tiles: parity, same-box profiles on/off/on.
set -o pipefail
mkdir -p gpurun_out/sail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onnx_compat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sail/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/sail/fwd_on.txt 2>&1 && \
ZV_SA_IL=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/sail/fwd_off.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/sail/fwd_on2.txt 2>&1
