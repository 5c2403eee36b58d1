# Residual-linear tile A/B (128x128 default vs 64x128 vs 128x64), same box.
set -o pipefail
mkdir -p gpurun_out/rtile
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "decoder_forward" > gpurun_out/rtile/pytest.log 2>&1 && \
ZV_RESID_TILE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "decoder_forward" >> gpurun_out/rtile/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/rtile/fwd_0.txt 2>&1 && \
ZV_RESID_TILE=1 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/rtile/fwd_1.txt 2>&1 && \
ZV_RESID_TILE=2 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/rtile/fwd_2.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/rtile/fwd_0b.txt 2>&1
