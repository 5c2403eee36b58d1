# SelfAttention positional term on f32 MFMA: parity (default = MFMA form), then
# same-box forward profiles MFMA vs VALU form.
set -o pipefail
mkdir -p gpurun_out/samf
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onnx_compat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/samf/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/samf/fwd_mf.txt 2>&1 && \
ZV_SA_POS_MFMA=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/samf/fwd_valu.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/samf/fwd_mf2.txt 2>&1
