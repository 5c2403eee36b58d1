# LDS-tiled depthwise conv: parity (decoder/text-encoder fixtures, both modes),
# same-box forward profiles tiled vs register-window.
set -o pipefail
mkdir -p gpurun_out/dwconv
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onnx_compat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dwconv/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/dwconv/fwd_tiled.txt 2>&1 && \
ZV_DWCONV_TILED=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/dwconv/fwd_win.txt 2>&1
