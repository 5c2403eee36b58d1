# In-model A/B: default policy (plain linears 256x128 3-stage, FF3 without the
# dead bf16 copy) vs the 128x128-everywhere arm vs 256-row fused-epilogue tiles.
set -o pipefail
mkdir -p gpurun_out/inmodel2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/inmodel2/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/inmodel2/fwd_def.txt 2>&1 && \
ZV_GEMM_TILE=4 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/inmodel2/fwd_t4.txt 2>&1 && \
ZV_GEMM_FUSED_TILE=1 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/inmodel2/fwd_ft1.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/inmodel2/fwd_def2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode > gpurun_out/inmodel2/bench.json 2> gpurun_out/inmodel2/bench.err
