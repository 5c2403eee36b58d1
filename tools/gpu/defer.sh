# Deferred epilogue stores (counted vmcnt across the tile boundary): bitwise
# self-check vs the draining kernel, microbench, parity, in-model A/B.
set -o pipefail
mkdir -p gpurun_out/defer
timeout -k 10 120 python -u tools/gemm_selftest.py 40 "1000x384x200;78016x1536x512;4096x512x1920;777x1024x48;300x128x64" > gpurun_out/defer/selftest.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/defer/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_gemm.py 0,40 1,3 "78016x1536x512;78016x1920x512;78016x1152x512;39040x1536x512" > gpurun_out/defer/gemm.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/defer/fwd_on.txt 2>&1 && \
ZV_GEMM_DEFER=0 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/defer/fwd_off.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/defer/fwd_on2.txt 2>&1
