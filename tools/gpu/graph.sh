set -o pipefail
mkdir -p gpurun_out/graph
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/graph/pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/latency_c1.py bf16 > gpurun_out/graph/latency.txt 2>&1 && \
ZV_GRAPH=0 timeout -k 10 200 python -u tools/latency_c1.py bf16 > gpurun_out/graph/latency_nograph.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode > gpurun_out/graph/bench.json 2> gpurun_out/graph/bench.err
