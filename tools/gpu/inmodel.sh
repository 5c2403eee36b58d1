# In-model A/B after the epilogue change: per-shape forward profile (default
# tiles vs ZV_GEMM_TILE=3), then the benchmark line.
set -o pipefail
mkdir -p gpurun_out/inmodel
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/inmodel/fwd_t0.txt 2>&1 && \
ZV_GEMM_TILE=3 timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > gpurun_out/inmodel/fwd_t3.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode > gpurun_out/inmodel/bench.json 2> gpurun_out/inmodel/bench.err
