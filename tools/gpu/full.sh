# Round validation + measurement: GPU tests, smoke, bench, rocprofv3 kernel stats,
# PMC traffic passes for the dominant GEMM.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out/full
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/full/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > gpurun_out/full/rp_bench.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d gpurun_out/full/pmc_fetch -o run -- python3 tools/profile_forward.py --iters 1 > gpurun_out/full/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d gpurun_out/full/pmc_write -o run -- python3 tools/profile_forward.py --iters 1 > gpurun_out/full/pmc_write.log 2>&1 && \
timeout -k 10 200 python -u tools/latency_c1.py bf16 > gpurun_out/full/latency.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/full/rp_lat -o run -- python3 tools/latency_c1.py bf16 > gpurun_out/full/rp_lat.log 2>&1
