# Profiling pass: per-shape event profile of one guided forward, library-GEMM
# yardstick, GEMM microbench, rocprofv3 kernel stats of a short bench run.
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 200 python -u tools/profile_forward.py --report > gpurun_out/prof/forward_report.txt 2>&1 && \
timeout -k 10 200 python -u tools/torch_gemm_ref.py > gpurun_out/prof/torch_gemm.txt 2>&1 && \
timeout -k 10 200 python -u tools/bench_gemm.py 0,3 1,2 > gpurun_out/prof/gemm_variants.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > gpurun_out/prof/rp_bench.log 2>&1
