# Round validation + measurement on the current tree: every GPU test, smoke,
# PMC traffic of the two roofline GEMM instantiations (residual-stream linears,
# ROLE = 1, and the plain linears; separate FETCH_SIZE / WRITE_SIZE passes),
# the benchmark line (reading that traffic), a rocprofv3 kernel-trace of the
# benchmark, and the C1 latency.  Each GPU step has its own time limit.
set -o pipefail
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
RXP='zv_gemm_kernel<128, 128, 2, 2, 1, 0, 2, 2, 64, 0, 0, 0, 0>'
RXR='zv_gemm_kernel<128, 128, 2, 2, 1, 0, 2, 2, 64, 0, 0, 0, 1>'
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d $OUT/pmc_fetch -o run -- python3 tools/profile_forward.py --iters 1 > $OUT/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d $OUT/pmc_write -o run -- python3 tools/profile_forward.py --iters 1 > $OUT/pmc_write.log 2>&1 && \
python3 tools/pmc_traffic.py $(ls $OUT/pmc_fetch/*counter_collection.csv | head -1) $(ls $OUT/pmc_write/*counter_collection.csv | head -1) "$RXP" $OUT/gemm_traffic.json > $OUT/pmc_traffic.log 2>&1 && \
python3 tools/pmc_traffic.py $(ls $OUT/pmc_fetch/*counter_collection.csv | head -1) $(ls $OUT/pmc_write/*counter_collection.csv | head -1) "$RXR" $OUT/gemm_resid_traffic.json >> $OUT/pmc_traffic.log 2>&1 && \
cp $OUT/gemm_traffic.json profiles/r01_gemm_traffic.json && \
cp $OUT/gemm_resid_traffic.json profiles/r01_gemm_resid_traffic.json && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $OUT/rp_bench.log 2>&1 && \
timeout -k 10 200 python -u tools/latency_c1.py bf16 > $OUT/latency.txt 2>&1 && \
timeout -k 10 200 python -u tools/profile_forward.py --report --iters 3 > $OUT/forward_report.txt 2>&1
