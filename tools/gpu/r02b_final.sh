#!/bin/bash
# round 2 (second session) final measurement on the committed tree: PMC HBM traffic of the two roofline
# GEMMs, rocprofv3 kernel stats of the bench command (one decoder stream, as the bench
# roofline's per-kernel event timing), the full bench line, the other configurations, C1
# latency and smoke.  Each GPU step has its own time limit.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02cfinal
mkdir -p $O
RXP='zv_gemm_kernel<128, 128, 2, 2, 1, 0, 2, 2, 64, 0, 0, 0, 3, 1, 0>'
RXR='zv_gemm_kernel<128, 128, 2, 2, 1, 0, 2, 2, 64, 0, 0, 0, 1, 1, 0>'
ZV_SPLIT_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d $O/pmc_fetch -o run -- python3 tools/profile_forward.py --iters 1 > $O/pmc_fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
ZV_SPLIT_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d $O/pmc_write -o run -- python3 tools/profile_forward.py --iters 1 > $O/pmc_write.log 2>&1 || { echo "write rc=$?"; exit 1; }
python3 tools/pmc_traffic.py $(ls $O/pmc_fetch/*counter_collection.csv | head -1) $(ls $O/pmc_write/*counter_collection.csv | head -1) "$RXP" $O/gemm_traffic.json > $O/pmc_traffic.log 2>&1 && \
python3 tools/pmc_traffic.py $(ls $O/pmc_fetch/*counter_collection.csv | head -1) $(ls $O/pmc_write/*counter_collection.csv | head -1) "$RXR" $O/gemm_resid_traffic.json >> $O/pmc_traffic.log 2>&1 && \
cp $O/gemm_traffic.json profiles/r02c_gemm_traffic.json && cp $O/gemm_resid_traffic.json profiles/r02c_gemm_resid_traffic.json || { echo "traffic rc=$?"; exit 1; }
ZV_SPLIT_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/rp_bench.log 2>&1 || { echo "rp rc=$?"; exit 1; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 400 python -u tools/config_bench.py C3,C4,C5 3 > $O/configs.txt 2>&1 || { echo "configs rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/config_bench.py C5 3 fp8 >> $O/configs.txt 2>&1 || { echo "configs fp8 rc=$?"; exit 1; }
timeout -k 10 400 python -u bench.py --config C3 --no-cpu-baseline --no-fp32-mode > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 rc=$?"; exit 1; }
timeout -k 10 200 python -u tools/latency_c1.py bf16 > $O/latency.txt 2>&1 || { echo "latency rc=$?"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?"
