#!/bin/bash
# round 2 measurement: counter list, PMC HBM traffic of the two roofline GEMMs, SQ
# instruction counters of the attention kernels (VALU vs Toeplitz scoring), rocprofv3
# kernel stats of the bench command (one decoder stream: the roofline's per-kernel
# durations are single-stream), then the full default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02prof
mkdir -p $O
RXP='zv_gemm_kernel<128, 128, 2, 2, 1, 0, 2, 2, 64, 0, 0, 0, 0>'
RXR='zv_gemm_kernel<128, 128, 2, 2, 1, 0, 2, 2, 64, 0, 0, 0, 1>'
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list rc=$?"
ZV_SPLIT_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d $O/pmc_fetch -o run -- python3 tools/profile_forward.py --iters 1 > $O/pmc_fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
ZV_SPLIT_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex zv_gemm_kernel -d $O/pmc_write -o run -- python3 tools/profile_forward.py --iters 1 > $O/pmc_write.log 2>&1 || { echo "write rc=$?"; exit 1; }
python3 tools/pmc_traffic.py $(ls $O/pmc_fetch/*counter_collection.csv | head -1) $(ls $O/pmc_write/*counter_collection.csv | head -1) "$RXP" $O/gemm_traffic.json > $O/pmc_traffic.log 2>&1 && \
python3 tools/pmc_traffic.py $(ls $O/pmc_fetch/*counter_collection.csv | head -1) $(ls $O/pmc_write/*counter_collection.csv | head -1) "$RXR" $O/gemm_resid_traffic.json >> $O/pmc_traffic.log 2>&1 && \
cp $O/gemm_traffic.json profiles/r02_gemm_traffic.json && cp $O/gemm_resid_traffic.json profiles/r02_gemm_resid_traffic.json || { echo "traffic rc=$?"; exit 1; }
SQ=""
for c in SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU; do
  grep -q "\b$c\b" $O/counters.txt && SQ="$SQ $c"
done
echo "SQ counters: $SQ" | tee $O/sq_set.txt
for tp in 0 1; do
  ZV_SA_TP=$tp ZV_SPLIT_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc $SQ -f csv --kernel-include-regex zv_attn -d $O/sq_tp$tp -o run -- python3 tools/profile_forward.py --iters 1 > $O/sq_tp$tp.log 2>&1 || { echo "sq $tp rc=$?"; exit 1; }
done
ZV_SPLIT_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rp -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/rp_bench.log 2>&1 || { echo "rp rc=$?"; exit 1; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"
