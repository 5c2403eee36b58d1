#!/bin/bash
# round 2: fp8 (MX) mode performance - C5 bf16 vs fp8, C2 bench in fp8, rocprof kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fp8
mkdir -p $O
timeout -k 10 300 python -u tools/config_bench.py C5 3 bf16 > $O/c5_bf16.txt 2>&1 || { echo "c5 bf16 rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/config_bench.py C5 3 fp8 > $O/c5_fp8.txt 2>&1 || { echo "c5 fp8 rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --precision fp8 --no-cpu-baseline --no-fp32-mode > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench rc=$?"; exit 1; }
ZV_SPLIT_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rp -o run -- python3 bench.py --steps 1 --warmup 1 --precision fp8 --no-cpu-baseline --no-fp32-mode > $O/rp.log 2>&1 || { echo "rp rc=$?"; exit 1; }
echo done
