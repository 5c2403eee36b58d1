#!/bin/bash
# round 2: row-block small linear (time-embedding MLP) - parity suite, bench, kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/smalllin
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; exit 1; }
ZV_SPLIT_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rp -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/rp.log 2>&1 || { echo "rp rc=$?"; exit 1; }
echo done
