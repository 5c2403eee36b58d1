#!/bin/bash
# round 2: decoder row halves on two streams (ZV_SPLIT_STREAMS) - bitwise test, then bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_streams.py -v -s --timeout 250 --timeout-method thread > $O/r02_split_test.log 2>&1 || { echo "split test failed rc=$?"; exit 1; }
for f in 0 1 0 1; do
  ZV_SPLIT_STREAMS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_split_bench_$f.json 2> $O/r02_split_bench_$f.err || { echo "bench $f rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_split_bench_$f.json'));print('split=$f', d['ms_per_step'], d['value'])" | tee -a $O/r02_split_ab.txt
done
