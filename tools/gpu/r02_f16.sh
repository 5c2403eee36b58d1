#!/bin/bash
# round 2: fp16-operand parity-grade mode: GPU test suite (all precisions) + bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/r02_gputest4.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit 1
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $O/r02_bench4.json 2> $O/r02_bench4.err
echo "bench rc=$?"
