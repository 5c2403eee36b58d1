#!/bin/bash
# round 2: fp8 (MX) mode - layout probe, GEMM vs numpy spec, model parity
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 5 60 ./tools/probe/mx8_probe > $O/mx8_probe.txt 2>&1 || { echo "probe rc=$?"; cat $O/mx8_probe.txt; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -v -s --timeout 300 --timeout-method thread > $O/r02_fp8_test.log 2>&1
echo "fp8 tests rc=$?"
