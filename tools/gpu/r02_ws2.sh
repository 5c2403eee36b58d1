#!/bin/bash
# round 2: wave-specialised residual GEMM with the fragment preload, on every residual linear
# (ZV_RESID_WS=2) vs K <= 64 only (default 1); bitwise test first
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resid_ws.py -v -s --timeout 250 --timeout-method thread > $O/r02_ws2_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for ws in 1 2 1 2; do
  ZV_RESID_WS=$ws timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_ws2_$ws.json 2> $O/r02_ws2_$ws.err || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_ws2_$ws.json'));r=d['roofline'];k=r['per_kernel_ms_per_step'];print('resid_ws=$ws', d['ms_per_step'], d['value'], 'resid', k.get('gemm_bf16_resid'), 'resid_ws', k.get('gemm_bf16_resid_ws'))" | tee -a $O/r02_ws2_ab.txt
done
