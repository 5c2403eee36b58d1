#!/bin/bash
# round 2: dual-group residual GEMM - bitwise tests, microbench vs the 128x128 kernel, bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_dual.py -v -s --timeout 120 --timeout-method thread > $O/r02_dual_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/bench_gemm.py 100,60 2 "78016x512x1536;78016x512x512;78016x512x1152;78016x512x384;78016x512x1920;19520x512x512" > $O/r02_dual_gemm.log 2>&1 || { echo "gemm rc=$?"; exit 1; }
for f in 0 1; do
  ZV_GEMM_DUAL=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_dual_b$f.json 2> $O/r02_dual_b$f.err || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_dual_b$f.json'));k=d['roofline']['per_kernel_ms_per_step'];print('dual=$f', d['ms_per_step'], d['value'], 'resid', k.get('gemm_bf16_resid'), 'dual', k.get('gemm_bf16_resid_dual'))" | tee -a $O/r02_dual_ab.txt
done
