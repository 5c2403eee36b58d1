#!/bin/bash
# round 2: 96-wide tiles for the N=272 projection - parity subset, bench x2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_split_streams.py -v -s --timeout 400 --timeout-method thread > $O/r02_n96_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_n96_b$i.json 2> $O/r02_n96_b$i.err || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_n96_b$i.json'));k=d['roofline']['per_kernel_ms_per_step'];print('n96+dw-r01', d['ms_per_step'], d['value'], 'gemm_bf16', k.get('gemm_bf16'), 'n96', k.get('gemm_bf16_n96'), 'dwconv', k.get('dwconv_bf16'))" | tee -a $O/r02_n96_ab.txt
done
