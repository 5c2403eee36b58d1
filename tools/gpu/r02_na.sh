#!/bin/bash
# round 2: pipelined NonlinAttention - parity subset, then two bench lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sa_tp.py -v -s --timeout 400 --timeout-method thread > $O/r02_na_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_na_b$i.json 2> $O/r02_na_b$i.err || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_na_b$i.json'));k=d['roofline']['per_kernel_ms_per_step'];print('na-pipelined', d['ms_per_step'], d['value'], 'na', k.get('attn_na_bf16'), 'stats', k.get('attn_stats_bf16'))" | tee -a $O/r02_na_ab.txt
done
