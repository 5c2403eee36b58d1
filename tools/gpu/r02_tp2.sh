#!/bin/bash
# round 2: Toeplitz scoring in the stats / NonlinAttention kernels too; parity + bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_sa_tp.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -v -s --timeout 400 --timeout-method thread > $O/r02_tp2_test.log 2>&1 || { echo "tests failed rc=$?"; exit 1; }
for tp in 0 1 0 1; do
  ZV_SA_TP=$tp timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_tp2_$tp.json 2> $O/r02_tp2_$tp.err || { echo "bench $tp rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_tp2_$tp.json'));k=d['roofline']['per_kernel_ms_per_step'];print('sa_tp=$tp', d['ms_per_step'], d['value'], 'sa/na/stats ms/step', k.get('attn_sa_bf16'), k.get('attn_na_bf16'), k.get('attn_stats_bf16'))" | tee -a $O/r02_tp2_ab.txt
done
