#!/bin/bash
# round 2: full GPU suite on the current tree, then two bench lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/r02_gputest7.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_dw_b$i.json 2> $O/r02_dw_b$i.err || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_dw_b$i.json'));k=d['roofline']['per_kernel_ms_per_step'];print('dw', d['ms_per_step'], d['value'], 'dwconv ms/step', k.get('dwconv_bf16'))" | tee -a $O/r02_dw_ab.txt
done
