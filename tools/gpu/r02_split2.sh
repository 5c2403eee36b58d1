#!/bin/bash
# round 2: k-way split decoder + Toeplitz-positional SelfAttention: tests, bench A/B, GPU suite
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split_streams.py tests/test_gpu_sa_tp.py -v -s --timeout 250 --timeout-method thread > $O/r02_split2_test.log 2>&1 || { echo "tests failed rc=$?"; exit 1; }
for cfg in "1 0" "2 0" "2 1" "3 1" "4 1" "1 1"; do
  set -- $cfg
  ZV_SPLIT_STREAMS=$1 ZV_SA_TP=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_s2_$1_$2.json 2> $O/r02_s2_$1_$2.err || { echo "bench $cfg rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_s2_$1_$2.json'));k=d['roofline']['per_kernel_ms_per_step'];print('split=$1 sa_tp=$2', d['ms_per_step'], d['value'], 'attn_sa ms/step', k.get('attn_sa_bf16'))" | tee -a $O/r02_split2_ab.txt
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/r02_gputest6.log 2>&1
echo "pytest rc=$?"
