#!/bin/bash
# round 2: counted plain epilogue (ROLE 3) - bitwise tests, microbench, bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
rm -f $O/r02_plain_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_res.py tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread > $O/r02_plain_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/bench_gemm.py 100,172 7 "78016x1536x512;78016x1024x512;19520x1536x512" > $O/r02_plain_micro.txt 2>&1 || { echo "micro rc=$?"; exit 1; }
run() {  # tag flag i
  timeout -k 10 300 env ZV_RES_COUNTED=$2 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_plain_$1$3.json 2> $O/r02_plain_$1$3.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/r02_plain_$1$3.json'));k=d['roofline']['per_kernel_ms_per_step'];print('$1', d['ms_per_step'], d['value'], 'resid', k.get('gemm_bf16_resid'), 'gemm', k.get('gemm_bf16'), 'glu', k.get('gemm_bf16_glu'), 'na', k.get('gemm_bf16_na'))" | tee -a $O/r02_plain_ab.txt
}
run counted 1 1 && run general 0 1 && run counted 1 2 && run general 0 2 || exit 1
