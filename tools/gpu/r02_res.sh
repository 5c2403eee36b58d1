#!/bin/bash
# round 2: counted residual epilogue (ROLE 1/2) - bitwise tests, parity subset, microbench,
# bench A/B (ZV_RES_COUNTED=0/1), rocprof kernel stats (one decoder stream)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
rm -f $O/r02_res_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_res.py tests/test_gpu_resid_ws.py tests/test_gpu_parity.py tests/test_gpu_split_streams.py -v -s --timeout 300 --timeout-method thread > $O/r02_res_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/bench_gemm.py 100,170 5,6 "78016x512x1536;78016x512x512;19520x512x512;78016x512x1152" > $O/r02_res_micro.txt 2>&1 || { echo "micro rc=$?"; exit 1; }
run() {  # tag flag i
  timeout -k 10 300 env ZV_RES_COUNTED=$2 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_res_$1$3.json 2> $O/r02_res_$1$3.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/r02_res_$1$3.json'));k=d['roofline']['per_kernel_ms_per_step'];print('$1', d['ms_per_step'], d['value'], 'resid', k.get('gemm_bf16_resid'), 'gemm', k.get('gemm_bf16'), 'sa', k.get('attn_sa_bf16'), 'roof', d['roofline']['achieved'], d['roofline']['frac'])" | tee -a $O/r02_res_ab.txt
}
run counted 1 1 && run general 0 1 && run counted 1 2 && run general 0 2 || exit 1
ZV_SPLIT_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/r02res -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/r02_res_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
f=$(find $O/r02res -name '*kernel_stats.csv' | head -1); head -8 "$f" | cut -c1-200 | tee -a $O/r02_res_ab.txt
