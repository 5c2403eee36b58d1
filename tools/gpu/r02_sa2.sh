#!/bin/bash
# round 2: SA Toeplitz loop unrolled by two with unconditional prefetch, fp16-pair key mask;
# tests, bench x2; then the same tree built with -fno-slp-vectorize (no packed-f32 VALU
# beside MFMAs) x2; rocprof stats of the default build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
rm -f $O/r02_sa2_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_sa_tp.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -v -s --timeout 400 --timeout-method thread > $O/r02_sa2_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
run() {  # tag lib i
  timeout -k 10 300 env ZV_LIB_PATH=$2 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_sa2_$1$3.json 2> $O/r02_sa2_$1$3.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/r02_sa2_$1$3.json'));k=d['roofline']['per_kernel_ms_per_step'];print('$1', d['ms_per_step'], d['value'], 'sa', k.get('attn_sa_bf16'), 'resid', k.get('gemm_bf16_resid'), 'gemm', k.get('gemm_bf16'), 'dw', k.get('dwconv_bf16'), 'ws', k.get('gemm_bf16_resid_ws'))" | tee -a $O/r02_sa2_ab.txt
}
run sa2 "" 1 && run noslp zipvoice_amd/alt/libzv_noslp.so 1 && run sa2 "" 2 && run noslp zipvoice_amd/alt/libzv_noslp.so 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r02sa2 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-mode > $O/r02_sa2_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
f=$(find $O/r02sa2 -name '*kernel_stats.csv' | head -1); grep -E "sa_tp|Name" "$f" | tee -a $O/r02_sa2_ab.txt
