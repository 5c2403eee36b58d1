#!/bin/bash
# round 2: GEMM K step with every fragment read up front (PRELOAD): microbench, bitwise GEMM
# tests, bench A/B against the round's previous measurement (r02_minw_ab.txt: 534-538 ms)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/bench_gemm.py 0 4,1,2,3 "78016x512x1536;78016x1024x512;78016x1536x512;78016x512x512;78016x1920x512;19520x512x512" > $O/r02_preload_gemm.log 2>&1 || { echo "gemm rc=$?"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_pp.py tests/test_gpu_resid_ws.py tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread > $O/r02_preload_test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/r02_preload_b$i.json 2> $O/r02_preload_b$i.err || { echo "bench rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('$O/r02_preload_b$i.json'));r=d['roofline'];print('preload', d['ms_per_step'], d['value'], r['avg_launch_us'], r['frac'], r['secondary']['avg_launch_us'], r['secondary']['achieved'])" | tee -a $O/r02_preload_ab.txt
done
