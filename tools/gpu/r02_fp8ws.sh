#!/bin/bash
# round 2: default ROLE 5 copy (bf16) check + fp8-mode SelfAttention out-projection on the counted
# ROLE 4 epilogue with the fp8 copy (ZV_RESID_WS=0) vs the wave-specialised kernel
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fp8ws
mkdir -p $O
rm -f $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_res.py tests/test_gpu_fp8.py tests/test_gpu_split_streams.py -x -v -s --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
ZV_RESID_WS=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -x -v -s --timeout 300 --timeout-method thread > $O/test_ws0.log 2>&1 || { echo "tests ws0 rc=$?"; exit 1; }
run() {  # flag tag
  timeout -k 10 300 env ZV_RESID_WS=$1 python -u bench.py --precision fp8 --no-cpu-baseline --no-fp32-mode --steps 4 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));k=d['roofline']['per_kernel_ms_per_step'];print('fp8 resid_ws=$1', d['ms_per_step'], 'ws', round(k.get('gemm_bf16_resid_ws',0),1), 'resid', round(k.get('gemm_bf16_resid',0),1))" | tee -a $O/ab.txt
}
run 0 a && run 1 a && run 0 b && run 1 b || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/bf16.json 2>&1 || { echo "bench bf16 rc=$?"; exit 1; }
echo done
