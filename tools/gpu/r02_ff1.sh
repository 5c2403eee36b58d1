#!/bin/bash
# round 2: FF1 residual read as src + temb (ZV_FF1_SRC): BiasNorm and the stack entry skip the fp32 working stream
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ff1
mkdir -p $O
rm -f $O/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gemm_res.py tests/test_gpu_split_streams.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py tests/test_gpu_fp8.py tests/test_gpu_onnx_compat.py -x -v -s --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
run() {  # flag tag
  timeout -k 10 300 env ZV_FF1_SRC=$1 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));k=d['roofline']['per_kernel_ms_per_step'];print('ff1src=$1', d['ms_per_step'], 'resid', round(k.get('gemm_bf16_resid',0),1), 'resid_ws', round(k.get('gemm_bf16_resid_ws',0),1))" | tee -a $O/ab.txt
}
run 1 a && run 0 a && run 1 b && run 0 b || exit 1
echo done
