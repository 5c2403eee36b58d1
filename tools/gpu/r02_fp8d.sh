#!/bin/bash
# round 2: fp8 fused-copy A/B (ZV_FP8_FUSE) after the DPP block max: tests, then bench per setting
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fp8d
mkdir -p $O
rm -f $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -x -v -s --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { echo "tests rc=$?"; exit 1; }
run() {  # fuse tag
  timeout -k 10 300 env ZV_FP8_FUSE=$1 python -u bench.py --precision fp8 --no-cpu-baseline --no-fp32-mode --steps 4 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench rc=$?"; return 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));k=d['roofline']['per_kernel_ms_per_step'];print('fuse=$1', d['ms_per_step'], 'resid_ws', round(k.get('gemm_bf16_resid_ws',0),1), 'dwconv', round(k.get('dwconv_bf16',0),1))" | tee -a $O/ab.txt
}
run 7 a && run 0 a && run 4 a && run 6 a && run 7 b && run 0 b || exit 1
echo done
