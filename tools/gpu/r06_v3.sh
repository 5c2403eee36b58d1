set -o pipefail
mkdir -p gpurun_out/r06_v3
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv_fused.py -s > gpurun_out/r06_v3/conv.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_attn2.py -s > gpurun_out/r06_v3/attn2.log 2>&1; echo "attn2 rc=$?" >> gpurun_out/r06_v3/attn2.log
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -s > gpurun_out/r06_v3/parity.log 2>&1; echo "parity rc=$?" >> gpurun_out/r06_v3/parity.log
timeout -k 10 300 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r06_v3/bench.json 2> gpurun_out/r06_v3/bench.err || exit 1
ZV_GLU_DW=0 timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v3/b0.json 2>/dev/null || exit 1
