# round 6: skinny value projection (bitwise test + bench A/B); attention lab at a wider score range
mkdir -p gpurun_out/r06_v6
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_vt_proj.py -s > gpurun_out/r06_v6/vt.log 2>&1 || exit 1
for i in 1 2; do for a in 1 0; do ZV_VT_PROJ=$a timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v6/b${a}_$i.json 2>/dev/null || exit 1; done; done
for v in bf16 f16; do timeout -k 10 60 ./tools/lab/attn2_time_$v 21 1219 20 3.0 >> gpurun_out/r06_v6/lab.txt 2>&1 || exit 1; done
