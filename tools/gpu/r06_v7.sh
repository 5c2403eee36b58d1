# round 6: persistent skinny value projection (bitwise test + bench A/B)
mkdir -p gpurun_out/r06_v7
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_vt_proj.py -s > gpurun_out/r06_v7/vt.log 2>&1 || exit 1
for i in 1 2; do for a in 1 0; do ZV_VT_PROJ=$a timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v7/b${a}_$i.json 2>/dev/null || exit 1; done; done
