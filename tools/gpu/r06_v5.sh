# round 6: conv front with uniform chunk bounds + asm packed-FMA blocks; attention timing lab; per-shape report
mkdir -p gpurun_out/r06_v5
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv_fused.py -s > gpurun_out/r06_v5/conv.log 2>&1 || exit 1
for i in 1 2; do for a in 1 0; do ZV_GLU_DW=$a timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v5/b${a}_$i.json 2>/dev/null || exit 1; done; done
for L in 1219 610 305; do for v in bf16 f16; do timeout -k 10 60 ./tools/lab/attn2_time_$v 21 $L 20 >> gpurun_out/r06_v5/lab.txt 2>&1 || exit 1; done; done
timeout -k 10 200 python -u tools/profile_forward.py --iters 2 --report > gpurun_out/r06_v5/report.txt 2>&1
