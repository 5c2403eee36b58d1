# round 6: fused FeedForward row threshold (ZV_FFN_MIN_ROWS 15000 / 20000 / 40000), C2 bench
mkdir -p gpurun_out/r06_v10
for i in 1 2; do for a in 15000 20000 40000; do ZV_FFN_MIN_ROWS=$a timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v10/b${a}_$i.json 2>/dev/null || exit 1; done; done
for i in 1 2; do for a in 0 1; do ZV_NA_TILE=$a timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v10/na${a}_$i.json 2>/dev/null || exit 1; done; done
