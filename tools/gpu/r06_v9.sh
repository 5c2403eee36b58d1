# round 6: residual-linear tile arms (ZV_RESID_TILE 0 / 1 / 2), C2 bench
mkdir -p gpurun_out/r06_v9
for i in 1 2; do for a in 0 1 2; do ZV_RESID_TILE=$a timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v9/b${a}_$i.json 2>/dev/null || exit 1; done; done
