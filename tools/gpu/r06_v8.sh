# round 6: attention-score projection tile arms (ZV_N96 2 / 3 / 4), C2 bench
mkdir -p gpurun_out/r06_v8
for i in 1 2; do for a in 2 3 4; do ZV_N96=$a timeout -k 10 200 python -u bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-mode > gpurun_out/r06_v8/b${a}_$i.json 2>/dev/null || exit 1; done; done
