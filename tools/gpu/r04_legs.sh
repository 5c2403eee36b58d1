#!/bin/bash
# Round 4: the bench's later legs (fp32, fp16 engines built after the bf16 one in the same process)
# with the earlier engines collected before the next is built (ZV_BENCH_GC=1, default) or left to
# the collector (0), and the fp16 mode as the process's first engine (--precision fp16).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_legs}; mkdir -p $O
for rep in 1 2; do
  for gc in 1 0; do
    n=gc${gc}_${rep}
    ZV_BENCH_GC=$gc timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$n.json'));print('gc $gc rep $rep bf16', d['ms_per_step'], 'fp32', d['fp32_accurate_mode']['ms_per_step'], 'fp16', d['fp16_parity_mode']['ms_per_step'])" | tee -a $O/summary.txt
  done
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --precision fp16 > $O/f16_$rep.json 2> $O/f16_$rep.err || { tail -20 $O/f16_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f16_$rep.json'));print('fp16 first engine rep $rep', d['ms_per_step'])" | tee -a $O/summary.txt
done
