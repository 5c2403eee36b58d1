#!/bin/bash
# Round 4: hardware queues per process (GPU_MAX_HW_QUEUES: 4, the box's default, vs 8) x decoder
# row-block streams (ZV_SPLIT_STREAMS 3 default, 4): bench C2 bf16 step, interleaved runs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_hwq}; mkdir -p $O
for rep in 1 2; do
  for q in 4 8; do
    for sp in 3 4; do
      n=q${q}_s${sp}_${rep}
      GPU_MAX_HW_QUEUES=$q ZV_SPLIT_STREAMS=$sp timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-fp32-mode > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$n.json'));print('hwq $q split $sp rep $rep', d['ms_per_step'])" | tee -a $O/summary.txt
    done
  done
done
