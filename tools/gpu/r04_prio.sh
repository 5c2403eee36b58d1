#!/bin/bash
# Round 4: the split decoder's row-block stream priority (ZV_STREAM_PRIO: 0 default, 1 the two
# side streams at the greatest priority, -1 at the least), bench C2 bf16 step, interleaved runs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_prio}; mkdir -p $O
for rep in 1 2; do
  for p in 0 1 -1; do
    ZV_STREAM_PRIO=$p timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-fp32-mode > $O/b_${p}_${rep}.json 2> $O/b_${p}_${rep}.err || { tail -20 $O/b_${p}_${rep}.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${p}_${rep}.json'));print('prio $p rep $rep', d['ms_per_step'])" | tee -a $O/summary.txt
  done
done
