#!/bin/bash
# Round 4: the joined FeedForward launch over the split decoder's row blocks (ZV_FFN_JOIN=1) vs
# per-stream launches (0, default) on the final FF kernel: bench C2 bf16 step, interleaved runs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_join}; mkdir -p $O
for rep in 1 2; do
  for j in 0 1; do
    n=j${j}_${rep}
    ZV_FFN_JOIN=$j timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-fp32-mode > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$n.json'));print('join $j rep $rep', d['ms_per_step'])" | tee -a $O/summary.txt
  done
done
