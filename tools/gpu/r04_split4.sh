#!/bin/bash
# Round 4: decoder row blocks on 4 streams (the new default) vs 3: the split / host-sync GPU tests,
# then interleaved bench runs (C2 bf16 step, --steps 8) with ZV_SPLIT_STREAMS explicit.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_split4}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_streams.py tests/test_gpu_host_sync.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | tail -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for sp in 3 4; do
    n=s${sp}_${rep}
    ZV_SPLIT_STREAMS=$sp timeout -k 10 300 python -u bench.py --steps 8 --no-cpu-baseline --no-fp32-mode > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$n.json'));print('split $sp rep $rep', d['ms_per_step'], d.get('fp16_parity_mode', {}).get('ms_per_step'))" | tee -a $O/summary.txt
  done
done
