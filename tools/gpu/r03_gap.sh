#!/bin/bash
# Host calls inside the timed step's idle gaps (kernel + HIP runtime trace, no counters).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/gap2; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $O/t -o run -- python3 tools/trace_step.py --steps 2 > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
grep timed $O/t.log
k=$(ls $O/t/*kernel_trace.csv | head -1); h=$(ls $O/t/*hip_api_trace.csv | head -1)
python3 tools/schedule_account.py "$k" --steps 2 | head -8
python3 tools/gap_api.py "$k" "$h" --top 5
rm -f "$k" "$h"
