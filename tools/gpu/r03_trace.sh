#!/bin/bash
# Kernel traces of the timed C2 step (default decoder streams) under policy environments,
# accounted by tools/schedule_account.py:   tools/gpu/r03_trace.sh OUTDIR "ENV_A" "ENV_B" ...
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p "$O"
i=0
for e in "$@"; do
  i=$((i + 1))
  envs=(); [ "$e" != "-" ] && read -r -a envs <<< "$e"
  for kv in "${envs[@]}"; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$O/t$i" -o run -- python3 tools/trace_step.py --steps 2 \
    > "$O/t$i.log" 2>&1 || { echo "trace rc=$? ($e)"; tail -5 "$O/t$i.log"; exit 1; }
  for kv in "${envs[@]}"; do unset "${kv%%=*}"; done
  f=$(ls "$O"/t$i/*kernel_trace.csv | head -1)
  echo "=== $e: $(grep timed "$O/t$i.log")"
  python3 tools/schedule_account.py "$f" --steps 2 --json "$O/t$i.json" | tee "$O/t$i.txt"
  rm -f "$f"
done
echo done
