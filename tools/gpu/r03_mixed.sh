#!/bin/bash
# fp16 parity mode variants: full-size accuracy (C2-C5 velocity vs the oracle, bar 1e-3) and
# the per-kernel step profile, per environment:  tools/gpu/r03_mixed.sh OUT "ENV" ...
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p "$O"
i=0
for e in "$@"; do
  i=$((i + 1))
  envs=(); [ "$e" != "-" ] && read -r -a envs <<< "$e"
  timeout -k 10 400 env "${envs[@]}" python -u -m pytest tests/test_gpu_fullsize.py -x -q -s --timeout 200 \
    --timeout-method thread -k "velocity_full_size_vs_oracle and fp16" > "$O/t$i.log" 2>&1
  echo "=== $e: pytest rc=$?"; grep -E "mean|passed|failed" "$O/t$i.log" | tail -8
  timeout -k 10 300 env "${envs[@]}" python -u tools/mode_profile.py fp16 > "$O/p$i.txt" 2>&1 || { echo "profile rc=$?"; exit 1; }
  tail -3 "$O/p$i.txt"
done
