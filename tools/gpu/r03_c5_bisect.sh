#!/bin/bash
# C5 (stereo) / C3 per-GPU step time under policy environments (tools/config_bench.py).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/c5b; mkdir -p $O
cfgs=$1; shift
i=0
for e in "$@"; do
  i=$((i + 1))
  envs=(); [ "$e" != "-" ] && read -r -a envs <<< "$e"
  timeout -k 10 300 env "${envs[@]}" python -u tools/config_bench.py $cfgs 3 > $O/r$i.txt 2>&1 || { echo "rc=$? ($e)"; tail -5 $O/r$i.txt; exit 1; }
  python3 -c "
import json,sys
for l in open('$O/r$i.txt'):
    if l.startswith('{'): d=json.loads(l); print('$e', d['config'], d['ms_per_step'])"
done
