#!/bin/bash
# Same-box A/B of engine environments on C3 / C4 / C5 (tools/config_bench.py), interleaved:
#   tools/gpu/r05_cfg_ab.sh OUT ROUNDS CONFIGS "ENV_A" "ENV_B" ...   (ENV_x: "K=V K2=V2" or "-")
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; C=$3; shift 3
mkdir -p "$O"
: > "$O/ab.txt"
for r in $(seq 1 "$R"); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=(); [ "$e" != "-" ] && read -r -a envs <<< "$e"
    timeout -k 10 300 env "${envs[@]}" python -u tools/config_bench.py "$C" 2 > "$O/c_${i}_$r.json" 2> "$O/c_${i}_$r.err" \
      || { echo "config_bench rc=$? ($e)"; tail -5 "$O/c_${i}_$r.err"; exit 1; }
    python3 -c "
import json
for l in open('$O/c_${i}_$r.json'):
    d=json.loads(l); print('$e', d['config'], d['ms_per_step'])" | tee -a "$O/ab.txt"
  done
done
echo done
