#!/bin/bash
# Same-box A/B of the full bench line (bf16 + the fp16 / fp32 legs in one process) across engine
# environments:  tools/gpu/r05_legs_ab.sh OUT ROUNDS "ENV_A" "ENV_B" ...
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 "$R"); do
  i=0
  for e in "$@"; do
    i=$((i + 1)); envs=(); [ "$e" != "-" ] && read -r -a envs <<< "$e"
    timeout -k 10 400 env "${envs[@]}" python -u bench.py --steps 3 --no-cpu-baseline > $O/b_${i}_$r.json 2> $O/b_${i}_$r.err || { echo "rc=$? ($e)"; tail -5 $O/b_${i}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${i}_$r.json'));print('$e', d['ms_per_step'], {k:v['ms_per_step'] for k,v in d.items() if isinstance(v,dict) and 'ms_per_step' in v})" | tee -a $O/ab.txt
  done
done
