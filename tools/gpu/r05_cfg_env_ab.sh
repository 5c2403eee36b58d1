#!/bin/bash
# Same-box interleaved A/B of engine environments on tools/config_bench.py configurations:
#   tools/gpu/r05_cfg_env_ab.sh OUT ROUNDS "CFG ..." "ENV_A" "ENV_B" ...   (ENV_x: "K=V" or "-")
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; CFGS=$3; shift 3
mkdir -p "$O"; : > "$O/ab.txt"
for r in $(seq 1 "$R"); do
  for c in $CFGS; do
    i=0
    for e in "$@"; do
      i=$((i + 1))
      envs=(ZV_NOTHING=0); [ "$e" != "-" ] && read -r -a envs <<< "$e"
      timeout -k 10 300 env "${envs[@]}" python -u tools/config_bench.py $c 3 > "$O/${c}_${i}_$r.json" 2> "$O/${c}_${i}_$r.err" \
        || { echo "$c $e rc=$?"; tail -5 "$O/${c}_${i}_$r.err"; exit 1; }
      echo "$c [$e] $(python3 -c "import json;print(json.load(open('$O/${c}_${i}_$r.json'))['ms_per_step'])")" | tee -a "$O/ab.txt"
    done
  done
done
echo done
