#!/bin/bash
# Same-box interleaved A/B of two engine libraries on tools/config_bench.py configurations
# (per-GPU shares of the 8-GPU configs): tools/gpu/r05_cfg_tiles_ab.sh OUT ROUNDS OLD_LIB CFG...
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; OLD=$3; shift 3
mkdir -p "$O"; : > "$O/ab.txt"
for r in $(seq 1 "$R"); do
  for c in "$@"; do
    for arm in new old; do
      if [ $arm = old ]; then L="ZV_LIB_PATH=$OLD"; else L="ZV_NOTHING=0"; fi
      timeout -k 10 300 env "$L" python -u tools/config_bench.py $c 3 > "$O/${c}_${arm}_$r.json" 2> "$O/${c}_${arm}_$r.err" \
        || { echo "$c $arm rc=$?"; tail -5 "$O/${c}_${arm}_$r.err"; exit 1; }
      echo "$c $arm $(tail -1 "$O/${c}_${arm}_$r.json")" | tee -a "$O/ab.txt"
    done
  done
done
echo done
