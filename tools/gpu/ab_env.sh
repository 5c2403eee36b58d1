#!/bin/bash
# Same-box A/B of engine policy environments on the C2 bench (bf16 leg only), interleaved:
#   tools/gpu/ab_env.sh OUTDIR ROUNDS "ENV_A" "ENV_B" ...   (ENV_x: "K=V K2=V2" or "-")
# Optional PYTEST=1 runs the GPU parity subset first (stops on failure).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; shift 2
mkdir -p "$O"
: > "$O/ab.txt"
if [ "${PYTEST:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
for r in $(seq 1 "$R"); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=(); [ "$e" != "-" ] && read -r -a envs <<< "$e"
    timeout -k 10 300 env "${envs[@]}" python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 4 ${BENCH_ARGS:-} \
      > "$O/b_${i}_$r.json" 2> "$O/b_${i}_$r.err" || { echo "bench rc=$? ($e)"; tail -5 "$O/b_${i}_$r.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${i}_$r.json'));print('$e', d['ms_per_step'])" | tee -a "$O/ab.txt"
  done
done
echo done
