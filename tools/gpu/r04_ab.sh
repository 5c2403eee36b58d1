#!/bin/bash
# Round 4 bench A/B (C2, bf16 leg) after a GPU test subset: tools/gpu/r04_ab.sh OUT ROUNDS "TESTS" ENV...
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
N=$1; O=gpurun_out/$1; R=$2; T=$3; shift 3
mkdir -p $O
if [ "$T" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  grep -E "PASS|FAIL|passed|failed" $O/pytest.log | tail -20
fi
bash tools/gpu/ab_env.sh $N/ab $R "$@"
