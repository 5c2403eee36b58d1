#!/bin/bash
# Round-5 validation: the GPU suite (all failures listed, not -x), then the C2 bench line (no CPU
# baseline, no fp32 leg) with per-kernel event timings.   tools/gpu/r05_val.sh OUT [PYTEST_ARGS]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_val}; mkdir -p $O
shift
timeout -k 10 700 python -u -m pytest tests -m gpu --timeout 150 --timeout-method thread ${@:--q} > $O/pytest.log 2>&1
rc=$?
tail -25 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc       # 1 = test failures (reported); anything else: stop
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-fp32-mode --steps 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('ms/step', d['ms_per_step'], 'value', d['value'])
for k in ('roofline','legs','per_kernel_ms_per_step'):
    print(k, json.dumps(d.get(k))[:1500])
"
exit $rc
