#!/bin/bash
# Round 4 GPU session Q: the final tree's FF / split / parity / fullsize tests and the bench line.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_q}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_split_streams.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_host_sync.py -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['ms_per_step'],d['value'],r['kernel'],r['frac'],r['avg_launch_us'],r.get('traffic_over_algorithmic'));print({k:v['ms_per_step'] for k,v in d.items() if isinstance(v,dict) and 'ms_per_step' in v})"
