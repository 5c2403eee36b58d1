cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/v5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_split_streams.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/config_bench.py C3,C4,C5 3 > $O/cfg1.txt 2>&1 || { tail -5 $O/cfg1.txt; exit 1; }
timeout -k 10 400 python -u tools/config_bench.py C5,C3,C4 3 > $O/cfg2.txt 2>&1 || { tail -5 $O/cfg2.txt; exit 1; }
grep -h '^{' $O/cfg1.txt $O/cfg2.txt | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], d['ms_per_step'])"
bash tools/gpu/ab_env.sh v5ab 1 "-" "ZV_FFN_MIN_ROWS=0"
