cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r02_gputest1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r02_gputest1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench1.json 2> gpurun_out/r02_bench1.err
  echo "bench rc=$?" >> gpurun_out/r02_gputest1.log
fi
