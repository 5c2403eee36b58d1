# round 6 final tree: the whole GPU suite (as the driver runs it) + smoke
mkdir -p gpurun_out/r06_tests
timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06_tests/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r06_tests/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_tests/smoke.log 2>&1; echo "smoke rc=$?" >> gpurun_out/r06_tests/smoke.log
