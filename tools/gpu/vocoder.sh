set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoder.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_vocoder.log 2>&1
