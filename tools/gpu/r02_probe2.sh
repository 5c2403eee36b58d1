mkdir -p gpurun_out
timeout -k 5 60 ./tools/probe/mx8_probe2 > gpurun_out/mx8_probe2.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
timeout -k 10 400 python -u tools/counted_bisect.py fp32 > gpurun_out/cb_fp32.txt 2>&1 || { echo "bisect rc=$?"; exit 1; }
