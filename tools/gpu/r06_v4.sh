# round 6: fp16 second-generation attention with step 0 peeled: kernel + parity tests, mode profile
mkdir -p gpurun_out/r06_v4
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_attn2.py -s > gpurun_out/r06_v4/attn2.log 2>&1; echo "attn2 rc=$?" >> gpurun_out/r06_v4/attn2.log
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k fp16 -s > gpurun_out/r06_v4/parity.log 2>&1; echo "parity rc=$?" >> gpurun_out/r06_v4/parity.log
timeout -k 10 400 python -u tools/mode_profile.py bf16,fp16 --steps 3 > gpurun_out/r06_v4/mode.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/fallback_probe.py fp16 1219 > gpurun_out/r06_v4/fb.txt 2>&1
