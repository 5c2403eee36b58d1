# round 6: fp16 diagonal step walked back past a padded tail -- exact-path counts on ragged batches,
# the attention kernel tests and the fp16 / ragged parity tests
O=gpurun_out/r06_ragged; mkdir -p $O
ZV_PROBE_RAGGED=1 timeout -k 10 200 python -u tools/fallback_probe.py bf16,fp16 1219 3376 > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
grep exact $O/probe.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_attn2.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
