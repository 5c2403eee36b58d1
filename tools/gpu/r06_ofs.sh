# round 6: fp16 offsets from step 0 + the diagonal step -- exact-path counts, attention tests, fp16 parity
# tests, the per-tag mode profile (bf16 vs fp16) and the bench's modes
O=gpurun_out/r06_ofs; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step probe
timeout -k 10 200 python -u tools/fallback_probe.py bf16,fp16 1219 3376 > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
cat $O/probe.txt | grep exact
step tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn2.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step modes
timeout -k 10 400 python -u tools/mode_profile.py bf16,fp16 > $O/modes.txt 2>&1 || { tail -5 $O/modes.txt; exit 1; }
grep -E "attn_|sum|timed" $O/modes.txt
step done
