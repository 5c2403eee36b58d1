#!/usr/bin/env python3
"""GEMM tile-variant microbenchmark on the engine's kernels (random bf16 operands).

usage: bench_gemm.py [variants] [modes] [shapes]
  variants: comma list (+100 = one tile per block instead of the persistent grid)
  modes:    comma list of 0 fp32 C, 1 bf16 C, 2 residual (fp32 C += .., bf16 copy),
            5 residual + bias (the residual linears' epilogue; variant 70 = counted), 6 + bypass,
            7 bias + SwooshL -> bf16 (a plain linear's; variant 72 = counted),
            3 SwooshL -> bf16, 4 no output (epilogue store ablation)
  shapes:   "MxNxK;MxNxK" (default: the decoder's full-length shapes)
"""
import ctypes
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402,F401

from zipvoice_amd import engine  # noqa: E402

MODES = {0: "f32", 1: "bf16", 2: "resid", 3: "swooshl", 4: "none", 5: "resid+bias", 6: "resid+bias+orig", 7: "bias+swooshl"}
lib = engine.load_library()
shapes = [(78016, 1536, 512), (78016, 512, 1536), (78016, 1152, 512), (78016, 512, 512),
          (78016, 1024, 512), (78016, 512, 48), (4096, 4096, 4096)]
variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else range(8))]
modes = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else (0, 1))]
if len(sys.argv) > 3:
    shapes = [tuple(int(x) for x in s.split("x")) for s in sys.argv[3].split(";")]
for (M, N, K) in shapes:
    for v in variants:
        for mode in modes:
            ms = ctypes.c_float()
            rc = lib.zv_bench_gemm(M, N, K, v, 10, mode, ctypes.byref(ms))
            if rc:
                print(M, N, K, v, "ERR", lib.zv_last_error().decode())
                continue
            tf = 2.0 * M * N * K / (ms.value * 1e-3) / 1e12
            out_b = {0: 4, 1: 2, 2: 10, 3: 2, 4: 0, 5: 10, 6: 14, 7: 2}[mode] * M * N
            gbs = (out_b + 2 * M * K) / (ms.value * 1e-3) / 1e9
            print(f"M={M} N={N} K={K} variant={v} out={MODES[mode]}: "
                  f"{ms.value*1e3:8.1f} us  {tf:7.1f} TFLOP/s  {gbs:7.0f} GB/s(min traffic)",
                  flush=True)
