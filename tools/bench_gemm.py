#!/usr/bin/env python3
"""GEMM tile-variant microbenchmark on the engine's kernels (random bf16 operands)."""
import ctypes
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402,F401

from zipvoice_amd import engine  # noqa: E402

lib = engine.load_library()
shapes = [(78016, 1536, 512), (78016, 512, 1536), (78016, 1152, 512), (78016, 512, 512),
          (78016, 1024, 512), (4096, 4096, 4096)]
variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else range(8))]
for (M, N, K) in shapes:
    for v in variants:
        for ob in (0, 1):
            ms = ctypes.c_float()
            rc = lib.zv_bench_gemm(M, N, K, v, 10, ob, ctypes.byref(ms))
            if rc:
                print(M, N, K, v, "ERR", lib.zv_last_error().decode())
                continue
            tf = 2.0 * M * N * K / (ms.value * 1e-3) / 1e12
            print(f"M={M} N={N} K={K} variant={v} out={'bf16' if ob else 'f32'}: "
                  f"{ms.value*1e3:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)
