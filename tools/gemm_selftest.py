#!/usr/bin/env python3
"""Bitwise self-check of GEMM tile variants against the 128x128 kernel (random
bf16 operands; same MFMA order per output, so the fp32 results must agree).

usage: gemm_selftest.py [variants] [shapes]"""
import ctypes
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402,F401

from zipvoice_amd import engine  # noqa: E402

lib = engine.load_library()
variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else (20, 21, 22, 23))]
shapes = [(1000, 300, 200), (78016, 1536, 512), (4096, 512, 1920), (777, 1024, 48), (256, 256, 64)]
if len(sys.argv) > 2:
    shapes = [tuple(int(x) for x in s.split("x")) for s in sys.argv[2].split(";")]
bad = 0
for (M, N, K) in shapes:
    for v in variants:
        for mode in ((0, 1) if v == 40 else (0, 1, 2)):
            d, r = ctypes.c_float(), ctypes.c_float()
            rc = lib.zv_gemm_selftest(M, N, K, v, mode, ctypes.byref(d), ctypes.byref(r))
            if rc:
                print(M, N, K, v, mode, "ERR", lib.zv_last_error().decode(), flush=True)
                bad += 1
                continue
            ok = d.value <= 1e-5 * max(1.0, r.value)
            bad += not ok
            print(f"M={M} N={N} K={K} variant={v} mode={mode}: maxdiff {d.value:.3e} "
                  f"(max |ref| {r.value:.3e}) {'ok' if ok else 'MISMATCH'}", flush=True)
sys.exit(1 if bad else 0)
