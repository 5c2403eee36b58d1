#!/usr/bin/env python3
"""Library-GEMM yardstick (torch.matmul -> hipBLASLt, bf16) at the decoder's
linear shapes: what a vendor GEMM reaches on the same M x N x K, for comparison
with the engine's own kernel (tools/bench_gemm.py).  Not part of the product."""
import torch

shapes = [(78016, 1536, 512), (78016, 512, 1536), (78016, 1152, 512), (78016, 512, 512),
          (78016, 1024, 512), (78016, 272, 512), (78016, 512, 384), (78016, 48, 512),
          (78016, 512, 48), (4096, 4096, 4096)]
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"torch bf16 M={M} N={N} K={K}: {ms*1e3:8.1f} us {2*M*N*K/ms/1e9:7.1f} TFLOP/s", flush=True)
