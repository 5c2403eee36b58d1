#!/usr/bin/env python3
"""One guided decoder evaluation at the benchmark shape (C2: B=32 -> 64 CFG rows,
T=1219) — a short, representative command for rocprofv3 kernel-trace and PMC
passes (the full benchmark step is 16 of these)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from zipvoice_amd.config import default_config  # noqa: E402
from zipvoice_amd.models import build_model  # noqa: E402
from zipvoice_amd.weights import synthetic_state_dict  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="bf16")
ap.add_argument("--iters", type=int, default=2)
ap.add_argument("--B", type=int, default=32)
ap.add_argument("--T", type=int, default=1219)
a = ap.parse_args()
cfg = default_config("zipvoice")
m = build_model(cfg, precision=a.precision)
m.load_state_dict(synthetic_state_dict(cfg, 0))
m = m.to("cuda:0")
rng = np.random.default_rng(0)
dev = torch.device("cuda:0")
x = torch.from_numpy(rng.standard_normal((a.B, a.T, 100), dtype=np.float32)).to(dev)
tc = torch.from_numpy(rng.standard_normal((a.B, a.T, 100), dtype=np.float32)).to(dev)
sc = torch.from_numpy(rng.standard_normal((a.B, a.T, 100), dtype=np.float32)).to(dev)
pm = torch.zeros(a.B, a.T, dtype=torch.bool, device=dev)
for _ in range(a.iters):
    v = m.engine.velocity(0.3, 1.0, x, tc, sc, pm)
torch.cuda.synchronize()
print("ok", float(v.abs().mean()))
