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
ap.add_argument("--report", action="store_true", help="per-shape event-profiler table")
ap.add_argument("--alg-json", default=None,
                help="event-profile the --iters loop itself and write {tag: launches, bytes, flops}: the "
                     "algorithmic bytes of the same launch set a PMC pass of this command counts")
ap.add_argument("--text", action="store_true",
                help="also one text-encoder pass of the batch (its residual linears include the bypass ROLE 2)")
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
if a.alg_json:
    from zipvoice_amd import engine
    engine.profile(True)
for _ in range(a.iters):
    v = m.engine.velocity(0.3, 1.0, x, tc, sc, pm)
    if a.text:                      # the C2 shape's text: 40 prompt + 134 text tokens + 1 pad
        tok = torch.from_numpy(rng.integers(1, 360, (a.B, 175))).to(dev)
        m.engine.text_encode(tok, torch.zeros(a.B, 175, dtype=torch.bool, device=dev))
torch.cuda.synchronize()
print("ok", float(v.abs().mean()))
if a.alg_json:
    import json
    rep = engine.profile_report()
    engine.profile(False)
    json.dump({k: {f: r[f] for f in ("launches", "bytes", "flops")} for k, r in rep.items()},
              open(a.alg_json, "w"), indent=1)
if a.report:
    from zipvoice_amd import engine
    engine.profile(True, detail=True)
    m.engine.velocity(0.3, 1.0, x, tc, sc, pm)
    torch.cuda.synchronize()
    rep = engine.profile_report()
    engine.profile(False)
    tot = sum(r["ms"] for r in rep.values())
    print(f"# one guided forward, event-profiled launches: {tot:.3f} ms")
    print(f"{'launch':64s} {'n':>4s} {'ms':>8s} {'avg_us':>8s} {'TF/s':>7s} {'pct':>5s}")
    for k, r in sorted(rep.items(), key=lambda kv: -kv[1]["ms"]):
        tf = r["flops"] / (r["ms"] * 1e-3) / 1e12 if r["flops"] else 0.0
        print(f"{k:64s} {r['launches']:4d} {r['ms']:8.3f} {1e3 * r['ms'] / r['launches']:8.1f} "
              f"{tf:7.1f} {100 * r['ms'] / tot:5.1f}")
