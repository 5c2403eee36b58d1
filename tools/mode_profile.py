#!/usr/bin/env python3
"""Per-kernel-family time of one C2 bench step in each precision mode (engine HIP-event
profiler, one decoder stream), plus the timed step: where a mode's extra time goes.

usage: python tools/mode_profile.py [bf16,fp16,fp8] [--steps 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("modes", nargs="?", default="bf16,fp16")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    conf = bench.CONFIGS["C2"]
    voc = bench.build_vocoder(dev)
    out = {}
    for mode in args.modes.split(","):
        m = bench.build(conf["variant"], mode, dev)
        job = bench.Job(conf, m, voc, conf["per_gpu"], dev)
        ms = bench.timed(job, args.steps, 2, 1) * 1e3
        r = bench.roofline(job)
        out[mode] = {"ms_per_step": round(ms, 2), "per_kernel_ms": r["per_kernel_ms_per_step"]}
        print(json.dumps({mode: out[mode]}), flush=True)
        del job, m
        torch.cuda.empty_cache()
    keys = sorted({k for v in out.values() for k in v["per_kernel_ms"]},
                  key=lambda k: -max(v["per_kernel_ms"].get(k, 0) for v in out.values()))
    print(f"{'kernel':32s}" + "".join(f"{m:>10s}" for m in out))
    for k in keys:
        print(f"{k:32s}" + "".join(f"{v['per_kernel_ms'].get(k, 0):10.2f}" for v in out.values()))
    print(f"{'(sum)':32s}" + "".join(f"{sum(v['per_kernel_ms'].values()):10.2f}" for v in out.values()))
    print(f"{'(timed step)':32s}" + "".join(f"{v['ms_per_step']:10.2f}" for v in out.values()))


if __name__ == "__main__":
    main()
